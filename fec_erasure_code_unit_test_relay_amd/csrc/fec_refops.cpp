// fec_refops.cpp -- the reference's free GF(2^8) / block-code functions (include/fec_amd_refops.h)
// over the library's host field (fec_host.h: exp/log tables of poly 0x11d, generator 2), so that the
// reference's remaining sources link without basicOperations.cpp, codingOperations.cpp or ISA-L
// (tests/test_dropin_compile.py links them with -Wl,--no-undefined against this library).
//
// Each function cites the reference lines it follows.  The ISA-L routines the reference calls
// (gf_mul, gf_inv, gf_invert_matrix, gf_gen_cauchy1_matrix, gf_gen_rs_matrix; ISA-L 2.23.0
// erasure_code/ec_base.c) are restated from their published definitions.
#include "fec_amd_refops.h"

#include <algorithm>
#include <cstring>
#include <random>
#include <utility>
#include <vector>

#include "fec_host.h"

namespace {

const fec::Field& F() { return fec::field(); }

// A small scratch array on the stack, on the heap past `Cap` bytes (the reference uses VLAs).
template <int Cap>
struct Scratch {
    unsigned char local[Cap];
    std::vector<unsigned char> heap;
    unsigned char* p;
    explicit Scratch(size_t bytes) {
        if (bytes <= Cap) {
            p = local;
        } else {
            heap.resize(bytes);
            p = heap.data();
        }
    }
};

void print_rows(const int* v, int row, int column) {  // basicOperations.cpp:142-200's layout
    std::cout << "[";
    for (int i = 0; i < row; i++) {
        if (i > 0) std::cout << " ";
        for (int j = 0; j < column; j++) {
            const int d = v[i * column + j];
            const int digits = d >= 100 ? 3 : (d >= 10 ? 2 : 1);
            for (int s = 0; s < 3 - digits; s++) std::cout << " ";
            std::cout << d << " ";
        }
        if (i < row - 1) std::cout << std::endl;
        else std::cout << "]" << std::endl << std::endl;
    }
}

}  // namespace

// ---- basicOperations.cpp --------------------------------------------------------------------

unsigned char gf256_add(unsigned char a, unsigned char b) { return a ^ b; }  // :14-16

unsigned char gf256_mul(unsigned char a, unsigned char b) { return F().mul(a, b); }  // :18-20 (ISA-L gf_mul)

unsigned char gf256_inv(unsigned char a) { return F().inv(a); }  // :22-24 (ISA-L gf_inv)

void gf256_transpose(unsigned char* in, unsigned char* out, int k, int n) {  // :26-33
    for (int r = 0; r < k; r++)
        for (int c = 0; c < n; c++) out[c * k + r] = in[r * n + c];
}

// :35-41 over ISA-L's gf_invert_matrix: Gauss-Jordan on a copy of `in` with row swaps; -1 if singular.
int gf256_invert_matrix(unsigned char* in, unsigned char* out, const int n) {
    if (n <= 0) return 0;
    Scratch<1024> work(static_cast<size_t>(n) * n);
    unsigned char* a = work.p;
    std::memcpy(a, in, static_cast<size_t>(n) * n);
    std::memset(out, 0, static_cast<size_t>(n) * n);
    for (int i = 0; i < n; i++) out[i * n + i] = 1;
    for (int c = 0; c < n; c++) {
        if (a[c * n + c] == 0) {  // a row below with a non-zero in column c, swapped up
            int r = c + 1;
            while (r < n && a[r * n + c] == 0) r++;
            if (r == n) return -1;
            for (int x = 0; x < n; x++) {
                std::swap(a[c * n + x], a[r * n + x]);
                std::swap(out[c * n + x], out[r * n + x]);
            }
        }
        const unsigned char s = F().inv(a[c * n + c]);
        for (int x = 0; x < n; x++) {
            a[c * n + x] = F().mul(a[c * n + x], s);
            out[c * n + x] = F().mul(out[c * n + x], s);
        }
        for (int r = 0; r < n; r++) {
            if (r == c) continue;
            const unsigned char f = a[r * n + c];
            for (int x = 0; x < n; x++) {
                out[r * n + x] ^= F().mul(f, out[c * n + x]);
                a[r * n + x] ^= F().mul(f, a[c * n + x]);
            }
        }
    }
    return 0;
}

// :43-122: column reduction of the m x n matrix `in` (row-major) into `out`, with the n x n
// action matrix such that in * action = out.  Column i pivots on row i + offset; a zero pivot is
// swapped with the first later column that is non-zero in that row, or, if there is none, the
// pivot row moves down one (offset) and column i is tried again.
void gf256_rref_matrix(unsigned char* in, unsigned char* out, unsigned char* action, int m, int n) {
    const fec::Field& f = F();
    std::memset(action, 0, static_cast<size_t>(n) * n);
    for (int i = 0; i < n; i++) action[i * n + i] = 1;
    std::memcpy(out, in, static_cast<size_t>(m) * n);
    auto swap_cols = [&](unsigned char* a, int rows, int c0, int c1) {
        for (int r = 0; r < rows; r++) std::swap(a[r * n + c0], a[r * n + c1]);
    };
    int offset = 0;
    for (int i = 0; i < n; i++) {
        const int row = i + offset;
        if (row >= m) break;
        if (out[row * n + i] == 0) {
            int j = i + 1;
            while (j < n && out[row * n + j] == 0) j++;
            if (j == n) {  // no pivot in this row: the next row, same column
                offset++;
                i--;
                continue;
            }
            swap_cols(out, m, i, j);
            swap_cols(action, n, i, j);
        }
        const unsigned char s = f.inv(out[row * n + i]);
        for (int r = 0; r < m; r++) out[r * n + i] = f.mul(out[r * n + i], s);
        for (int r = 0; r < n; r++) action[r * n + i] = f.mul(action[r * n + i], s);
        for (int j = 0; j < n; j++) {  // clear the pivot row in every other column (zeros skipped)
            if (j == i) continue;
            const unsigned char e = out[row * n + j];
            if (e == 0) continue;
            for (int r = 0; r < m; r++) out[r * n + j] ^= f.mul(e, out[r * n + i]);
            for (int r = 0; r < n; r++) action[r * n + j] ^= f.mul(e, action[r * n + i]);
        }
    }
}

// :124-140
void gf256_matrix_mul(unsigned char* inMatrix1, unsigned char* inMatrix2, unsigned char* outMatrix, int m1, int m2,
                      int m3) {
    const fec::Field& f = F();
    for (int r = 0; r < m1; r++)
        for (int c = 0; c < m3; c++) {
            unsigned char acc = 0;
            for (int x = 0; x < m2; x++) acc ^= f.mul(inMatrix1[r * m2 + x], inMatrix2[x * m3 + c]);
            outMatrix[r * m3 + c] = acc;
        }
}

void fec_print_matrix_u8(const unsigned char* matrix, int row, int column) {  // :142-172
    std::vector<int> v(static_cast<size_t>(row > 0 && column > 0 ? row * column : 0));
    for (size_t i = 0; i < v.size(); i++) v[i] = matrix[i];
    print_rows(v.data(), row, column);
}

void printMatrix(bool* matrix, int row, int column) {  // :175-202
    std::vector<int> v(static_cast<size_t>(row > 0 && column > 0 ? row * column : 0));
    for (size_t i = 0; i < v.size(); i++) v[i] = matrix[i] ? 1 : 0;
    print_rows(v.data(), row, column);
}

// ---- codingOperations.cpp -------------------------------------------------------------------

// :27-46: the payload bytes, or `payload` zero bytes for a lost packet
void save_to_file(unsigned char* data, int payload, ofstream* file) {
    if (payload > 0 && data != nullptr) {
        file->write(reinterpret_cast<const char*>(data), payload);
    } else if (payload > 0) {
        const std::vector<char> zero(static_cast<size_t>(payload), 0);
        file->write(zero.data(), payload);
    }
}

// :48-95: ISA-L's gf_gen_cauchy1_matrix (or gf_gen_rs_matrix for (10,8,4) and (11,5,4)) as an
// n x k matrix, transposed to k x n, then the burst-structure zeros of the parity columns.
void gen_G_cauchy(unsigned char* G, int T, int B, int N, int k, int n) {
    const fec::Field& f = F();
    Scratch<1024> gt(static_cast<size_t>(n) * k);
    unsigned char* a = gt.p;  // n x k
    std::memset(a, 0, static_cast<size_t>(n) * k);
    for (int i = 0; i < k && i < n; i++) a[i * k + i] = 1;
    if ((T == 10 && B == 8 && N == 4) || (T == 11 && B == 5 && N == 4)) {
        unsigned char gen = 1;
        for (int i = k; i < n; i++) {
            unsigned char p = 1;
            for (int j = 0; j < k; j++) {
                a[i * k + j] = p;
                p = f.mul(p, gen);
            }
            gen = f.mul(gen, 2);
        }
    } else {
        for (int i = k; i < n; i++)
            for (int j = 0; j < k; j++) a[i * k + j] = f.inv(static_cast<unsigned char>(i ^ j));
    }
    gf256_transpose(a, G, n, k);
    if (B == 0) return;
    const int d = B - N;
    if (2 * k >= n) {  // high rate
        for (int i = 0; i < d; i++) {
            for (int j = k + N + i; j < n; j++) G[i * n + j] = 0;
            for (int j = 0; j < i; j++) G[i * n + k + j] = 0;
        }
        for (int i = d; i < B; i++)
            for (int j = 0; j < d; j++) G[i * n + k + j] = 0;
    } else {  // low rate
        for (int i = 0; i < d; i++) {
            for (int j = k + N + i; j < n; j++) G[i * n + j] = 0;
            for (int j = 0; j < i; j++) G[i * n + B + j] = 0;
        }
        for (int i = d; i < k; i++)
            for (int j = 0; j < d; j++) G[i * n + B + j] = 0;
    }
}

int init_at_sender(int T, int B, int N, unsigned char* G, int k, int n) {  // :113-116
    gen_G_cauchy(G, T, B, N, k, n);
    return 1;
}

void generateData(unsigned char* data, int payload) {  // :118-129 (random bytes, fresh seed)
    std::random_device rd;
    std::mt19937 gen(rd());
    std::uniform_int_distribution<int> dist(0, 255);
    for (int i = 0; i < payload; i++) data[i] = static_cast<unsigned char>(dist(gen));
}

// :131-147: symbol t of the codeword, and at t = k-1 every parity symbol too
void encodeBlock(unsigned char* data, unsigned char* generator, unsigned char* codeword, int k, int n, int t) {
    const fec::Field& f = F();
    unsigned char acc = 0;
    for (int i = 0; i < k; i++) acc ^= f.mul(data[i], generator[i * n + t]);
    codeword[t] = acc;
    if (t != k - 1) return;
    for (int j = k; j < n; j++) {
        unsigned char p = 0;
        for (int i = 0; i < k; i++) p ^= f.mul(data[i], generator[i * n + j]);
        codeword[j] = p;
    }
}

// :149-232: the window w = min(t+T+1, n) of columns, erased columns zeroed, column-reduced; the
// decoded data are the codeword times the action matrix; an erased data symbol i is recovered when
// row i's first unit entry among columns i..k-1 heads a column that is zero below row i.
void decodeBlock(unsigned char* data, unsigned char* generator, unsigned char* codeword, bool* erasure, int k, int n,
                 int T, int t) {
    if (t < k && !erasure[t]) data[t] = codeword[t];
    const int w = std::min(t + T + 1, n);
    if (w <= 0) return;
    Scratch<512> dm(static_cast<size_t>(k) * w), rr(static_cast<size_t>(k) * w), act(static_cast<size_t>(w) * w);
    Scratch<64> dd(static_cast<size_t>(w));
    int erased = 0;
    for (int c = 0; c < w; c++) {
        const bool e = erasure[c];
        erased += e ? 1 : 0;
        for (int r = 0; r < k; r++) dm.p[r * w + c] = e ? 0 : generator[r * n + c];
    }
    if (erased == w) return;
    gf256_rref_matrix(dm.p, rr.p, act.p, k, w);
    gf256_matrix_mul(codeword, act.p, dd.p, 1, w, w);
    for (int i = 0; i < k; i++) {
        if (!erasure[i]) continue;
        int j = i;
        while (j < k && rr.p[i * w + j] != 1) j++;
        if (j == k) continue;
        int below = i + 1;
        while (below < k && rr.p[below * w + j] == 0) below++;
        if (below < k) continue;
        erasure[i] = false;
        data[i] = dd.p[j];
        codeword[i] = data[i];
    }
}

// :234-252: the fraction of packets (beyond the first T) whose bytes differ from the source
float calculateLoss(unsigned char* data, unsigned char* recovered_data, int max_payload, int* payload,
                    int stream_duration, int T) {
    float lost = 0;
    for (int t = 0; t < stream_duration; t++)
        for (int i = 0; i < payload[t]; i++)
            if (data[t * max_payload + i] != recovered_data[t * max_payload + i]) {
                lost++;
                break;
            }
    return lost / static_cast<float>(stream_duration - T);
}

// :254-297: the fraction of bytes that differ between two equally long files (1 if their sizes differ)
float calculateLossMessage(string file_original, string file_recovered) {
    std::ifstream a(file_original, std::ios::in | std::ios::binary), b(file_recovered, std::ios::in | std::ios::binary);
    a.seekg(0, std::ios::end);
    const long na = static_cast<long>(a.tellg());
    a.seekg(0, std::ios::beg);
    b.seekg(0, std::ios::end);
    const long nb = static_cast<long>(b.tellg());
    b.seekg(0, std::ios::beg);
    if (na != nb) {
        std::cout << "THe two files have different sizes!" << std::endl;
        return 1;
    }
    std::vector<char> x(static_cast<size_t>(na > 0 ? na : 0)), y(x.size());
    a.read(x.data(), na);
    b.read(y.data(), nb);
    float loss = 0;
    for (long i = 0; i < na; i++)
        if (x[static_cast<size_t>(i)] != y[static_cast<size_t>(i)]) loss++;
    return loss / static_cast<float>(na);
}
