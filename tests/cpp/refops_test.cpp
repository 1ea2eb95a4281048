// refops_test.cpp -- the reference-signature free functions of libfec_amd.so (include/fec_amd_refops.h,
// replacing basicOperations.h / codingOperations.h under the header swap) against the oracle's
// restatements (oracle/fec_oracle.c): field, generator matrices, column reduction, block encode and
// decode on random inputs and erasure patterns, matrix inversion and product.  Host-only: no GPU
// call is made.  Prints "REFOPS OK" when every comparison holds.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "fec_amd_refops.h"

extern "C" {
#include "../../oracle/fec_oracle.h"
}

static int fails = 0;
#define CHECK(c, ...)                          \
    do {                                       \
        if (!(c)) {                            \
            if (fails < 20) {                  \
                std::printf("FAIL: " __VA_ARGS__); \
                std::printf("\n");             \
            }                                  \
            ++fails;                           \
        }                                      \
    } while (0)

int main() {
    std::mt19937 rng(12345);
    // field
    for (int a = 0; a < 256; ++a) {
        CHECK(gf256_inv(uint8_t(a)) == or_gf_inv(uint8_t(a)), "inv %d", a);
        for (int b = 0; b < 256; ++b) CHECK(gf256_mul(uint8_t(a), uint8_t(b)) == or_gf_mul(uint8_t(a), uint8_t(b)), "mul %d %d", a, b);
    }
    // generators: every (T, B, N) the codec accepts with T <= 11, plus the RS special cases
    int ngen = 0;
    for (int T = 0; T <= 11; ++T)
        for (int N = 0; N <= T; ++N)
            for (int B = N; B <= T; ++B) {
                const int k = T - N + 1, n = k + B;
                if (n > 32) continue;
                std::vector<uint8_t> g1(size_t(k) * n), g2(size_t(k) * n);
                init_at_sender(T, B, N, g1.data(), k, n);
                or_gen_G(g2.data(), T, B, N, k, n);
                CHECK(g1 == g2, "gen_G (%d,%d,%d)", T, B, N);
                ++ngen;
            }
    // column reduction of random matrices (with zero columns and rows, as decodeBlock makes them)
    for (int it = 0; it < 4000; ++it) {
        const int m = 1 + int(rng() % 12), n = 1 + int(rng() % 22);
        std::vector<uint8_t> in(size_t(m) * n), o1(in.size()), o2(in.size()), a1(size_t(n) * n), a2(a1.size());
        const int zc = int(rng() % 4);
        for (auto& x : in) x = uint8_t(rng() % 4 == 0 ? 0 : rng());
        for (int z = 0; z < zc; ++z) {
            const int c = int(rng() % n);
            for (int r = 0; r < m; ++r) in[size_t(r) * n + c] = 0;
        }
        gf256_rref_matrix(in.data(), o1.data(), a1.data(), m, n);
        or_rref_matrix(in.data(), o2.data(), a2.data(), m, n);
        CHECK(o1 == o2 && a1 == a2, "rref %dx%d it %d", m, n, it);
        // in * action = out (the reference's contract)
        std::vector<uint8_t> prod(in.size());
        gf256_matrix_mul(in.data(), a1.data(), prod.data(), m, n, n);
        CHECK(prod == o1, "in*action != out %dx%d", m, n);
    }
    // block encode / decode as the reference's per-diagonal decoder calls them
    const int cfg[][3] = {{10, 3, 3}, {10, 5, 2}, {10, 1, 1}, {10, 10, 10}, {10, 8, 4}, {6, 2, 2}, {8, 4, 1}};
    int ndec = 0, nrec = 0;
    for (const auto& c : cfg) {
        const int T = c[0], B = c[1], N = c[2], k = T - N + 1, n = k + B;
        std::vector<uint8_t> G(size_t(k) * n);
        init_at_sender(T, B, N, G.data(), k, n);
        for (int it = 0; it < 3000; ++it) {
            std::vector<uint8_t> d(k), cw(n);
            for (auto& x : d) x = uint8_t(rng());
            for (int t = 0; t < k; ++t) encodeBlock(d.data(), G.data(), cw.data(), k, n, t);
            std::vector<uint8_t> cw2(n);
            for (int t = 0; t < k; ++t) or_encode_block(d.data(), G.data(), cw2.data(), k, n, t);
            CHECK(cw == cw2, "encodeBlock (%d,%d,%d)", T, B, N);
            // an erasure pattern, garbage in the erased symbols
            std::vector<uint8_t> e8(n);
            bool eb[64];
            const int pr = 1 + int(rng() % 6);
            for (int q = 0; q < n; ++q) {
                e8[q] = (rng() % 10) < unsigned(pr) ? 1 : 0;
                eb[q] = e8[q] != 0;
            }
            std::vector<uint8_t> c1 = cw, c2 = cw, d1(k, 0), d2(k, 0);
            for (int q = 0; q < n; ++q)
                if (e8[q]) c1[q] = c2[q] = uint8_t(rng());
            const int Td = int(rng() % (n + 1)), td = int(rng() % n);
            decodeBlock(d1.data(), G.data(), c1.data(), eb, k, n, Td, td);
            or_decode_block(d2.data(), G.data(), c2.data(), e8.data(), k, n, Td, td);
            bool same = c1 == c2 && d1 == d2;
            for (int q = 0; q < n; ++q) same = same && (eb[q] == (e8[q] != 0));
            CHECK(same, "decodeBlock (%d,%d,%d) T=%d t=%d", T, B, N, Td, td);
            for (int i = 0; i < k; ++i)
                if (e8[i] == 0 && eb[i] == false && d1[i] != 0) ++nrec;
            ++ndec;
        }
    }
    // inversion: A * A^-1 = I for random invertible A; a singular one returns -1
    int ninv = 0;
    for (int it = 0; it < 500; ++it) {
        const int n = 1 + int(rng() % 12);
        std::vector<uint8_t> A(size_t(n) * n), Ai(A.size()), P(A.size());
        for (auto& x : A) x = uint8_t(rng());
        const std::vector<uint8_t> keep = A;
        if (gf256_invert_matrix(A.data(), Ai.data(), n) != 0) continue;
        CHECK(A == keep, "invert_matrix changed its input");
        gf256_matrix_mul(A.data(), Ai.data(), P.data(), n, n, n);
        for (int r = 0; r < n; ++r)
            for (int c = 0; c < n; ++c) CHECK(P[size_t(r) * n + c] == (r == c ? 1 : 0), "A*inv(A) n=%d", n);
        ++ninv;
    }
    {
        uint8_t S[4] = {1, 2, 2, 4}, Si[4];  // rows 1, 2 dependent: 2*(1,2) = (2,4)
        CHECK(gf256_invert_matrix(S, Si, 2) == -1, "singular matrix not reported");
    }
    uint8_t t[6] = {1, 2, 3, 4, 5, 6}, tt[6];
    gf256_transpose(t, tt, 2, 3);
    CHECK(tt[0] == 1 && tt[1] == 4 && tt[2] == 2 && tt[3] == 5 && tt[4] == 3 && tt[5] == 6, "transpose");
    CHECK(gf256_add(0x53, 0xCA) == (0x53 ^ 0xCA), "add");
    std::printf("generators %d, decodeBlock calls %d, inversions %d\n", ngen, ndec, ninv);
    if (fails) {
        std::printf("%d failures\n", fails);
        return 1;
    }
    std::printf("REFOPS OK\n");
    return 0;
}
