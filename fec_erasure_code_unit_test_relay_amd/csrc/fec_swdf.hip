// fec_swdf.hip -- the relay's symbol-wise decode-and-forward (SWDF, RELAYING_TYPE 2) and the
// destination's symbol-wise decode, batched over many packets of one relay stream.
//
// Reference: Decoder_Symbol_Wise (src/Decoder_Symbol_Wise.cpp) driven by Variable_Rate_FEC_Decoder
// (relay :950-1601, destination :1603-1879) and the local simulation's relay loop with
// FLAG_FOR_CONSTANT_TRANS = 1 (application_local_simulation.cpp:532-587: one relay frame per seq).
//
// Per seq t the relay keeps a window of the last n1 = T1+1 received source codewords
// (push_current_codeword / rotate_pointers_and_insert_zero_word, :119-176; an erased packet is an
// all-zero slot flagged erased; slots before the first packet are zero and NOT erased) and, per
// code block j < S, takes the diagonal  d[m] = symbol (j, m) of packet t-n1+1+m  (:564-568),
// decodes it with decodeBlock(T = n1-1, t = 0) when 0 < erasures(window) < n1-k+1 (:570-573), and
// forwards the k data symbols reversed, Y_t[j][i] = d[k-1-i] (:577-578).  Its frame for seq t is
// the second hop's diagonal code over Y (:593-618):
//   frame = [size BE16][0, 0][S blocks of n2: Y_t[j][p] (p < k), parity p >= k =
//            XOR_{i<k} G2[i][p] * Y_{t-(p-i)}[j][i]][n2-2 zero bytes],  size = (S+1)*n2
// (the 2 zero bytes are codeword_new_vector's offset-2 start, the trailing ones the extra block
// of codeword_r_d_size, Variable_Rate_FEC_Decoder.cpp:998, 1482-1491).
// The destination keeps the same window over the relay frames and outputs, per seq t2, the
// data_with_header of source packet t2 - (n1 + n2 - k - 1) (symbol_wise_decode_1 + extract_data,
// :621-665): out[j*k + i] = d2[k-1-i] with d2 the decoded hop-2 diagonal.
//
// Every decision depends only on the erasure flags: decodeBlock's outcome for a full window is
// the codec's decode rule for (w = n, erasure mask) (fec_host.cpp DecodeRules).  So the byte work
// is two data-parallel kernels: a diagonal decode (one thread per (packet, block)) used by both
// the relay and the destination, and the relay's re-encode.  Undefined behaviour of the reference
// defined away ("Relay"): n flags (not n-1 plus garbage) reach decodeBlock, slots hold
// zero-padded packets, k2 == k.  The block count is the reference's ceil(max_payload/k)+1 on ints
// (:553, :632; at most S): the blocks past it are not relayed and stay zero, as in the reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <utility>
#include <vector>
#include <new>

#include "fec_amd.h"
#include "fec_device.h"
#include "fec_host.h"
#include "fec_kernels.h"
#include "fec_status.h"

namespace fec {

constexpr int kSwThreads = 256;

struct SwDecodeArgs {
    const uint8_t* in;      // rows of in_stride bytes; symbol (row, j, m) at in_off + j*n + m
    int64_t in_stride;
    int in_off;
    const uint8_t* er;      // per row: 1 = erased
    int64_t P;
    int k, n, S, blocks;
    const uint8_t* rules;   // window-n rule table (raw coefficients)
    int ES;
    const uint8_t* gf;      // exp[512], log[256]
    uint8_t* out;           // rows of out_stride bytes: out[j*k + i]
    int64_t out_stride;
    uint8_t* flag;          // per row (may be null): erasures >= n-k+1
};

struct SwEncodeArgs {
    const uint8_t* y;       // rows of S*k bytes
    int64_t P;
    int k, n2, S, blocks;
    const uint8_t* G2;      // k x n2
    const uint8_t* gf;
    uint8_t* frames;        // rows of F = 2 + (S+1)*n2 bytes
    int F;
};

__global__ __launch_bounds__(kSwThreads) void fec_swdf_decode_kernel(SwDecodeArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    for (int i = threadIdx.x; i < 512; i += kSwThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kSwThreads) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int k = a.k, n = a.n, S = a.S;
    const int64_t total = a.P * S;
    for (int64_t id = static_cast<int64_t>(blockIdx.x) * kSwThreads + threadIdx.x; id < total;
         id += static_cast<int64_t>(gridDim.x) * kSwThreads) {
        const int64_t t = id / S;
        const int j = static_cast<int>(id - t * S);
        uint8_t* o = a.out + t * a.out_stride + j * k;
        if (j >= a.blocks) {  // not relayed / decoded (:553, :632)
            for (int i = 0; i < k; ++i) o[i] = 0;
            continue;
        }
        uint32_t mask = 0;
        uint8_t d[32];
        for (int m = 0; m < n; ++m) {
            const int64_t r = t - n + 1 + m;
            const bool erased = r >= 0 && a.er[r] != 0;
            mask |= (erased ? 1u : 0u) << m;
            d[m] = (r >= 0 && !erased) ? a.in[r * a.in_stride + a.in_off + j * n + m] : 0;
        }
        const int cnt = __popc(mask);
        if (cnt > 0 && cnt < n - k + 1) {  // decodeBlock(T = n-1, t = 0) on the diagonal
            const uint8_t* e = a.rules + static_cast<int64_t>(mask) * a.ES;
            uint8_t rec[32];
            uint32_t done = 0;
            for (int i = 0; i < k; ++i) {
                if (!((mask >> i) & 1u) || e[i] == 0xFF) continue;
                const uint8_t* col = e + k + i * n;
                uint8_t acc = 0;
                for (int c = 0; c < n; ++c) {
                    const uint8_t cf = col[c];
                    if (cf && d[c]) acc ^= gexp[glog[cf] + glog[d[c]]];
                }
                rec[i] = acc;
                done |= 1u << i;
            }
            for (int i = 0; i < k; ++i)
                if ((done >> i) & 1u) d[i] = rec[i];
        }
        for (int i = 0; i < k; ++i) o[i] = d[k - 1 - i];
        if (a.flag && j == 0) a.flag[t] = cnt >= n - k + 1 ? 1 : 0;
    }
}

__global__ __launch_bounds__(kSwThreads) void fec_swdf_encode_kernel(SwEncodeArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ int16_t lg[32 * 32];  // log of G2[i][p], -1 = zero
    for (int i = threadIdx.x; i < 512; i += kSwThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kSwThreads) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int k = a.k, n2 = a.n2, S = a.S, Sk = a.S * a.k;
    for (int i = threadIdx.x; i < k * n2; i += kSwThreads) lg[i] = a.G2[i] ? glog[a.G2[i]] : -1;
    __syncthreads();
    const int64_t total = a.P * S;
    for (int64_t id = static_cast<int64_t>(blockIdx.x) * kSwThreads + threadIdx.x; id < total;
         id += static_cast<int64_t>(gridDim.x) * kSwThreads) {
        const int64_t t = id / S;
        const int j = static_cast<int>(id - t * S);
        uint8_t* f = a.frames + t * a.F;
        if (j == 0) {
            const int size = (S + 1) * n2;
            f[0] = static_cast<uint8_t>(size >> 8);
            f[1] = static_cast<uint8_t>(size);
            f[2] = 0;
            f[3] = 0;
        }
        if (j == S - 1)
            for (int o = 4 + S * n2; o < a.F; ++o) f[o] = 0;
        uint8_t* blk = f + 4 + j * n2;
        if (j >= a.blocks) {
            for (int p = 0; p < n2; ++p) blk[p] = 0;
            continue;
        }
        const uint8_t* yt = a.y + t * Sk + j * k;
        for (int p = 0; p < k; ++p) blk[p] = yt[p];
        for (int p = k; p < n2; ++p) {
            uint8_t acc = 0;
            for (int i = 0; i < k; ++i) {
                const int64_t r = t - (p - i);
                const int lc = lg[i * n2 + p];
                if (r < 0 || lc < 0) continue;
                const uint8_t v = a.y[r * Sk + j * k + i];
                if (v) acc ^= gexp[lc + glog[v]];
            }
            blk[p] = acc;
        }
    }
}


// ---- tiled relay / destination (the path both batched calls take) -------------------------
// One workgroup walks a contiguous run of tiles of kTR packets (so the history rows in front of a
// tile were loaded by the tile before it, on the same XCD: L2 hits, not HBM).  Per tile:
//  1. the erasure flags of the tile and of the H rows in front of it, and per packet the mask of
//     its decode window (the n flags of rows u-n+1..u);
//  2. the rows (one contiguous slab of rows*stride bytes) into LDS with 16-byte loads;
//  3. the data positions m < k of every row, transposed to position-major words:
//     CT[row][m][g] = bytes of blocks 4g..4g+3 at position m (0 for an erased row, a row before
//     packet 0 and blocks past `blocks`);
//  4. the decode (decodeBlock T = n-1, t = 0 through the window-n rule of the packet's mask) of every
//     packet whose window holds 0 < erasures < n-k+1, IN PLACE: the data symbol m of packet u's
//     diagonal is CT[u-n+1+m][m], and no other packet reads it (a diagonal belongs to one packet);
//  5. the output rows into an LDS tile (laid out as in HBM), then 16-byte stores.
// Relay (Decoder_Symbol_Wise.cpp:547-619): frame t block j position p = encodeBlock over G2 of the
// reversed decoded diagonal Y_u[i] = d_u[k-1-i]; parity p reads Y_{t-(p-i)}[i] = d_{t-p+i}[k-1-i],
// which is CT[t-p-n1+k][k-1-i] for every i: one row.  With G2 = [I | P] the systematic positions
// are the same formula (G2[k-1-m][p] = [m == k-1-p]), so frame word (t, g, p) =
//   XOR_m G2[k-1-m][p] * CT[t-p-n1+k][m][g]       (a copy for p < k)
// with the products as v_perm_b32 register tables per (p, m), p wave-uniform.
// Destination (:621-665): out[t][j*k + i] = d_t[k-1-i][j] = CT[t-n2+k-i][k-1-i][j].
constexpr int kTR = 32;          // packets per tile: kTR*F and kTR*S*k are multiples of 16
constexpr int kTThreads = 256;
constexpr int kTMaxH = 40;       // rows in front of a tile: n1 + n2 - 2 (n <= 17 each: rule tables)

struct SwTileArgs {
    const uint8_t* in;      // rows of in_stride bytes; symbol (row, j, m) at in_off + j*n + m
    int64_t in_stride;
    int in_off;
    const uint8_t* er;      // per row: 1 = erased
    int64_t P;
    int n;                  // code length of the rows read (n1 at the relay, n2 at the destination)
    int S, S4, blocks;      // S4 = S rounded up to 4 (CT words)
    int H;                  // rows staged in front of a tile
    int D0;                 // packets decoded in front of the tile (relay: n2-1, destination: 0)
    const uint8_t* rules;   // window-n rule table (raw coefficients)
    int ES;
    const uint8_t* gf;      // exp[512], log[256]
    uint8_t* flag;          // per packet (may be null): erasures >= n-k+1
    int n2;                 // relay: frame code length and generator (k x n2)
    const uint8_t* G2;
    uint8_t* out;           // relay: frames (rows of F bytes); destination: rows of S*k bytes
    int out_row;            // F or S*k
    int64_t ntiles;
    int tiles_per_wg;
    int off_tb, off_ct, off_raw, off_rule;  // LDS layout (bytes)
    uint64_t* stamps;       // diagnostics (FEC_SWDF_STAMPS): per workgroup, cycles per phase summed over tiles
};

constexpr int kTQ = 8;  // 16-byte chunks per thread of a tile's slab (32 KB of rows at most)

// Step (t, g) to the item `step` further on (items t*G + g).
__device__ __forceinline__ void item_step(int& t, int& g, int st, int sg, int G) {
    g += sg;
    t += st;
    if (g >= G) {
        g -= G;
        ++t;
    }
}

template <int K, bool RELAY>
__global__ __launch_bounds__(kTThreads) void fec_sw_tile_kernel(SwTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // exp[0..509] then zeros to 1039; log16[x] = log x, 512 for x = 0: exp[log16 a + log16 b] = a*b
    // for every a, b (a zero operand lands in the zeros), no branch
    uint8_t* gexp = smem;
    uint16_t* glog16 = reinterpret_cast<uint16_t*>(smem + 1040);
    uint64_t* fbits = reinterpret_cast<uint64_t*>(smem + 1552);       // [2]: erasure flags of local rows
    uint32_t* pmask = reinterpret_cast<uint32_t*>(smem + 1568);       // [kTR + kTMaxH]
    uint32_t* tb = reinterpret_cast<uint32_t*>(smem + a.off_tb);      // relay: [n2][K][5]
    const uint32_t ct = static_cast<uint32_t>(a.off_ct);               // LDS byte offsets
    const uint32_t raw = static_cast<uint32_t>(a.off_raw);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = a.n, S = a.S, S4 = a.S4, G = S4 >> 2, H = a.H, blocks = a.blocks;
    const int ctrow = K * S4;  // CT bytes per row
    const int rows = kTR + H;
    const int stride = static_cast<int>(a.in_stride);
    for (int i = tid; i < 1040; i += kTThreads) gexp[i] = i < 510 ? a.gf[i] : 0;
    for (int i = tid; i < 256; i += kTThreads) glog16[i] = i ? a.gf[512 + i] : 512;
    __syncthreads();
    if constexpr (RELAY) {
        // v_perm tables of G2[K-1-m][p]: c*{0..7}, c*({0..7}<<3), c*({0..3}<<6)
        for (int it = tid; it < a.n2 * K; it += kTThreads) {
            const int p = it / K, m = it - p * K;
            const int lc = glog16[a.G2[(K - 1 - m) * a.n2 + p]];
            uint32_t w[5] = {0, 0, 0, 0, 0};
            for (int x = 0; x < 8; ++x) {
                w[x >> 2] |= uint32_t(gexp[lc + glog16[x]]) << (8 * (x & 3));
                w[2 + (x >> 2)] |= uint32_t(gexp[lc + glog16[x << 3]]) << (8 * (x & 3));
            }
            for (int x = 0; x < 4; ++x) w[4] |= uint32_t(gexp[lc + glog16[x << 6]]) << (8 * x);
            for (int q = 0; q < 5; ++q) tb[it * 5 + q] = w[q];
        }
    }
    uint16_t* rl = reinterpret_cast<uint16_t*>(smem + a.off_rule) + wave * (16 + 16 * 17);  // this wave's rule
    uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t st_prev = 0;
    auto stamp = [&](int k) {
        if (a.stamps) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            if (k > 0) st_acc[k - 1] += now - st_prev;
            st_prev = now;
        }
    };
    // lane-constant item decompositions: CT items (m, g) = lane + 64i
    const int cm0 = lane / G, cg0 = lane - cm0 * G, cst = 64 / G, csg = 64 - cst * G;
    const int NB = (kTR * G + 63) >> 6;  // 64-item blocks of (t, g) items per output position
    const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * a.tiles_per_wg;
    const int64_t tile1 = min(tile0 + a.tiles_per_wg, a.ntiles);
    const uint8_t* in_end = a.in + a.P * a.in_stride;
    const __amdgpu_buffer_rsrc_t rer =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.er), 0, static_cast<int>(min<int64_t>(a.P, fec::kRsrcMax)), 0x00020000);

    // Loads of a tile's rows slab (16-byte chunks of the aligned span, through a buffer resource:
    // past the input's end they read zero) and flags, into registers.
    uint4 v[kTQ];
    uint32_t fl = 0;
    int delta = 0, lrs = 0;
    auto issue = [&](int64_t tile) {
        const int64_t t0 = tile * kTR, r0 = t0 - H, rs = r0 < 0 ? 0 : r0;
        const int nt = static_cast<int>(min<int64_t>(kTR, a.P - t0));
        const uint8_t* gstart = a.in + rs * a.in_stride;
        const uint8_t* ga = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(gstart) & ~uintptr_t(15));
        const int dl = static_cast<int>(gstart - ga);
        const int nch = (dl + static_cast<int>((t0 + nt - rs) * a.in_stride) + 15) >> 4;
        const int64_t span = in_end - ga;
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(ga), 0, static_cast<int>(min<int64_t>(span, fec::kRsrcMax)), 0x00020000);
#pragma unroll
        for (int q = 0; q < kTQ; ++q) {
            const int c = tid + q * kTThreads;
            const uint32_t off = c < nch ? static_cast<uint32_t>(16 * c) : 0x7ffffff0u;
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
            v[q] = make_uint4(x[0], x[1], x[2], x[3]);
        }
        const int64_t r = r0 + tid;
        const uint32_t foff = (tid < rows && r >= 0 && r < a.P) ? static_cast<uint32_t>(r) : 0x7ffffff0u;
        fl = __builtin_amdgcn_raw_buffer_load_b8(rer, foff, 0, 0);
        delta = dl;
        lrs = static_cast<int>(rs - r0);
    };
    if (tile0 < tile1) issue(tile0);
    for (int64_t tile = tile0; tile < tile1; ++tile) {
        const int64_t t0 = tile * kTR;
        const int nt = static_cast<int>(min<int64_t>(kTR, a.P - t0));
        stamp(0);
        // 1. this tile's rows and flags into LDS; the next tile's loads go out
#pragma unroll
        for (int q = 0; q < kTQ; ++q) {
            const int c = tid + q * kTThreads;
            if (16 * c < 16 + rows * stride) *reinterpret_cast<uint4*>(smem + raw + 16 * c) = v[q];
        }
        {
            const uint64_t bal = __ballot(fl != 0);
            if (wave < 2 && lane == 0) fbits[wave] = bal;
        }
        const int dlt = delta, lr0 = lrs;
        __syncthreads();
        stamp(1);
        // 2. per decoded packet u = t0 - D0 + d (d = wave + 4*lane, this wave's): the mask of its
        // window; the tile's flags; the first two decode rules this wave needs, into registers
        const int nd = a.D0 + nt;
        uint32_t dec = 0;  // lanes (d = wave + 4*lane) whose packet is decoded
        {
            const int d = wave + 4 * lane;
            uint32_t m = 0;
            if (d < nd) {
                const int lo = H - a.D0 + d - n + 1;  // local row of the window's first symbol
                const uint64_t f0 = fbits[0], f1 = fbits[1];
                const uint64_t w = lo < 64 ? ((f0 >> lo) | (lo ? f1 << (64 - lo) : 0)) : (f1 >> (lo - 64));
                m = static_cast<uint32_t>(w) & ((n >= 32) ? ~0u : ((1u << n) - 1u));
                pmask[d] = m;
                if (a.flag && d >= a.D0) a.flag[t0 + d - a.D0] = __popc(m) >= n - K + 1 ? 1 : 0;
            }
            const int cnt = __popc(m);
            dec = static_cast<uint32_t>(__ballot(d < nd && cnt > 0 && cnt < n - K + 1));
        }
        const int ESw = a.ES >> 2;  // rule entries are whole dwords
        uint32_t pre[2][2] = {{0, 0}, {0, 0}};
        {
            uint32_t dd = dec;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (!dd) break;
                const int i = __builtin_ctz(dd);
                dd &= dd - 1;
                const uint32_t* e = reinterpret_cast<const uint32_t*>(a.rules + static_cast<int64_t>(pmask[wave + 4 * i]) * a.ES);
                if (lane < ESw) pre[j][0] = e[lane];
                if (lane + 64 < ESw) pre[j][1] = e[lane + 64];
            }
        }
        if (tile + 1 < tile1) issue(tile + 1);
        // 3. CT[l][m][g] (a wave per row): four byte reads, then the blocks past `blocks` masked
        for (int l = wave; l < rows; l += kTThreads / 64) {
            const bool live = l >= lr0 && l < H + nt && !((l < 64 ? fbits[0] >> l : fbits[1] >> (l - 64)) & 1u);
            const uint32_t rowp = raw + dlt + max(l - lr0, 0) * stride + a.in_off;
            int m = cm0, g = cg0;
            for (int it = lane; it < K * G; it += 64) {
                const uint32_t src = rowp + m + 4 * g * n;
                const uint32_t b0 = smem[src], b1 = smem[src + n], b2 = smem[src + 2 * n], b3 = smem[src + 3 * n];
                const uint32_t w = (b0 | b1 << 8 | b2 << 16 | b3 << 24) & (live ? keep_bytes(blocks - 4 * g) : 0u);
                *reinterpret_cast<uint32_t*>(smem + ct + l * ctrow + m * S4 + 4 * g) = w;
                item_step(m, g, cst, csg, G);
            }
        }
        __syncthreads();
        stamp(2);
        // 4. decode in place (a wave per packet whose window holds 0 < erasures < n-k+1): the
        // window-n rule of the packet's mask into this wave's LDS slot (which data symbols are
        // recovered, their coefficients as logs), then per lane (4 blocks) the products
        {
            uint32_t dd = dec;
            for (int j = 0; dd; ++j) {
                const int i = __builtin_ctz(dd);
                dd &= dd - 1;
                const int d = wave + 4 * i;
                const uint32_t mask = pmask[d];
                const int lb = H - a.D0 + d - n + 1;  // local row of diagonal position 0
                uint32_t w0, w1;
                if (j < 2) {
                    w0 = j == 0 ? pre[0][0] : pre[1][0];
                    w1 = j == 0 ? pre[0][1] : pre[1][1];
                } else {
                    const uint32_t* e = reinterpret_cast<const uint32_t*>(a.rules + static_cast<int64_t>(mask) * a.ES);
                    w0 = lane < ESw ? e[lane] : 0;
                    w1 = lane + 64 < ESw ? e[lane + 64] : 0;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int i0 = 4 * lane + q, i1 = 4 * (lane + 64) + q;
                    const uint32_t c0 = (w0 >> (8 * q)) & 255, c1 = (w1 >> (8 * q)) & 255;
                    if (i0 < K + K * n) rl[i0] = i0 < K ? c0 : glog16[c0];
                    if (i1 < K + K * n) rl[i1] = i1 < K ? c1 : glog16[c1];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                uint32_t recm = 0;  // recovered data symbols (erased, rule present): wave-uniform
                for (int m = 0; m < K; ++m)
                    if (((mask >> m) & 1u) && rl[m] != 0xFF) recm |= 1u << m;
                for (int g = lane; g < G; g += 64) {
                    uint32_t acc[K];
#pragma unroll
                    for (int m = 0; m < K; ++m) acc[m] = 0;
                    for (int c = 0; c < n; ++c) {
                        if ((mask >> c) & 1u) continue;  // an erased symbol is zero
                        const int l = lb + c;
                        uint32_t x = 0;
                        if (c < K) {
                            x = *reinterpret_cast<const uint32_t*>(smem + ct + l * ctrow + c * S4 + 4 * g);
                        } else if (l >= lr0) {
                            const uint32_t src = raw + dlt + (l - lr0) * stride + a.in_off + c + 4 * g * n;
                            x = (uint32_t(smem[src]) | uint32_t(smem[src + n]) << 8 | uint32_t(smem[src + 2 * n]) << 16 |
                                 uint32_t(smem[src + 3 * n]) << 24) & keep_bytes(blocks - 4 * g);
                        }
                        const int lx0 = glog16[x & 255], lx1 = glog16[(x >> 8) & 255];
                        const int lx2 = glog16[(x >> 16) & 255], lx3 = glog16[x >> 24];
#pragma unroll
                        for (int m = 0; m < K; ++m) {
                            if (!((recm >> m) & 1u)) continue;
                            const int lc = rl[K + m * n + c];
                            acc[m] ^= uint32_t(gexp[lc + lx0]) | uint32_t(gexp[lc + lx1]) << 8 |
                                      uint32_t(gexp[lc + lx2]) << 16 | uint32_t(gexp[lc + lx3]) << 24;
                        }
                    }
#pragma unroll
                    for (int m = 0; m < K; ++m)
                        if ((recm >> m) & 1u) *reinterpret_cast<uint32_t*>(smem + ct + (lb + m) * ctrow + m * S4 + 4 * g) = acc[m];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the slot is reused by the next packet
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        __syncthreads();
        stamp(3);
        // 5. the output tile (aliases the raw rows: all reads of them are done); items (p, t, g)
        // in blocks of 64 with p wave-uniform
        const uint32_t otile = raw;
        const int orow = a.out_row;
        if constexpr (RELAY) {
            const int n2 = a.n2;
            // frame header [size BE16][0][0] and the n2-2 zero bytes after the S blocks
            const int size = (S + 1) * n2;
            for (int t = tid; t < nt; t += kTThreads) {
                uint8_t* f = smem + otile + t * orow;
                f[0] = uint8_t(size >> 8);
                f[1] = uint8_t(size);
                f[2] = 0;
                f[3] = 0;
                for (int b = 4 + S * n2; b < orow; ++b) f[b] = 0;
            }
            int cur_p = -1;
            uint32_t tab[K][5];
            for (int ib = wave; ib < n2 * NB; ib += kTThreads / 64) {
                const int p = ib / NB;  // wave-uniform
                const int item = (ib - p * NB) * 64 + lane;
                const int t = item / G, g = item - t * G;
                if (p >= K && p != cur_p) {
#pragma unroll
                    for (int m = 0; m < K; ++m)
#pragma unroll
                        for (int q = 0; q < 5; ++q) tab[m][q] = tb[(p * K + m) * 5 + q];
                    cur_p = p;
                }
                if (t >= nt) continue;
                const uint32_t src = ct + (H + t - p - n + K) * ctrow + 4 * g;  // local row t-p-n1+k
                uint32_t w;
                if (p < K) {
                    w = *reinterpret_cast<const uint32_t*>(smem + src + (K - 1 - p) * S4);
                } else {
                    uint32_t x[K];
#pragma unroll
                    for (int m = 0; m < K; ++m) x[m] = *reinterpret_cast<const uint32_t*>(smem + src + m * S4);
                    w = 0;
#pragma unroll
                    for (int m = 0; m < K; ++m) w ^= gf_mul4x(tab[m], x[m]);
                }
                uint8_t* o = smem + otile + t * orow + 4 + p + 4 * g * n2;
                const int ne = min(4, S - 4 * g);
                o[0] = uint8_t(w);
                if (ne > 1) o[n2] = uint8_t(w >> 8);
                if (ne > 2) o[2 * n2] = uint8_t(w >> 16);
                if (ne > 3) o[3 * n2] = uint8_t(w >> 24);
            }
        } else {
            for (int ib = wave; ib < K * NB; ib += kTThreads / 64) {
                const int i = ib / NB;  // wave-uniform
                const int item = (ib - i * NB) * 64 + lane;
                const int t = item / G, g = item - t * G;
                if (t >= nt) continue;
                const uint32_t w = *reinterpret_cast<const uint32_t*>(smem + ct + (H + t - n + K - i) * ctrow +
                                                                      (K - 1 - i) * S4 + 4 * g);  // local row t-n2+k-i
                uint8_t* o = smem + otile + t * orow + i + 4 * g * K;
                const int ne = min(4, S - 4 * g);
                o[0] = uint8_t(w);
                if (ne > 1) o[K] = uint8_t(w >> 8);
                if (ne > 2) o[2 * K] = uint8_t(w >> 16);
                if (ne > 3) o[3 * K] = uint8_t(w >> 24);
            }
        }
        __syncthreads();
        stamp(4);
        // 16-byte stores of the tile's rows (t0 * orow is a multiple of 16: kTR * orow is)
        uint8_t* gout = a.out + t0 * orow;
        const int obytes = nt * orow;
        for (int c = tid; c < (obytes >> 4); c += kTThreads)
            *reinterpret_cast<uint4*>(gout + 16 * c) = *reinterpret_cast<const uint4*>(smem + otile + 16 * c);
        for (int b = (obytes & ~15) + tid; b < obytes; b += kTThreads) gout[b] = smem[otile + b];
        __syncthreads();
        stamp(5);
    }
    if (a.stamps && tid == 0)
        for (int k = 0; k < 5; ++k) a.stamps[static_cast<int64_t>(blockIdx.x) * 8 + k] = st_acc[k];
}


// ---- compile-time (k, n) specialisations of the tiled relay / destination ------------------
// The generic tile kernel above spends its time on byte-granular LDS work (a 4-byte word of the
// transposed rows costs four ds_read_u8 and ~30 VALU; a frame word four ds_write_b8) and on
// barrier-separated phases with little work each.  With k, n1 and n2 known at compile time the data
// movement is dword-wide, and a tile is 64 packets over 512 threads:
//  * the rows slab lands in LDS exactly as in HBM (a row's bytes at raw + dlt + l*stride); rows
//    before packet 0 and past the input read as zero through the buffer range check, and an erased
//    row's bytes are masked to zero as the slab lands (so no later step tests flags);
//  * every wave loads the tile's flags itself (a ballot: no LDS, no barrier before the masks);
//  * the decode patches the recovered data symbols into the rows in place (symbol (row r, block j,
//    position m) belongs to the diagonal of packet r+n-1-m only), a lane per (block, recovered
//    symbol);
//  * destination: output dword w of the tile's rows is gathered from the rows (4 byte reads, the
//    (t, j, i) of its bytes stepped incrementally) and stored straight to HBM;
//  * relay: per (row, group of 4 blocks) the 4*n1-byte span as n1+1 dword reads + v_alignbyte, and
//    the k position words by v_perm (CT[row][m][g]); the parity words (v_perm tables of G2 in
//    registers, parity wave-uniform); per (frame t, group g) the n2 code words transposed by v_perm
//    into the frame's 4*n2-byte run, written as dwords to an LDS tile of 4-byte-aligned rows; then
//    the tile is re-packed to the frame stride, 16 bytes per lane.
typedef uint32_t fec_v4u32 __attribute__((ext_vector_type(4)));
constexpr int kFR = 64;          // packets per tile
constexpr int kFT = 512;         // threads per workgroup
constexpr int kFW = kFT / 64;    // waves

constexpr int al16(int x) { return (x + 15) & ~15; }
constexpr int cmax(int x, int y) { return x > y ? x : y; }

// The whole geometry at compile time (k, n1, n2 and the payload size L): every division,
// bound and LDS offset below is a constant.
template <int K_, int N1_, int N2_, int L_, bool RELAY_, int TR_ = kFR, bool V2_ = false, int NT_ = kFT>
struct FastGeo {
    static constexpr int K = K_, N1 = N1_, N2 = N2_, L = L_;
    static constexpr bool RELAY = RELAY_;
    static constexpr int TR = TR_;                        // packets per tile
    static constexpr int NT = NT_, NW = NT_ / 64;         // threads, waves per workgroup
    static constexpr bool V2 = RELAY_ && V2_;             // relay: the row-scatter kernel (no CT / parity tiles)
    static constexpr bool CT3 = RELAY && !V2;             // relay: the three-tile (CT, parity, words) kernel
    static constexpr int S = (L + 2 + K - 1) / K;        // code blocks (= sub-streams)
    static constexpr int S4 = (S + 3) & ~3, G = S4 / 4;  // CT words per position
    static constexpr int N = RELAY ? N1 : N2;            // code length of the rows read
    static constexpr int IN_OFF = RELAY ? 0 : 4;         // byte of symbol (j, 0) in a row
    static constexpr int F = 2 + (S + 1) * N2;           // frame bytes
    static constexpr int STRIDE = RELAY ? S * N1 : F;    // input row bytes
    static constexpr int H = RELAY ? N1 + N2 - 2 : N2 - 1;  // rows staged in front of a tile
    static constexpr int D0 = RELAY ? N2 - 1 : 0;        // packets decoded in front of a tile
    static constexpr int ROWS = TR + H;
    static constexpr int OUT_ROW = RELAY ? F : S * K;
    static constexpr int F4 = (F + 3) & ~3;              // LDS frame pitch
    static constexpr int ES = (K * (1 + N) + 3) & ~3;    // rule entry bytes (fec_host.h DecodeRules)
    static constexpr int CTROW = K * S4;
    static constexpr int QCH = (16 + ROWS * STRIDE + 16 * NT - 1) / (16 * NT);  // slab chunks per thread
    static constexpr int SCH = (TR * OUT_ROW + 16 * NT - 1) / (16 * NT);      // output chunks per thread
    static constexpr int OFF_PMASK = 1552;
    static constexpr int OFF_RULE = OFF_PMASK + 4 * (TR + 64);
    static constexpr int RULE_U16 = K + K * N + 4;      // per wave
    static constexpr int OFF_TB = al16(OFF_RULE + NW * 2 * RULE_U16);
    static constexpr int OFF_CT = al16(OFF_TB + (CT3 ? (N2 - K) * K * 20 : 0));
    static constexpr int OFF_OW = al16(OFF_CT + (CT3 ? ROWS * CTROW : 0));
    static constexpr int OFF_RAW = al16(OFF_OW + (CT3 ? (N2 - K) * TR * S4 : 0));
    static constexpr int RAWB = al16(cmax(16 + ROWS * STRIDE + 4 * N + 32, CT3 ? (TR + 1) * F4 : 0));
    static constexpr int OFF_FR = OFF_RAW + RAWB;         // V2: the tile's frames at their own stride F
    static constexpr int LDS = OFF_FR + (V2 ? al16(TR * F) : 0);
    // waves per SIMD (the register budget of __launch_bounds__: 128 VGPRs, two workgroups per CU)
    static constexpr int WPE = 4;
    static constexpr uint32_t MDIV = static_cast<uint32_t>((uint64_t(1) << 32) / OUT_ROW + 1);
    static constexpr uint32_t MSTRIDE = static_cast<uint32_t>((uint64_t(1) << 32) / STRIDE + 1);
    // the H rows in front of a tile that is not a workgroup's first are the last H rows of the tile
    // before: the slab's first NH 16-byte chunks (its rows start at byte DLT of chunk 0, and row H
    // at a chunk boundary: t0 * STRIDE is a multiple of 16) are carried over in registers
    static constexpr int DLT = (16 - (H * STRIDE) % 16) % 16;
    static constexpr int NH = (DLT + H * STRIDE) / 16;
    static constexpr int HQ = (NH + NT - 1) / NT;
    static_assert(H <= 64 && D0 + TR <= TR + 64 && D0 + TR <= NT, "rows in front of a tile");
    static_assert(TR % 16 == 0 && TR <= 64, "tile rows: t0 * STRIDE and t0 * F multiples of 16");
    static_assert((DLT + H * STRIDE) % 16 == 0, "carried rows");
};

struct SwFastArgs {
    const uint8_t* in;      // rows of STRIDE bytes (frames at the destination)
    const uint8_t* er;
    int64_t P;
    const uint8_t* rules;   // window-n rules of the code read
    const uint8_t* gf;
    uint8_t* flag;
    const uint32_t* tab;    // relay: v_perm tables of G2[k-1-m][p], [n2][k][5] dwords
    uint8_t* out;
    int64_t ntiles;
    int tiles_per_wg;
    uint64_t* stamps;       // diagnostics (FEC_SWDF_STAMPS): per workgroup, cycles per phase summed over tiles
    int carry;              // carry the rows in front of a tile over from the tile before (FEC_SWDF_CARRY=0: reload)
};

// Phase clock for the diagnostics: cycles between consecutive marks, summed over the tiles.
struct PhaseClock {
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t prev = 0;
    bool on;
    __device__ explicit PhaseClock(bool o) : on(o) {}
    __device__ void mark(int k) {
        if (!on) return;
        const uint64_t now = __builtin_amdgcn_s_memtime();
        if (k > 0) acc[k - 1] += now - prev;
        prev = now;
    }
    __device__ void flush(uint64_t* out) {
        if (on && threadIdx.x == 0)
            for (int k = 0; k < 8; ++k) out[static_cast<int64_t>(blockIdx.x) * 8 + k] = acc[k];
    }
};

template <typename F, int... Is>
__device__ __forceinline__ void tfor_sw_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void tfor_sw(F&& f) {  // f(integral_constant<0..N-1>), unrolled
    tfor_sw_impl(f, std::make_integer_sequence<int, N>{});
}

template <int NW>
__device__ __forceinline__ void align_words(uint32_t (&d)[NW], int s) {  // d <- bytes from offset s
#pragma unroll
    for (int i = 0; i + 1 < NW; ++i) d[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], static_cast<uint32_t>(s));
}

// Staging, masks and the in-place decode: shared by both kernels.
template <class GM>
struct FastTile {
    static constexpr int K = GM::K, N = GM::N, IN_OFF = GM::IN_OFF, H = GM::H, D0 = GM::D0, ROWS = GM::ROWS;
    static constexpr int STRIDE = GM::STRIDE, QCH = GM::QCH;
    uint8_t* smem;
    const SwFastArgs& a;
    int tid, lane, wave;
    uint8_t* gexp;
    uint16_t* glog16;
    uint32_t* pmask;
    uint16_t* rl;
    static constexpr int NH = GM::NH, HQ = GM::HQ;
    uint4 v[QCH];
    uint4 hc[HQ];                   // the next tile's first NH chunks (keep())
    bool carry = false, carry_next = false;
    uint32_t f0 = 0, f1 = 0;        // flags of local rows lane and 64 + lane (next tile)
    uint64_t fb0 = 0, fb1 = 0;      // flags of local rows 0..63, 64..127 (this tile)
    int dlt = 0, dlt_next = 0;      // LDS byte of local row 0 = raw + dlt
    uint32_t dec = 0;               // this wave's decoded packets (bit i: d = wave + GM::NW*i)
    uint32_t pre[2][2];

    __device__ FastTile(uint8_t* s, const SwFastArgs& args) : smem(s), a(args) {
        tid = threadIdx.x;
        lane = tid & 63;
        wave = tid >> 6;
        gexp = smem;
        glog16 = reinterpret_cast<uint16_t*>(smem + 1040);
        pmask = reinterpret_cast<uint32_t*>(smem + GM::OFF_PMASK);
        rl = reinterpret_cast<uint16_t*>(smem + GM::OFF_RULE) + wave * GM::RULE_U16;
        for (int i = tid; i < 1040; i += GM::NT) gexp[i] = i < 510 ? a.gf[i] : 0;
        for (int i = tid; i < 256; i += GM::NT) glog16[i] = i ? a.gf[512 + i] : 512;
    }
    // the slab of rows [r0, t0+nt) (r0 = t0 - H) and the tile's flags, into registers; with cont
    // (the tile follows this workgroup's previous one) its first NH chunks come from keep() instead
    __device__ void issue(int64_t tile, bool cont) {
        carry_next = cont;
        const int64_t t0 = tile * GM::TR, r0 = t0 - H;
        const int nt = static_cast<int>(min<int64_t>(GM::TR, a.P - t0));
        const int64_t g0 = r0 * STRIDE;                         // may be negative
        const int64_t A = g0 >= 0 ? (g0 & ~int64_t(15)) : -((-g0 + 15) & ~int64_t(15));
        const int64_t base = A > 0 ? A : 0;
        const int nch = static_cast<int>((g0 - A + static_cast<int64_t>(H + nt) * STRIDE + 15) >> 4);
        const int64_t span = a.P * STRIDE - base;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.in + base), 0, static_cast<int>(span < fec::kRsrcMax ? span : fec::kRsrcMax), 0x00020000);
#pragma unroll
        for (int q = 0; q < QCH; ++q) {
            const int c = tid + q * GM::NT;
            const int64_t o = A - base + 16 * static_cast<int64_t>(c);  // < 0: a row before packet 0
            const uint32_t off = (c < nch && o >= 0 && !(cont && c < NH)) ? static_cast<uint32_t>(o) : 0x7ffffff0u;
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
            v[q] = make_uint4(x[0], x[1], x[2], x[3]);
        }
        const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.er), 0, static_cast<int>(a.P < fec::kRsrcMax ? a.P : fec::kRsrcMax), 0x00020000);
        const int64_t ra = r0 + lane, rb = r0 + 64 + lane;
        f0 = __builtin_amdgcn_raw_buffer_load_b8(re, (lane < ROWS && ra >= 0) ? static_cast<uint32_t>(ra) : 0x7ffffff0u, 0, 0);
        f1 = __builtin_amdgcn_raw_buffer_load_b8(re, (64 + lane < ROWS && rb >= 0) ? static_cast<uint32_t>(rb) : 0x7ffffff0u, 0, 0);
        dlt_next = static_cast<int>(g0 - A);
    }
    // after the decode (the rows are final): the last H rows of this (full) tile, which the next
    // tile of the workgroup starts with, into registers -- chunk c of the next slab is chunk
    // TR * STRIDE / 16 + c of this one
    __device__ void keep() {
#pragma unroll
        for (int q = 0; q < HQ; ++q) {
            const int c = tid + q * GM::NT;
            if (c < NH) hc[q] = *reinterpret_cast<const uint4*>(smem + GM::OFF_RAW + GM::TR * STRIDE + 16 * c);
        }
    }
    __device__ uint32_t rowb(int l) const { return static_cast<uint32_t>(GM::OFF_RAW + dlt + l * STRIDE); }
    __device__ bool erased(int l) const { return ((l < 64 ? fb0 >> l : fb1 >> (l - 64)) & 1u) != 0; }
    // the slab into LDS, the bytes of erased rows zeroed
    __device__ void land() {
        fb0 = __ballot(f0 != 0);
        fb1 = __ballot(f1 != 0);
        dlt = dlt_next;
        carry = carry_next;
        const bool any = (fb0 | fb1) != 0;
#pragma unroll
        for (int q = 0; q < QCH; ++q) {
            const int c = tid + q * GM::NT;
            if (16 * c >= 16 + ROWS * STRIDE) continue;
            uint4 x = v[q];
            if (q < HQ && carry && c < NH) x = hc[q < HQ ? q : 0];  // (masking them again is harmless)
            if (any) {
                // chunk bytes [16c, 16c+16) = row bytes from (16c - dlt); at most two rows
                const int o = 16 * c - dlt;
                const int l = o < 0 ? -1 : static_cast<int>(__umulhi(static_cast<uint32_t>(o), GM::MSTRIDE));
                const int split = o < 0 ? -o : (l + 1) * STRIDE - o;  // first byte of the next row
                const bool e0 = l >= 0 && erased(l), e1 = erased(l + 1);
                if (e0 || e1) {
                    uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int q2 = 0; q2 < 4; ++q2) {
                        uint32_t keep = 0;
#pragma unroll
                        for (int y = 0; y < 4; ++y) {
                            const bool second = 4 * q2 + y >= split;
                            if (!(second ? e1 : e0)) keep |= 0xFFu << (8 * y);
                        }
                        w[q2] &= keep;
                    }
                    x = make_uint4(w[0], w[1], w[2], w[3]);
                }
            }
            *reinterpret_cast<uint4*>(smem + GM::OFF_RAW + 16 * c) = x;
        }
    }
    // masks of this wave's packets (d = wave + GM::NW*lane), flags out, the first two rules of this
    // wave into registers
    __device__ void masks(int64_t t0, int nt) {
        const int nd = D0 + nt;
        const int d = wave + GM::NW * lane;
        uint32_t m = 0;
        if (d < nd) {
            const int lo = H - D0 + d - N + 1;
            const uint64_t w = lo < 64 ? ((fb0 >> lo) | (lo ? fb1 << (64 - lo) : 0)) : (fb1 >> (lo - 64));
            m = static_cast<uint32_t>(w) & ((1u << N) - 1u);
            pmask[d] = m;
            if (a.flag && d >= D0) a.flag[t0 + d - D0] = __popc(m) >= N - K + 1 ? 1 : 0;
        }
        const int cnt = __popc(m);
        dec = static_cast<uint32_t>(__ballot(d < nd && cnt > 0 && cnt < N - K + 1));
        constexpr int ESw = GM::ES >> 2;
        uint32_t dd = dec;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            pre[j][0] = pre[j][1] = 0;
            if (dd) {
                const int i = __builtin_ctz(dd);
                dd &= dd - 1;
                const uint32_t mm = __builtin_amdgcn_readlane(m, i);
                const uint32_t* e = reinterpret_cast<const uint32_t*>(a.rules + static_cast<int64_t>(mm) * GM::ES);
                if (lane < ESw) pre[j][0] = e[lane];
                if (lane + 64 < ESw) pre[j][1] = e[lane + 64];
            }
        }
    }
    // decode in place: a wave per decoded packet; a lane per (block j, recovered symbol)
    __device__ void decode() {
        constexpr int ESw = GM::ES >> 2;
        uint32_t dd = dec;
        for (int jj = 0; dd; ++jj) {
            const int i = __builtin_ctz(dd);
            dd &= dd - 1;
            const int d = wave + GM::NW * i;
            const uint32_t mask = pmask[d];
            const int lb = H - D0 + d - N + 1;  // local row of diagonal position 0
            uint32_t w0, w1;
            if (jj < 2) {
                w0 = jj == 0 ? pre[0][0] : pre[1][0];
                w1 = jj == 0 ? pre[0][1] : pre[1][1];
            } else {
                const uint32_t* e = reinterpret_cast<const uint32_t*>(a.rules + static_cast<int64_t>(mask) * GM::ES);
                w0 = lane < ESw ? e[lane] : 0;
                w1 = lane + 64 < ESw ? e[lane + 64] : 0;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i0 = 4 * lane + q, i1 = 4 * (lane + 64) + q;
                const uint32_t c0 = (w0 >> (8 * q)) & 255, c1 = (w1 >> (8 * q)) & 255;
                if (i0 < K + K * N) rl[i0] = i0 < K ? c0 : glog16[c0];
                if (i1 < K + K * N) rl[i1] = i1 < K ? c1 : glog16[c1];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t recm = 0;
#pragma unroll
            for (int m = 0; m < K; ++m)
                if (((mask >> m) & 1u) && rl[m] != 0xFF) recm |= 1u << m;
            const int nrec = __popc(recm);
            for (int it = lane; it < GM::S * nrec; it += 64) {
                const int r = it / GM::S, j = it - r * GM::S;
                uint32_t mm = recm;
                for (int x = 0; x < r; ++x) mm &= mm - 1;
                const int m = __builtin_ctz(mm);
                const uint16_t* lc = rl + K + m * N;
                uint32_t acc = 0;
#pragma unroll
                for (int c = 0; c < N; ++c) {
                    const uint32_t x = ((mask >> c) & 1u) ? 0u : smem[rowb(lb + c) + IN_OFF + j * N + c];
                    acc ^= gexp[lc[c] + glog16[x]];
                }
                smem[rowb(lb + m) + IN_OFF + j * N + m] = uint8_t(acc);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
};

// Destination: out[t][j*k + i] = d_t[k-1-i][j] = frame row (t-n+k-i) byte 4 + j*n + k-1-i.
template <class GM>
__global__ __launch_bounds__(kFT) void fec_sw_fast_dest_kernel(SwFastArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int K = GM::K, N = GM::N, S = GM::S, SK = GM::OUT_ROW;
    FastTile<GM> T(smem, a);
    __syncthreads();
    const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * a.tiles_per_wg;
    const int64_t tile1 = min(tile0 + a.tiles_per_wg, a.ntiles);
    PhaseClock clk(a.stamps != nullptr);
    if (tile0 < tile1) T.issue(tile0, false);
    for (int64_t tile = tile0; tile < tile1; ++tile) {
        const int64_t t0 = tile * GM::TR;
        const int nt = static_cast<int>(min<int64_t>(GM::TR, a.P - t0));
        clk.mark(0);
        T.land();
        T.masks(t0, nt);
        if (tile + 1 < tile1) T.issue(tile + 1, a.carry != 0);
        __syncthreads();
        clk.mark(1);
        T.decode();
        __syncthreads();
        if (a.carry && tile + 1 < tile1) T.keep();
        clk.mark(2);
        // output bytes of the tile's rows, 16 per lane: byte b -> row t = b / SK, o = b - t*SK,
        // j = o / K, i = o % K; LDS byte = row (t + K-1-i) of the slab, 4 + j*N + K-1-i.  A fixed
        // number of buffer stores per lane (unused ones out of range).
        const int obytes = nt * SK;
        uint8_t* gout = a.out + t0 * SK;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(gout, 0, obytes & ~15, 0x00020000);
#pragma unroll
        for (int q = 0; q < GM::SCH; ++q) {
            asm volatile("" ::: "memory");  // one chunk's reads at a time (registers)
            const int c = T.tid + q * kFT;
            const uint32_t b = 16 * c;
            uint32_t val[4] = {0, 0, 0, 0};
            if constexpr (SK % 16 == 0 && 16 % K == 0) {
                // a row's output is whole chunks and a chunk whole blocks (k = 8: two): byte (jb, i)
                // of the chunk is at a compile-time offset from one address, (K-1-i) rows and jb
                // blocks on -- 16 byte reads with immediate offsets, no per-byte index arithmetic
                if (static_cast<int>(b) < obytes) {
                    constexpr int CPR = SK / 16, BPC = 16 / K;
                    const int t = static_cast<int>(b) / (16 * CPR);
                    const int j0 = (static_cast<int>(b) / 16 - t * CPR) * BPC;
                    const uint8_t* base = smem + T.rowb(t) + 4 + j0 * N;
                    tfor_sw<16>([&](auto xc) __attribute__((always_inline)) {
                        constexpr int x = decltype(xc)::value;
                        constexpr int jb = x / K, i = x % K;
                        const uint32_t byte = base[(K - 1 - i) * GM::STRIDE + jb * N + K - 1 - i];
                        val[x >> 2] |= byte << (8 * (x & 3));
                    });
                }
            } else if (static_cast<int>(b) < obytes) {
                int t = static_cast<int>(b / SK);
                const int o = static_cast<int>(b) - t * SK;
                int j = o / K, i = o - j * K;
                uint32_t acc = 0;
#pragma unroll 1
                for (int x = 0; x < 16; ++x) {
                    const uint32_t src = T.rowb(t + K - 1 - i) + 4 + j * N + K - 1 - i;
                    acc = (acc >> 8) | (uint32_t(smem[src]) << 24);  // bytes in order after four
                    if ((x & 3) == 3) {
                        val[0] = val[1];
                        val[1] = val[2];
                        val[2] = val[3];
                        val[3] = acc;
                    }
                    if (++i == K) {
                        i = 0;
                        if (++j == S) {
                            j = 0;
                            ++t;
                        }
                    }
                }
            }
            const uint32_t so = static_cast<int>(b) + 16 <= obytes ? b : 0x7ffffff0u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(fec_v4u32, make_uint4(val[0], val[1], val[2], val[3])), ro, so, 0, 0);
            if (static_cast<int>(b) < obytes && static_cast<int>(b) + 16 > obytes)  // the output's ragged end
                for (int x = 0; static_cast<int>(b) + x < obytes; ++x) gout[b + x] = uint8_t(val[x >> 2] >> (8 * (x & 3)));
        }
        __syncthreads();
        clk.mark(3);
    }
    clk.flush(a.stamps);
}

// Relay: frame t = [size BE16][0, 0][S blocks of n2][n2-2 zeros]; block j position p =
// XOR_m G2[k-1-m][p] * CT[t-p-n1+k][m][j] (a copy for p < k).
template <class GM>
__global__ __launch_bounds__(kFT, 4) void fec_sw_fast_relay_kernel(SwFastArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int K = GM::K, N1 = GM::N1, N2 = GM::N2, S = GM::S, S4 = GM::S4, G = GM::G, H = GM::H;
    constexpr int F = GM::F, F4 = GM::F4, CTROW = GM::CTROW;
    constexpr int size = (S + 1) * N2;
    FastTile<GM> T(smem, a);
    uint32_t* tbl = reinterpret_cast<uint32_t*>(smem + GM::OFF_TB);  // [p - k][m][5] v_perm tables
    for (int i = T.tid; i < (N2 - K) * K * 5; i += kFT) tbl[i] = a.tab[K * K * 5 + i];
    __syncthreads();
    const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * a.tiles_per_wg;
    const int64_t tile1 = min(tile0 + a.tiles_per_wg, a.ntiles);
    PhaseClock clk(a.stamps != nullptr);
    if (tile0 < tile1) T.issue(tile0, false);
    for (int64_t tile = tile0; tile < tile1; ++tile) {
        const int64_t t0 = tile * GM::TR;
        const int nt = static_cast<int>(min<int64_t>(GM::TR, a.P - t0));
        clk.mark(0);
        T.land();
        T.masks(t0, nt);
        if (tile + 1 < tile1) T.issue(tile + 1, a.carry != 0);
        __syncthreads();
        clk.mark(1);
        T.decode();
        __syncthreads();
        if (a.carry && tile + 1 < tile1) T.keep();
        clk.mark(2);
        // CT[l][m][g] from the (decoded) rows: a lane per (row, group of 4 blocks); only the rows
        // a frame of the tile reads (local rows >= k-1)
        for (int it = T.tid; it < (H + nt - (K - 1)) * G; it += kFT) {
            const int l = K - 1 + it / G, g = it % G;
            const uint32_t sb = T.rowb(l) + 4 * g * N1;
            uint32_t d[N1 + 1];
            const uint32_t ab = sb & ~3u;
#pragma unroll
            for (int q = 0; q <= N1; ++q) d[q] = *reinterpret_cast<const uint32_t*>(smem + ab + 4 * q);
            align_words(d, static_cast<int>(sb & 3));
            const uint32_t cb = GM::OFF_CT + l * CTROW + 4 * g;
#pragma unroll
            for (int m = 0; m < K; ++m)
                *reinterpret_cast<uint32_t*>(smem + cb + m * S4) = gather4(d, m, N1 + m, 2 * N1 + m, 3 * N1 + m);
        }
        __syncthreads();
        clk.mark(3);
        // parity words OW[p-k][t][g] = XOR_m G2[k-1-m][p] * CT[t-p-n1+k][m][g]: 64-item blocks with
        // p wave-uniform, the 5k v_perm tables of p in registers (reloaded when p changes)
        {
            const int NBk = (nt * G + 63) >> 6;
            const int nb = (N2 - K) * NBk, per = (nb + kFW - 1) / kFW;  // a contiguous run of blocks per wave
            int cur_p = -1;
            uint32_t tt[K][5];
            for (int ib = T.wave * per; ib < min(nb, (T.wave + 1) * per); ++ib) {
                const int pi = ib / NBk;  // wave-uniform
                const int p = K + pi;
                const int item = (ib - pi * NBk) * 64 + T.lane;
                if (p != cur_p) {
#pragma unroll
                    for (int m = 0; m < K; ++m)
#pragma unroll
                        for (int q = 0; q < 5; ++q) tt[m][q] = tbl[(pi * K + m) * 5 + q];
                    cur_p = p;
                }
                if (item >= nt * G) continue;
                const int t = item / G, g = item - t * G;
                const uint32_t src = GM::OFF_CT + (H + t - p - N1 + K) * CTROW + 4 * g;  // local row t-p-n1+k
                uint32_t x[K];
#pragma unroll
                for (int m = 0; m < K; ++m) x[m] = *reinterpret_cast<const uint32_t*>(smem + src + m * S4);
                uint32_t w = 0;
#pragma unroll
                for (int m = 0; m < K; ++m) w ^= gf_mul4x(tt[m], x[m]);
                *reinterpret_cast<uint32_t*>(smem + GM::OFF_OW + (pi * kFR + t) * S4 + 4 * g) = w;
            }
        }
        __syncthreads();
        clk.mark(4);
        // frame words of (t, g) -> the frame's 4*n2-byte run for blocks 4g..4g+3 in LDS rows of F4
        // (the rows' space: free once CT is built); group 0 also writes the header, the last group
        // the zero tail up to F4
        for (int it = T.tid; it < nt * G; it += kFT) {
            const int t = it / G, g = it % G;
            uint32_t W[N2];
#pragma unroll
            for (int p = 0; p < N2; ++p) {
                if (p < K)
                    W[p] = *reinterpret_cast<const uint32_t*>(smem + GM::OFF_CT + (H + t - p - N1 + K) * CTROW +
                                                              (K - 1 - p) * S4 + 4 * g);
                else
                    W[p] = *reinterpret_cast<const uint32_t*>(smem + GM::OFF_OW + ((p - K) * kFR + t) * S4 + 4 * g);
            }
            const uint32_t ob = GM::OFF_RAW + t * F4 + 4 + 4 * g * N2;
            const int lim = N2 * min(4, S - 4 * g);  // run bytes that are blocks < S
#pragma unroll
            for (int q = 0; q < N2; ++q) {
                // byte y = 4q + x of the run: block y / N2, position y % N2 = byte (y / N2) of W[y % N2]
                const int y0 = 4 * q, y1 = 4 * q + 1, y2 = 4 * q + 2, y3 = 4 * q + 3;
                uint32_t val = gather4(W, 4 * (y0 % N2) + y0 / N2, 4 * (y1 % N2) + y1 / N2,
                                       4 * (y2 % N2) + y2 / N2, 4 * (y3 % N2) + y3 / N2);
                val &= keep_bytes(lim - 4 * q);  // the blocks' end: the tail's zeros from there
                if (4 + 4 * g * N2 + 4 * q + 4 <= F4) *reinterpret_cast<uint32_t*>(smem + ob + 4 * q) = val;
            }
            if (g == 0) *reinterpret_cast<uint32_t*>(smem + GM::OFF_RAW + t * F4) = uint32_t(size >> 8) | (uint32_t(size & 255) << 8);
            if (g == G - 1)  // the tail's zero dwords after the run
                for (int o = 4 + 4 * G * N2; o + 4 <= F4; o += 4) *reinterpret_cast<uint32_t*>(smem + GM::OFF_RAW + t * F4 + o) = 0;
        }
        __syncthreads();
        clk.mark(5);
        // re-pack rows of F4 to the frame stride F, 16 bytes per lane (t0*F is a multiple of 16); a
        // fixed number of buffer stores per lane
        const int obytes = nt * F;
        uint8_t* gout = a.out + t0 * F;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(gout, 0, obytes & ~15, 0x00020000);
#pragma unroll
        for (int qq = 0; qq < GM::SCH; ++qq) {
            asm volatile("" ::: "memory");  // one chunk's reads at a time (registers)
            const int w = T.tid + qq * kFT;
            const uint32_t b = 16 * w;
            uint32_t val[4] = {0, 0, 0, 0};
            if (static_cast<int>(b) < obytes) {
                int t = static_cast<int>(b / F);
                int o = static_cast<int>(b) - t * F;
#pragma unroll 1
                for (int q = 0; q < 4; ++q) {
                    const uint32_t s0 = GM::OFF_RAW + t * F4 + o;
                    const uint32_t d0 = *reinterpret_cast<const uint32_t*>(smem + (s0 & ~3u));
                    const uint32_t d1 = *reinterpret_cast<const uint32_t*>(smem + (s0 & ~3u) + 4);
                    uint32_t v = __builtin_amdgcn_alignbyte(d1, d0, s0 & 3u);
                    const int kk = F - o;  // bytes of frame t in this dword
                    if (kk < 4) {
                        const uint32_t e0 = *reinterpret_cast<const uint32_t*>(smem + GM::OFF_RAW + (t + 1) * F4);
                        v = (v & ((1u << (8 * kk)) - 1u)) | (e0 << (8 * kk));
                    }
                    val[0] = val[1];  // shifted in: val[3] is this dword after four
                    val[1] = val[2];
                    val[2] = val[3];
                    val[3] = v;
                    o += 4;
                    if (o >= F) {
                        o -= F;
                        ++t;
                    }
                }
            }
            const uint32_t so = static_cast<int>(b) + 16 <= obytes ? b : 0x7ffffff0u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(fec_v4u32, make_uint4(val[0], val[1], val[2], val[3])), ro, so, 0, 0);
            if (static_cast<int>(b) < obytes && static_cast<int>(b) + 16 > obytes)  // the output's ragged end
                for (int x = 0; static_cast<int>(b) + x < obytes; ++x) gout[b + x] = uint8_t(val[x >> 2] >> (8 * (x & 3)));
        }
        __syncthreads();
        clk.mark(6);
    }
    clk.flush(a.stamps);
}

// Relay, row scatter: frame t block j position p depends on one (decoded) row only, row
// t - p - n1 + k: its data symbols m of block j (p < k: symbol k-1-p; p >= k: XOR_m G2[k-1-m][p] *
// symbol m).  A lane per (row, group of 4 blocks) reads the row's 4*n1-byte span once (n1+1 dword
// reads + v_alignbyte), forms the k symbol words by v_perm, the n2-k parity words with the G2
// tables in scalar registers, and writes each position's 4 bytes straight into the frames of the
// tile, laid out in LDS at their own stride F (one base address, every byte at a compile-time
// offset); the frames then go out as 16-byte chunks.  Three barriers per tile.
template <class GM>
__global__ __launch_bounds__(GM::NT, GM::WPE) void fec_sw_fast_relay2_kernel(SwFastArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int K = GM::K, N1 = GM::N1, N2 = GM::N2, S = GM::S, G = GM::G, F = GM::F, TR = GM::TR;
    constexpr int size = (S + 1) * N2;
    constexpr int TAIL = F - 4 - S * N2;  // zero bytes after the blocks
    static_assert(GM::OFF_FR >= (N2 - 1) * F, "frame base addresses stay non-negative");
    FastTile<GM> T(smem, a);
    // the G2 tables are read with uniform, compile-time indices: scalar loads into SGPRs
    const auto* tab = (const __attribute__((address_space(4))) uint32_t*)(a.tab);
    __syncthreads();
    const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * a.tiles_per_wg;
    const int64_t tile1 = min(tile0 + a.tiles_per_wg, a.ntiles);
    PhaseClock clk(a.stamps != nullptr);
    if (tile0 < tile1) T.issue(tile0, false);
    for (int64_t tile = tile0; tile < tile1; ++tile) {
        const int64_t t0 = tile * TR;
        const int nt = static_cast<int>(min<int64_t>(TR, a.P - t0));
        clk.mark(0);
        T.land();
        T.masks(t0, nt);
        if (tile + 1 < tile1) T.issue(tile + 1, a.carry != 0);
        __syncthreads();
        clk.mark(1);
        T.decode();
        __syncthreads();
        if (a.carry && tile + 1 < tile1) T.keep();
        clk.mark(2);
        // rows k-1 .. k-1 + nt+n2-2 feed the tile's frames: row k-1+r, position p -> frame r-(n2-1)+p.
        // Interior rows (r in [n2-1, nt)) reach a frame of the tile at every position; with a full
        // group of 4 blocks their lanes write every byte without a test.  The other items -- the
        // n2-1 rows at each end of the span and the partial last group -- test each position.
        auto scatter = [&](int r, int g, auto checked) __attribute__((always_inline)) {
            constexpr bool CHK = decltype(checked)::value;
            const uint32_t sb = T.rowb(K - 1 + r) + 4 * g * N1;
            const uint32_t ab = sb & 0x1fffcu;
            uint32_t d[N1 + 1];
#pragma unroll
            for (int q = 0; q <= N1; ++q) d[q] = *reinterpret_cast<const uint32_t*>(smem + ab + 4 * q);
            align_words(d, static_cast<int>(sb & 3));
            uint32_t x[K], n0[K], n1[K], n2[K];  // symbol words and their 3-3-2 bit groups (gf_mul4x)
#pragma unroll
            for (int m = 0; m < K; ++m) {
                x[m] = gather4(d, m, N1 + m, 2 * N1 + m, 3 * N1 + m);
                n0[m] = x[m] & 0x07070707u;
                n1[m] = (x[m] >> 3) & 0x07070707u;
                n2[m] = (x[m] >> 6) & 0x03030303u;
            }
            const int tf = r - (N2 - 1);  // frame of position 0
            const uint32_t fb = static_cast<uint32_t>(GM::OFF_FR + tf * F + 4 + 4 * g * N2) & 0x1ffffu;
            const int nb = CHK ? min(4, S - 4 * g) : 4;
            tfor_sw<N2>([&](auto pc) __attribute__((always_inline)) {
                constexpr int p = decltype(pc)::value;
                const int t = tf + p;
                if (!CHK || (t >= 0 && t < nt)) {
                    uint32_t w;
                    if constexpr (p < K) {
                        w = x[K - 1 - p];
                    } else {
                        w = 0;
#pragma unroll
                        for (int m = 0; m < K; ++m) {
                            const int e = (p * K + m) * 5;
                            w ^= __builtin_amdgcn_perm(tab[e + 1], tab[e], n0[m]) ^
                                 __builtin_amdgcn_perm(tab[e + 3], tab[e + 2], n1[m]) ^
                                 __builtin_amdgcn_perm(tab[e + 4], tab[e + 4], n2[m]);
                        }
                    }
                    uint8_t* dst = smem + fb + p * (F + 1);
#ifdef FEC_RELAY2_ABLATE_WRITES  // diagnostic build only (wrong output): one byte write per position
                    dst[0] = static_cast<uint8_t>(w ^ (w >> 8) ^ (w >> 16) ^ (w >> 24));
#else
                    dst[0] = static_cast<uint8_t>(w);
                    if (!CHK || nb > 1) dst[N2] = static_cast<uint8_t>(w >> 8);
                    if (!CHK || nb > 2) dst[2 * N2] = static_cast<uint8_t>(w >> 16);
                    if (!CHK || nb > 3) dst[3 * N2] = static_cast<uint8_t>(w >> 24);
#endif
                }
            });
        };
        {
            constexpr int GF = S / 4;                      // full groups
            constexpr int GP = G - GF;                     // 0 or 1 partial group
            const int nint = max(0, nt - (N2 - 1));        // interior rows
            const int back0 = max(N2 - 1, nt);             // first row of the back end
            const int nback = nt + N2 - 1 - back0;
            const int n_int = nint * GF;
            const int n_all = n_int + (N2 - 1 + nback) * G + nint * GP;
            for (int it = T.tid; it < n_all; it += GM::NT) {
                if (it < n_int) {
                    const int r = N2 - 1 + it / GF, g = it - (it / GF) * GF;
                    scatter(r, g, std::false_type{});
                } else {
                    int i = it - n_int, r, g;
                    if (i < (N2 - 1) * G) {
                        r = i / G;
                        g = i - r * G;
                    } else if ((i -= (N2 - 1) * G) < nback * G) {
                        r = back0 + i / G;
                        g = i - (i / G) * G;
                    } else {
                        r = N2 - 1 + (i - nback * G);
                        g = GF;
                    }
                    scatter(r, g, std::true_type{});
                }
            }
        }
        // each frame's 4 header bytes (BE16 size, two zeros) and its zero tail
        for (int it = T.tid; it < nt * (4 + TAIL); it += GM::NT) {
            const int t = it / (4 + TAIL), b = it - t * (4 + TAIL);
            const uint8_t v = b == 0 ? uint8_t(size >> 8) : b == 1 ? uint8_t(size & 255) : uint8_t(0);
            smem[GM::OFF_FR + t * F + (b < 4 ? b : S * N2 + b)] = v;
        }
        __syncthreads();
        clk.mark(3);
        // the frames out, 16 bytes per lane (t0*F is a multiple of 16)
        const int obytes = nt * F;
        uint8_t* gout = a.out + t0 * F;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(gout, 0, obytes & ~15, 0x00020000);
#pragma unroll
        for (int qq = 0; qq < GM::SCH; ++qq) {
            const int c = T.tid + qq * GM::NT;
            const uint32_t b = 16 * c;
            if (static_cast<int>(b) >= obytes) break;
            const uint4 v = *reinterpret_cast<const uint4*>(smem + GM::OFF_FR + b);
            if (static_cast<int>(b) + 16 <= obytes) {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(fec_v4u32, v), ro, b, 0, 0);
            } else {  // the output's ragged end
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
                for (int x = 0; static_cast<int>(b) + x < obytes; ++x) gout[b + x] = uint8_t(vv[x >> 2] >> (8 * (x & 3)));
            }
        }
        clk.mark(4);
    }
    clk.flush(a.stamps);
}

}  // namespace fec

struct fec_swdf {
    fec_codec* hop1 = nullptr;  // Decoder(n1-1, n1-k, n1-k): the relay's decoder_current
    fec_codec* hop2 = nullptr;  // Encoder(n2-1, n2-k, n2-k) / the destination's decoder_current
    fec::CodecView v1, v2;
    int F = 0;
    int blocks = 0;  // ceil(max_payload / k) + 1 on ints (Decoder_Symbol_Wise.cpp:553, :632)
    uint32_t* d_tab = nullptr;  // v_perm tables of G2[k-1-m][p] for the specialised relay
    ~fec_swdf() {
        if (hop1) fec_codec_destroy(hop1);
        if (hop2) fec_codec_destroy(hop2);
        if (d_tab) (void)hipFree(d_tab);
    }
};

namespace {

int grid_for(int64_t items) {
    return static_cast<int>(std::min<int64_t>((items + fec::kSwThreads - 1) / fec::kSwThreads, 8192));
}

// The tiled kernel for k = K (template) when its LDS fits 64 KB; false = not launched (the
// per-(packet, block) kernels below run instead).
template <bool RELAY>
bool launch_tile(int K, fec::SwTileArgs a, hipStream_t s, hipError_t* err) {
    using fec::kTR;
    if (K < 1 || K > 16 || a.n > 17 || a.H > fec::kTMaxH || a.D0 + kTR > kTR + fec::kTMaxH) return false;
    if ((reinterpret_cast<uintptr_t>(a.out) & 15) != 0) return false;
    const int rows = kTR + a.H;
    const int tbb = RELAY ? a.n2 * K * 20 : 0;
    const int64_t ctb = static_cast<int64_t>(rows) * K * a.S4;
    // the slab plus slack for the CT build's reads past a row's last block (masked off)
    const int64_t rawb = std::max<int64_t>(16 + static_cast<int64_t>(rows) * a.in_stride + 4 * a.n + 4,
                                           int64_t(kTR) * a.out_row);
    if (16 + static_cast<int64_t>(rows) * a.in_stride > int64_t(16) * fec::kTThreads * fec::kTQ) return false;
    if ((reinterpret_cast<uintptr_t>(a.in) & 15) != 0) return false;
    a.off_rule = 1568 + 4 * (kTR + fec::kTMaxH);  // 4 waves x (K + K*17) u16
    a.off_tb = (a.off_rule + 4 * 2 * (16 + 16 * 17) + 15) & ~15;
    a.off_ct = (a.off_tb + tbb + 15) & ~15;
    a.off_raw = static_cast<int>((a.off_ct + ctb + 15) & ~int64_t(15));
    const int64_t lds = a.off_raw + ((rawb + 15) & ~int64_t(15));
    if (lds > 65536) return false;
    a.ntiles = (a.P + kTR - 1) / kTR;
    // one wave of resident workgroups (registers and LDS both limit them), each walking a
    // contiguous run of tiles
    auto launch = [&](auto kern) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, fec::kTThreads, static_cast<size_t>(lds)) !=
                hipSuccess || per_cu < 1)
            per_cu = 1;
        static const int cus = [] {
            int dev = 0, c = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1)
                c = 256;
            return c;
        }();
        const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(a.ntiles, int64_t(cus) * per_cu));
        a.tiles_per_wg = static_cast<int>((a.ntiles + grid - 1) / grid);
        const unsigned g = static_cast<unsigned>((a.ntiles + a.tiles_per_wg - 1) / a.tiles_per_wg);
        hipLaunchKernelGGL(kern, dim3(g), dim3(fec::kTThreads), static_cast<size_t>(lds), s, a);
        return g;
    };
    unsigned g = 0;
#define FEC_SW_TILE_CASE(KK)                                   \
    case KK:                                                   \
        g = launch(fec::fec_sw_tile_kernel<KK, RELAY>);        \
        break;
    switch (K) {
        FEC_SW_TILE_CASE(1) FEC_SW_TILE_CASE(2) FEC_SW_TILE_CASE(3) FEC_SW_TILE_CASE(4)
        FEC_SW_TILE_CASE(5) FEC_SW_TILE_CASE(6) FEC_SW_TILE_CASE(7) FEC_SW_TILE_CASE(8)
        FEC_SW_TILE_CASE(9) FEC_SW_TILE_CASE(10) FEC_SW_TILE_CASE(11) FEC_SW_TILE_CASE(12)
        FEC_SW_TILE_CASE(13) FEC_SW_TILE_CASE(14) FEC_SW_TILE_CASE(15) FEC_SW_TILE_CASE(16)
        default: return false;
    }
#undef FEC_SW_TILE_CASE
    *err = hipGetLastError();
    if (a.stamps && *err == hipSuccess) {
        // diagnostics: mean cycles per tile of each phase over the workgroups
        std::vector<uint64_t> h(static_cast<size_t>(g) * 8);
        *err = hipMemcpyAsync(h.data(), a.stamps, h.size() * 8, hipMemcpyDeviceToHost, s);
        if (*err == hipSuccess) *err = hipStreamSynchronize(s);
        double sum[5] = {0, 0, 0, 0, 0};
        for (unsigned b = 0; b < g; ++b)
            for (int k = 0; k < 5; ++k) sum[k] += static_cast<double>(h[b * 8 + k]);
        const double tiles = static_cast<double>(a.ntiles);
        std::fprintf(stderr,
                     "FEC_SWDF_STAMPS %s K=%d grid=%u tiles/wg=%d lds=%lld: cycles per tile: stage %.0f, masks+CT %.0f, "
                     "decode %.0f, output %.0f, store %.0f\n",
                     RELAY ? "relay" : "dest", K, g, a.tiles_per_wg, static_cast<long long>(lds), sum[0] / tiles,
                     sum[1] / tiles, sum[2] / tiles, sum[3] / tiles, sum[4] / tiles);
    }
    return true;
}

uint64_t* stamps_buffer() {  // FEC_SWDF_STAMPS set: a device buffer for the phase stamps
    static uint64_t* p = [] {
        uint64_t* q = nullptr;
        if (std::getenv("FEC_SWDF_STAMPS") && hipMalloc(&q, 8 * 8 * 65536) != hipSuccess) q = nullptr;
        if (q) (void)hipMemset(q, 0, 8 * 8 * 65536);
        return q;
    }();
    return p;
}

// The specialised kernels: n1 = n2 = 11 (T = 10, the T_TOT family of every adaptive tuple),
// k = 7..11, L = 300 (the reference's packet payload), every block relayed (blocks == S), input
// rows at the code's own width, 16-byte aligned input, 4-byte aligned output.
constexpr int kFastN = 11, kFastL = 300;

template <class GM>
bool launch_fast_geo(fec::SwFastArgs a, hipStream_t s, hipError_t* err) {
    constexpr int kFT = GM::NT;
    constexpr int kFR = GM::TR;
    auto kern = [] {
        if constexpr (GM::V2) return fec::fec_sw_fast_relay2_kernel<GM>;
        else if constexpr (GM::RELAY) return fec::fec_sw_fast_relay_kernel<GM>;
        else return fec::fec_sw_fast_dest_kernel<GM>;
    }();
    constexpr int lds = GM::LDS;
    if (lds > 160 * 1024) return false;
    static const bool attr_ok =
        lds <= 65536 || hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    if (!attr_ok) return false;
    static const int per_cu = [&] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, kFT, static_cast<size_t>(lds)) != hipSuccess || n < 1)
            n = 1;
        return n;
    }();
    static const int cus = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1)
            c = 256;
        return c;
    }();
    a.ntiles = (a.P + kFR - 1) / kFR;
    // one wave of resident workgroups, each walking a contiguous run of tiles
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(a.ntiles, int64_t(cus) * per_cu));
    a.tiles_per_wg = static_cast<int>((a.ntiles + grid - 1) / grid);
    const unsigned g = static_cast<unsigned>((a.ntiles + a.tiles_per_wg - 1) / a.tiles_per_wg);
    hipLaunchKernelGGL(kern, dim3(g), dim3(kFT), static_cast<size_t>(lds), s, a);
    *err = hipGetLastError();
    if (a.stamps && *err == hipSuccess) {
        std::vector<uint64_t> h(static_cast<size_t>(g) * 8);
        *err = hipMemcpyAsync(h.data(), a.stamps, h.size() * 8, hipMemcpyDeviceToHost, s);
        if (*err == hipSuccess) *err = hipStreamSynchronize(s);
        double sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (unsigned b = 0; b < g; ++b)
            for (int k = 0; k < 8; ++k) sum[k] += static_cast<double>(h[b * 8 + k]);
        const double tl = static_cast<double>(a.ntiles);
        std::fprintf(stderr,
                     "FEC_SWDF_STAMPS fast %s K=%d grid=%u tiles/wg=%d lds=%d: cycles per tile of %d: %s %.0f %.0f %.0f "
                     "%.0f %.0f %.0f\n",
                     GM::RELAY ? "relay" : "dest", GM::K, g, a.tiles_per_wg, lds, kFR,
                     GM::V2 ? "land+masks/decode/scatter/store" : GM::RELAY ? "land+masks/decode/CT/parity/words/store"
                                                                       : "land+masks/decode/out",
                     sum[0] / tl,
                     sum[1] / tl, sum[2] / tl, sum[3] / tl, sum[4] / tl, sum[5] / tl);
    }
    return true;
}

// The relay's kernel: the row scatter (default; tiles of 64 packets for k >= 7, of 32 / 16 for the
// longer rows of k = 5..6 / 4, 512 threads), or FEC_SWDF_RELAY=3 round 5's three-tile kernel (k >= 7,
// kept for A/B).
int relay_variant() {
    static const int v = [] {
        const char* r = std::getenv("FEC_SWDF_RELAY");
        return (r && r[0] == '3') ? 0 : 1;
    }();
    return v;
}

template <bool RELAY>
bool launch_fast(int K, fec::SwFastArgs a, int L, int n1, int n2, int blocks, int S, int64_t stride, hipStream_t s,
                 hipError_t* err) {
    if (L != kFastL || n2 != kFastN || (RELAY && n1 != kFastN) || blocks != S) return false;
    if ((reinterpret_cast<uintptr_t>(a.in) & 15) || (reinterpret_cast<uintptr_t>(a.out) & 3)) return false;
    const int rv = RELAY ? relay_variant() : 0;
#define FEC_SW_FAST_CASE(KK)                                                                      \
    case KK: {                                                                                    \
        using GM = fec::FastGeo<KK, kFastN, kFastN, kFastL, RELAY>;                                \
        if (stride != GM::STRIDE) return false;                                                   \
        if constexpr (RELAY) {                                                                    \
            if (rv) return launch_fast_geo<fec::FastGeo<KK, kFastN, kFastN, kFastL, true, (KK >= 7 ? 64 : KK >= 5 ? 32 : 16), true>>(a, s, err); \
            if constexpr (KK < 7) return false;                                                   \
            else return launch_fast_geo<GM>(a, s, err);                                           \
        } else {                                                                                  \
            return launch_fast_geo<GM>(a, s, err);                                                \
        }                                                                                         \
    }
    switch (K) {
        FEC_SW_FAST_CASE(4) FEC_SW_FAST_CASE(5) FEC_SW_FAST_CASE(6)
        FEC_SW_FAST_CASE(7) FEC_SW_FAST_CASE(8) FEC_SW_FAST_CASE(9) FEC_SW_FAST_CASE(10) FEC_SW_FAST_CASE(11)
        default: return false;
    }
#undef FEC_SW_FAST_CASE
}

bool fast_enabled() {
    static const bool on = [] {
        const char* v = std::getenv("FEC_SWDF_FAST");
        return !(v && v[0] == '0');
    }();
    return on;
}

// the specialised kernels carry a tile's front rows over from the workgroup's previous tile
// (FEC_SWDF_CARRY=0: every tile reloads them from HBM)
bool carry_enabled() {
    static const bool on = [] {
        const char* v = std::getenv("FEC_SWDF_CARRY");
        return !(v && v[0] == '0');
    }();
    return on;
}

bool tiles_enabled() {
    static const bool on = [] {
        const char* v = std::getenv("FEC_SWDF_TILE");
        return !(v && v[0] == '0');
    }();
    return on;
}

int launch_diag_decode(const fec::CodecView& v, int blocks, const uint8_t* in, int64_t in_stride, int in_off,
                       const uint8_t* er, int64_t P, uint8_t* out, int64_t out_stride, uint8_t* flag,
                       hipStream_t s) {
    fec::SwDecodeArgs a;
    a.in = in;
    a.in_stride = in_stride;
    a.in_off = in_off;
    a.er = er;
    a.P = P;
    a.k = v.k;
    a.n = v.n;
    a.S = v.S;
    a.blocks = blocks;
    if (v.wbase_n < 0) return FEC_ERR_ARG;  // n > 17: no window-n rule table
    a.rules = v.rules + v.wbase_n;
    a.ES = v.ES;
    a.gf = v.gf;
    a.out = out;
    a.out_stride = out_stride;
    a.flag = flag;
    hipLaunchKernelGGL(fec::fec_swdf_decode_kernel, dim3(grid_for(P * v.S)), dim3(fec::kSwThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // namespace

extern "C" {

int fec_swdf_create(int max_payload, int T1, int N1, int T2, int N2, fec_swdf** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    // n2 >= 2: a frame's (S+1)*n2 code bytes hold the 2 offset bytes and S blocks only then
    if (T1 < 0 || N1 < 0 || T2 < 1 || N2 < 0 || T1 - N1 != T2 - N2 || T1 - N1 + 1 < 1) return FEC_ERR_ARG;
    try {
        std::unique_ptr<fec_swdf> w(new fec_swdf());
        // Variable_Rate_FEC_Decoder.cpp:953-954 / :1608: Decoder(n-1, n-k, n-k), Encoder(n2-1,
        // n2-k2, n2-k2) with n = T+1, k = T-N+1 (Application_Layer_Receiver.cpp: n = T_value+1)
        if (int st = fec_codec_create(max_payload, T1, N1, N1, &w->hop1)) return st;
        if (int st = fec_codec_create(max_payload, T2, N2, N2, &w->hop2)) return st;
        fec::codec_view(w->hop1, &w->v1);
        fec::codec_view(w->hop2, &w->v2);
        if (w->v1.S != w->v2.S || w->v1.n > 32 || w->v2.n > 32) return FEC_ERR_ARG;
        w->F = 2 + (w->v1.S + 1) * w->v2.n;
        w->blocks = max_payload / w->v1.k + 1;
        *out = w.release();
        return FEC_OK;
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}

int fec_swdf_destroy(fec_swdf* w) {
    delete w;
    return FEC_OK;
}

int fec_swdf_geometry(const fec_swdf* w, int* k, int* n1, int* n2, int* S, int* frame_bytes, int* delay) {
    if (!w) return FEC_ERR_ARG;
    if (k) *k = w->v1.k;
    if (n1) *n1 = w->v1.n;
    if (n2) *n2 = w->v2.n;
    if (S) *S = w->v1.S;
    if (frame_bytes) *frame_bytes = w->F;
    if (delay) *delay = w->v1.n + w->v2.n - w->v1.k - 1;
    return FEC_OK;
}

size_t fec_swdf_workspace_bytes(const fec_swdf* w, int64_t P) {
    if (!w || P < 0) return 0;
    return static_cast<size_t>(P) * w->v1.S * w->v1.k;
}

int fec_swdf_relay_batch(fec_swdf* w, const uint8_t* d_cw, int64_t cw_stride, const uint8_t* d_erasure,
                         int64_t P, uint8_t* d_frames, uint8_t* d_flag, void* d_work, size_t work_bytes,
                         void* stream) {
    if (!w || P < 0) return FEC_ERR_ARG;
    if (P == 0) return FEC_OK;
    if (!d_cw || !d_erasure || !d_frames || cw_stride < w->v1.S * w->v1.n) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (fast_enabled() && w->v1.wbase_n >= 0) {
        if (!w->d_tab) {
            // v_perm tables of G2[k-1-m][p] (fec_device.h gf_mul4x): c*{0..7}, c*({0..7}<<3), c*({0..3}<<6)
            const int k = w->v2.k, n2 = w->v2.n;
            const std::vector<uint8_t> G2 = fec::make_generator(w->v2.T, w->v2.B, w->v2.N);
            const fec::Field& f = fec::field();
            std::vector<uint32_t> tab(static_cast<size_t>(n2) * k * 5, 0);
            for (int p = 0; p < n2; ++p)
                for (int m = 0; m < k; ++m) {
                    const uint8_t c = G2[(k - 1 - m) * n2 + p];
                    uint32_t* t = &tab[(static_cast<size_t>(p) * k + m) * 5];
                    for (int x = 0; x < 8; ++x) {
                        t[x >> 2] |= uint32_t(f.mt[c][x]) << (8 * (x & 3));
                        t[2 + (x >> 2)] |= uint32_t(f.mt[c][x << 3]) << (8 * (x & 3));
                    }
                    for (int x = 0; x < 4; ++x) t[4] |= uint32_t(f.mt[c][x << 6]) << (8 * x);
                }
            if (hipMalloc(&w->d_tab, tab.size() * 4) != hipSuccess) return FEC_ERR_NOMEM;
            FEC_HIP(hipMemcpy(w->d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
        }
        fec::SwFastArgs a{};
        a.carry = carry_enabled() ? 1 : 0;
        a.in = d_cw;
        a.er = d_erasure;
        a.P = P;
        a.rules = w->v1.rules + w->v1.wbase_n;
        a.gf = w->v1.gf;
        a.flag = d_flag;
        a.tab = w->d_tab;
        a.out = d_frames;
        a.stamps = stamps_buffer();
        hipError_t e = hipSuccess;
        if (launch_fast<true>(w->v1.k, a, w->v1.L, w->v1.n, w->v2.n, w->blocks, w->v1.S, cw_stride, s, &e))
            return e == hipSuccess ? FEC_OK : FEC_ERR_HIP;
    }
    if (tiles_enabled() && w->v1.wbase_n >= 0) {
        // decode + re-encode in one pass over the codewords (no workspace)
        fec::SwTileArgs a{};
        a.in = d_cw;
        a.in_stride = cw_stride;
        a.in_off = 0;
        a.er = d_erasure;
        a.P = P;
        a.n = w->v1.n;
        a.S = w->v1.S;
        a.S4 = (w->v1.S + 3) & ~3;
        a.blocks = w->blocks;
        a.H = w->v1.n + w->v2.n - 2;
        a.D0 = w->v2.n - 1;
        a.rules = w->v1.rules + w->v1.wbase_n;
        a.ES = w->v1.ES;
        a.gf = w->v1.gf;
        a.flag = d_flag;
        a.n2 = w->v2.n;
        a.G2 = w->v2.G;
        a.out = d_frames;
        a.out_row = w->F;
        a.stamps = stamps_buffer();
        hipError_t e = hipSuccess;
        if (launch_tile<true>(w->v1.k, a, s, &e)) return e == hipSuccess ? FEC_OK : FEC_ERR_HIP;
    }
    if (!d_work || work_bytes < fec_swdf_workspace_bytes(w, P)) return FEC_ERR_WORKSPACE;
    uint8_t* y = static_cast<uint8_t*>(d_work);
    const int Sk = w->v1.S * w->v1.k;
    if (int st = launch_diag_decode(w->v1, w->blocks, d_cw, cw_stride, 0, d_erasure, P, y, Sk, d_flag, s)) return st;
    fec::SwEncodeArgs a;
    a.y = y;
    a.P = P;
    a.k = w->v2.k;
    a.n2 = w->v2.n;
    a.S = w->v2.S;
    a.blocks = w->blocks;
    a.G2 = w->v2.G;
    a.gf = w->v2.gf;
    a.frames = d_frames;
    a.F = w->F;
    hipLaunchKernelGGL(fec::fec_swdf_encode_kernel, dim3(grid_for(P * a.S)), dim3(fec::kSwThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int fec_swdf_destination_batch(fec_swdf* w, const uint8_t* d_frames, const uint8_t* d_erasure, int64_t P,
                               uint8_t* d_out, uint8_t* d_flag, void* stream) {
    if (!w || P < 0) return FEC_ERR_ARG;
    if (P == 0) return FEC_OK;
    if (!d_frames || !d_erasure || !d_out) return FEC_ERR_ARG;
    // frame symbol (j, m) at byte 4 + j*n2 + m (size header + codeword_new_vector's offset 2)
    if (fast_enabled() && w->v2.wbase_n >= 0) {
        fec::SwFastArgs a{};
        a.carry = carry_enabled() ? 1 : 0;
        a.in = d_frames;
        a.er = d_erasure;
        a.P = P;
        a.rules = w->v2.rules + w->v2.wbase_n;
        a.gf = w->v2.gf;
        a.flag = d_flag;
        a.out = d_out;
        a.stamps = stamps_buffer();
        hipError_t e = hipSuccess;
        if (launch_fast<false>(w->v2.k, a, w->v2.L, w->v1.n, w->v2.n, w->blocks, w->v2.S, w->F,
                               static_cast<hipStream_t>(stream), &e))
            return e == hipSuccess ? FEC_OK : FEC_ERR_HIP;
    }
    if (tiles_enabled() && w->v2.wbase_n >= 0) {
        fec::SwTileArgs a{};
        a.in = d_frames;
        a.in_stride = w->F;
        a.in_off = 4;
        a.er = d_erasure;
        a.P = P;
        a.n = w->v2.n;
        a.S = w->v2.S;
        a.S4 = (w->v2.S + 3) & ~3;
        a.blocks = w->blocks;
        a.H = w->v2.n - 1;
        a.D0 = 0;
        a.rules = w->v2.rules + w->v2.wbase_n;
        a.ES = w->v2.ES;
        a.gf = w->v2.gf;
        a.flag = d_flag;
        a.out = d_out;
        a.out_row = w->v2.S * w->v2.k;
        a.stamps = stamps_buffer();
        hipError_t e = hipSuccess;
        if (launch_tile<false>(w->v2.k, a, static_cast<hipStream_t>(stream), &e))
            return e == hipSuccess ? FEC_OK : FEC_ERR_HIP;
    }
    return launch_diag_decode(w->v2, w->blocks, d_frames, w->F, 4, d_erasure, P, d_out, w->v2.S * w->v2.k, d_flag,
                              static_cast<hipStream_t>(stream));
}

}  // extern "C"
