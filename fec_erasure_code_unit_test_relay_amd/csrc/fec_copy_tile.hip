// fec_copy_tile.hip -- decode of received packets over contiguous per-workgroup runs of tiles.
//
// Same output as fec_copy_fast_kernel (the reference's fast path, Decoder.cpp:77-108, and the slow
// path's received packets, which output their systematic bytes unchanged; the length header is
// clamped to max_payload in the slow path only, Decoder.cpp:148-149): for every packet x < Pout,
// row x = bytes 2 .. 2+len of [sub-stream s: k systematic bytes] over s, zero beyond, and
// out_len[x] = len, or 0 / a zero row for an erased packet (fec_recover_kernel overwrites the
// recovered ones afterwards).
//
// Organisation: a workgroup walks a contiguous run of TP-packet tiles.  The next tile's codewords
// (one contiguous TP*CW-byte slab, 16-byte aligned) and erasure flags are loaded into registers
// while the current tile is converted and stored, and written to LDS at the top of the next
// iteration; two barriers per tile.  Item (packet p, group g of 4 sub-streams) picks its 4K
// systematic bytes out of the group's 4n codeword bytes with constant-selector v_perm_b32,
// shifts out the 2-byte header and writes the payload dwords into the LDS output tile, which
// leaves as 16-byte stores.  The slow-path clamp of packet p needs the erasure flags of
// [p, p+T]: every wave holds the tile's TP+T flags as one 64-bit ballot.
#include "fec_device.h"
#include "fec_kernels.h"

namespace fec {
namespace {
constexpr int kCopyThreads = 256;
constexpr int kCopyStage = 4;  // 16-byte codeword pieces per thread per tile (TP*CW <= 16 KB)
}  // namespace

template <int K, int NP>
__global__ __launch_bounds__(kCopyThreads) void fec_copy_tile_kernel(CopyTileArgs a) {
    constexpr int n = K + NP;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int L = a.L, CW = a.CW, NS4 = a.NS4, T = a.T, TP = a.TP;
    uint8_t* raw = smem;                          // TP*CW codeword bytes (+ 64 slack)
    uint8_t* xo = smem + a.raw_bytes;             // TP*L payload bytes
    const int64_t first = static_cast<int64_t>(blockIdx.x) * a.tiles_per_wg;
    const int64_t last = min<int64_t>(first + a.tiles_per_wg, a.ntiles);
    if (first >= last) return;

    uint4 st[kCopyStage];
    uint32_t stf = 0;  // erasure flag of packet x0 + lane (lane < TP + T)
    auto load = [&](int64_t tile) __attribute__((always_inline)) {
        const int64_t x0 = tile * TP;
        const int ntile = static_cast<int>(min<int64_t>(TP, a.Pout - x0));
        const int bytes = ntile * CW;
        const uint4* src = reinterpret_cast<const uint4*>(a.cw + x0 * CW);
#pragma unroll
        for (int j = 0; j < kCopyStage; ++j) {
            const int c = tid + j * kCopyThreads;
            st[j] = (c * 16 + 16 <= bytes) ? src[c] : make_uint4(0, 0, 0, 0);
        }
        stf = (lane < ntile + T) ? a.er[x0 + lane] : 0;  // every wave: the tile's TP+T flags
    };
    load(first);
    for (int64_t tile = first; tile < last; ++tile) {
        const int64_t x0 = tile * TP;
        const int ntile = static_cast<int>(min<int64_t>(TP, a.Pout - x0));
        const int bytes = ntile * CW;
        // staged tile -> LDS
#pragma unroll
        for (int j = 0; j < kCopyStage; ++j) {
            const int c = tid + j * kCopyThreads;
            if (c * 16 < bytes) reinterpret_cast<uint4*>(raw)[c] = st[j];
        }
        if ((bytes & 15) && tid < 4) {  // last partial piece: its whole dwords (then bytes)
            const int b0 = (bytes & ~15) + 4 * tid;
            if (b0 + 4 <= bytes)
                *reinterpret_cast<uint32_t*>(raw + b0) = *reinterpret_cast<const uint32_t*>(a.cw + x0 * CW + b0);
            else
                for (int b = b0; b < bytes; ++b) raw[b] = a.cw[x0 * CW + b];
        }
        const uint32_t myflag = stf;
        __syncthreads();
        if (tile + 1 < last) load(tile + 1);  // in flight while this tile is converted and stored

        // erasure flags of packets x0 .. x0+TP+T-1 of this tile, one bit each
        const uint64_t emask = __builtin_amdgcn_ballot_w64(lane < TP + T && myflag != 0);
        const uint64_t fmask = (T + 1 >= 64) ? ~0ull : ((1ull << (T + 1)) - 1);

        for (int it = tid; it < ntile * NS4; it += kCopyThreads) {
            const int t = it / NS4;
            const int g = it - t * NS4;
            const bool erased = (emask >> t) & 1ull;
            const bool slow = ((emask >> t) & fmask) != 0;
            const uint8_t* row = raw + t * CW;
            int cl = 0, ln = 0;
            if (!erased) {
                const int hdr = row[0] * 256 + row[(1 / K) * n + 1 % K];
                ln = slow ? min(hdr, L) : hdr;
                cl = min(ln, L);
            }
            if (g == 0) a.out_len[x0 + t] = ln;
            uint32_t W[K + 1];
            if (cl > 0) {
                const int off = t * CW + 4 * n * g;
                const int a4 = off & ~3;
                uint32_t D[n + 1];
#pragma unroll
                for (int m = 0; m <= n; ++m) D[m] = *reinterpret_cast<const uint32_t*>(raw + a4 + 4 * m);
                uint32_t S[n];
#pragma unroll
                for (int m = 0; m < n; ++m) S[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], off & 3);
#pragma unroll
                for (int m = 0; m < K; ++m) {
                    const int i0 = 4 * m, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3;
                    W[m] = gather4(S, (i0 / K) * n + i0 % K, (i1 / K) * n + i1 % K, (i2 / K) * n + i2 % K,
                                   (i3 / K) * n + i3 % K);
                }
            } else {
#pragma unroll
                for (int m = 0; m < K; ++m) W[m] = 0;
            }
            W[K] = 0;
            // payload bytes b in [4gK-2, 4gK+4K-2): head (2 bytes), K-1 dwords, tail (2 bytes)
            uint8_t* orow = xo + t * L;
            const int bh = 4 * g * K - 2;
            if (bh >= 0 && bh < L)
                *reinterpret_cast<uint16_t*>(orow + bh) = static_cast<uint16_t>(W[0] & keep_bytes(cl - bh));
#pragma unroll
            for (int m = 0; m < K - 1; ++m) {
                const int b = 4 * g * K + 4 * m;
                if (b < L)
                    *reinterpret_cast<uint32_t*>(orow + b) =
                        __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & keep_bytes(cl - b);
            }
            const int bt = 4 * g * K + 4 * K - 4;
            if (bt < L)
                *reinterpret_cast<uint16_t*>(orow + bt) = static_cast<uint16_t>((W[K - 1] >> 16) & keep_bytes(cl - bt));
        }
        __syncthreads();
        // output tile -> HBM: ntile*L bytes at x0*L (16-byte aligned: TP*L % 16 == 0)
        const int ob = ntile * L;
        uint8_t* dst = a.out + x0 * L;
        for (int o = tid * 16; o < ob; o += kCopyThreads * 16) {
            if (o + 16 <= ob) {
                *reinterpret_cast<uint4*>(dst + o) = *reinterpret_cast<const uint4*>(xo + o);
            } else {
                for (int q = o; q < ob; q += 4)
                    *reinterpret_cast<uint32_t*>(dst + q) = *reinterpret_cast<const uint32_t*>(xo + q);
            }
        }
    }
}

#define FEC_COPY_TILE_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(1, 10) X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)

#define FEC_COPY_TILE_INST(K, NP) template __global__ void fec_copy_tile_kernel<K, NP>(CopyTileArgs);
FEC_COPY_TILE_LIST(FEC_COPY_TILE_INST)

const void* fec_copy_tile_kernel_for(int k, int np) {
#define FEC_COPY_TILE_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_copy_tile_kernel<K, NP>);
    FEC_COPY_TILE_LIST(FEC_COPY_TILE_CASE)
#undef FEC_COPY_TILE_CASE
    return nullptr;
}

}  // namespace fec
