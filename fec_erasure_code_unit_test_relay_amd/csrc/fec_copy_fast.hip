// fec_copy_fast.hip -- decode of received packets, specialised at compile time on k and n-k.
//
// The reference outputs a received packet's systematic bytes (fast path, Decoder.cpp:77-108; the
// slow path returns the same bytes for received packets).  In the codeword each sub-stream s is
// [k systematic | n-k parity]; the payload is the systematic bytes with the 2-byte length header
// removed.  One lane per (packet, group of 4 sub-streams): the group's 4n codeword bytes are read
// from the LDS tile as dwords, the 4k systematic bytes are picked with constant-selector
// v_perm_b32, shifted by the header's 2 bytes and written to the LDS output tile (one 16-bit
// store at each end, dwords in between).  Tiles move between HBM and LDS with 16-byte accesses.
#include "fec_device.h"
#include "fec_kernels.h"

namespace fec {

#ifndef FEC_COPY_STAGE_BATCH
#define FEC_COPY_STAGE_BATCH 8  // 16-byte loads in flight per thread while staging the tile
#endif

template <int K, int NP>
__global__ __launch_bounds__(256) void fec_copy_fast_kernel(CopyFastArgs a) {
    constexpr int n = K + NP;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* raw = smem;                           // codeword tile (+ slack)
    uint8_t* xo = smem + a.raw_bytes;              // payload tile
    int32_t* clen = reinterpret_cast<int32_t*>(xo + a.out_bytes);  // bytes to copy per packet
    uint8_t* erw = reinterpret_cast<uint8_t*>(clen + a.TP);         // erasure flags [x0, x0+TP+T)

    const int tid = threadIdx.x, NT = blockDim.x;
    phase_stamp(a.stamps, blockIdx.x, 0);
    const int L = a.L, CW = a.CW, NS4 = a.NS4, T = a.T;
    const int64_t x0 = static_cast<int64_t>(blockIdx.x) * a.TP;
    const int ntile = static_cast<int>(min<int64_t>(a.TP, a.Pout - x0));

    const uint8_t* gA = a.cw + x0 * CW;
    const int delta = static_cast<int>(reinterpret_cast<uintptr_t>(gA) & 15);
    if (a.nt)
        stage_to_lds<FEC_COPY_STAGE_BATCH, true>(raw, gA - delta, delta, delta + ntile * CW, tid, NT);
    else
        stage_to_lds<FEC_COPY_STAGE_BATCH>(raw, gA - delta, delta, delta + ntile * CW, tid, NT);
    for (int i = tid; i < ntile + T; i += NT) erw[i] = a.er[x0 + i];  // x0+ntile+T-1 < P
    __syncthreads();
    phase_stamp(a.stamps, blockIdx.x, 1);

    for (int t = tid; t < ntile; t += NT) {
        int ln = 0, copy = 0;
        if (!erw[t]) {
            const uint8_t* row = raw + delta + t * CW;
            // header bytes h = 0, 1: sub-stream 0 position 0 and h=1 -> (1/k)*n + 1%k
            const int hdr = row[0] * 256 + row[(1 / K) * n + 1 % K];
            bool slow = false;
            for (int d = 0; d <= T; ++d) slow = slow || erw[t + d];
            ln = slow ? min(hdr, L) : hdr;  // Decoder.cpp:148-149 clamps in the slow path only
            copy = min(ln, L);
        }
        clen[t] = copy;
        if (!(a.skip_erased && erw[t])) a.out_len[x0 + t] = ln;
    }
    __syncthreads();

    for (int it = tid; it < ntile * NS4; it += NT) {
        const int g = it / ntile;
        const int t = it - g * ntile;
        const int cl = clen[t];
        uint32_t W[K + 1];  // systematic bytes of the group: byte e*K+i = position i of sub-stream 4g+e
        if (cl > 0) {
            const int off = delta + t * CW + 4 * n * g;
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
                W[m] = gather4(S, (i0 / K) * n + i0 % K, (i1 / K) * n + i1 % K,
                               (i2 / K) * n + i2 % K, (i3 / K) * n + i3 % K);
            }
        } else {
#pragma unroll
            for (int m = 0; m < K; ++m) W[m] = 0;
        }
        W[K] = 0;
        // payload bytes b in [4gK-2, 4gK+4K-2): head (2 bytes), K-1 dwords, tail (2 bytes)
        uint8_t* orow = xo + t * L;
        const int bh = 4 * g * K - 2;
        if (bh >= 0 && bh < L) {
            const uint32_t v = W[0] & keep_bytes(cl - bh);
            *reinterpret_cast<uint16_t*>(orow + bh) = static_cast<uint16_t>(v);
        }
#pragma unroll
        for (int m = 0; m < K - 1; ++m) {
            const int b = 4 * g * K + 4 * m;
            if (b < L) {
                const uint32_t v = __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & keep_bytes(cl - b);
                *reinterpret_cast<uint32_t*>(orow + b) = v;
            }
        }
        const int bt = 4 * g * K + 4 * K - 4;
        if (bt < L) {
            const uint32_t v = (W[K - 1] >> 16) & keep_bytes(cl - bt);
            *reinterpret_cast<uint16_t*>(orow + bt) = static_cast<uint16_t>(v);
        }
    }
    __syncthreads();
    phase_stamp(a.stamps, blockIdx.x, 2);

    // With skip_erased the rows of erased packets are left to fec_recover_kernel (running
    // concurrently): a chunk touching one goes out dword by dword (L % 4 == 0: a dword never
    // straddles two rows).
    const int obytes = ntile * L;
    uint8_t* dst = a.out + x0 * L;
    const bool skip = a.skip_erased != 0;
    if ((obytes & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (int o = tid * 16; o < obytes; o += NT * 16) {
            if (!skip || (!erw[o / L] && !erw[(o + 15) / L])) {
                const uint4 v = *reinterpret_cast<const uint4*>(xo + o);
                if (a.nt)
                    nt_store16(dst + o, v);
                else
                    *reinterpret_cast<uint4*>(dst + o) = v;
            } else {
#pragma unroll
                for (int q = 0; q < 16; q += 4)
                    if (!erw[(o + q) / L])
                        *reinterpret_cast<uint32_t*>(dst + o + q) = *reinterpret_cast<const uint32_t*>(xo + o + q);
            }
        }
    } else {
        for (int o = tid * 4; o < obytes; o += NT * 4)
            if (!skip || !erw[o / L])
                *reinterpret_cast<uint32_t*>(dst + o) = *reinterpret_cast<const uint32_t*>(xo + o);
    }
    phase_stamp(a.stamps, blockIdx.x, 3);
}

// Two consecutive tiles per workgroup (FEC_COPY_PAIR=1): the second tile's codeword chunks are
// loaded into registers while the first tile is converted and stored, then written to the same LDS
// stage -- twice the loads in flight per workgroup at the same LDS.
template <int K, int NP>
__device__ __forceinline__ void copy_tile_convert(const CopyFastArgs& a, int64_t x0, int ntile, int delta,
                                                  const uint8_t* raw, uint8_t* xo, int32_t* clen, const uint8_t* erw) {
    constexpr int n = K + NP;
    const int tid = threadIdx.x, NT = blockDim.x;
    const int L = a.L, CW = a.CW, NS4 = a.NS4, T = a.T;
    for (int t = tid; t < ntile; t += NT) {
        int ln = 0, copy = 0;
        if (!erw[t]) {
            const uint8_t* row = raw + delta + t * CW;
            const int hdr = row[0] * 256 + row[(1 / K) * n + 1 % K];
            bool slow = false;
            for (int d = 0; d <= T; ++d) slow = slow || erw[t + d];
            ln = slow ? min(hdr, L) : hdr;
            copy = min(ln, L);
        }
        clen[t] = copy;
        if (!(a.skip_erased && erw[t])) a.out_len[x0 + t] = ln;
    }
    __syncthreads();
    for (int it = tid; it < ntile * NS4; it += NT) {
        const int g = it / ntile;
        const int t = it - g * ntile;
        const int cl = clen[t];
        uint32_t W[K + 1];
        if (cl > 0) {
            const int off = delta + t * CW + 4 * n * g;
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
        uint8_t* orow = xo + t * L;
        const int bh = 4 * g * K - 2;
        if (bh >= 0 && bh < L) *reinterpret_cast<uint16_t*>(orow + bh) = static_cast<uint16_t>(W[0] & keep_bytes(cl - bh));
#pragma unroll
        for (int m = 0; m < K - 1; ++m) {
            const int b = 4 * g * K + 4 * m;
            if (b < L) *reinterpret_cast<uint32_t*>(orow + b) = __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & keep_bytes(cl - b);
        }
        const int bt = 4 * g * K + 4 * K - 4;
        if (bt < L) *reinterpret_cast<uint16_t*>(orow + bt) = static_cast<uint16_t>((W[K - 1] >> 16) & keep_bytes(cl - bt));
    }
    __syncthreads();
    const int obytes = ntile * L;
    uint8_t* dst = a.out + x0 * L;
    const bool skip = a.skip_erased != 0;
    if ((obytes & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (int o = tid * 16; o < obytes; o += NT * 16) {
            if (!skip || (!erw[o / L] && !erw[(o + 15) / L])) {
                const uint4 v = *reinterpret_cast<const uint4*>(xo + o);
                if (a.nt) nt_store16(dst + o, v);
                else *reinterpret_cast<uint4*>(dst + o) = v;
            } else {
#pragma unroll
                for (int q = 0; q < 16; q += 4)
                    if (!erw[(o + q) / L]) *reinterpret_cast<uint32_t*>(dst + o + q) = *reinterpret_cast<const uint32_t*>(xo + o + q);
            }
        }
    } else {
        for (int o = tid * 4; o < obytes; o += NT * 4)
            if (!skip || !erw[o / L]) *reinterpret_cast<uint32_t*>(dst + o) = *reinterpret_cast<const uint32_t*>(xo + o);
    }
}

constexpr int kPairQ = 6;  // 16-byte chunks per thread a tile's stage may take (6 * 16 * 256 = 24 KB)

template <int K, int NP>
__global__ __launch_bounds__(256) void fec_copy_pair_kernel(CopyFastArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* raw = smem;
    uint8_t* xo = smem + a.raw_bytes;
    int32_t* clen = reinterpret_cast<int32_t*>(xo + a.out_bytes);
    uint8_t* erw = reinterpret_cast<uint8_t*>(clen + a.TP);
    const int tid = threadIdx.x;
    const int CW = a.CW, T = a.T;
    uint4 v[kPairQ];
    auto load = [&](int64_t x0, int ntile, int delta) __attribute__((always_inline)) {
        const uint8_t* gA = a.cw + x0 * CW - delta;
        const int total = delta + ntile * CW;
#pragma unroll
        for (int q = 0; q < kPairQ; ++q) {
            const int lo = (q * 256 + tid) << 4;
            const bool full = lo >= delta && lo + 16 <= total;
            v[q] = full ? nt_load16(gA + lo) : make_uint4(0, 0, 0, 0);
        }
    };
    auto land = [&](int64_t x0, int ntile, int delta) __attribute__((always_inline)) {
        const uint8_t* gA = a.cw + x0 * CW - delta;
        const int total = delta + ntile * CW;
#pragma unroll
        for (int q = 0; q < kPairQ; ++q) {
            const int lo = (q * 256 + tid) << 4;
            if (lo >= delta && lo + 16 <= total) *reinterpret_cast<uint4*>(raw + lo) = v[q];
        }
        if (tid == 0) {  // edge bytes / dwords, as stage_to_lds
            for (int b = delta; b < total && (b & 3); ++b) raw[b] = gA[b];
            for (int b = total & ~3; b < total && b >= ((delta + 3) & ~3); ++b) raw[b] = gA[b];
        }
        for (int o = tid * 4; o < 32; o += 256 * 4) {
            const int lo16 = delta & ~15, hi16 = total & ~15;
            const int oa = lo16 + o, ob = hi16 + (o - 16);
            if (o < 16 && oa >= delta && oa + 4 <= total && !(lo16 >= delta && lo16 + 16 <= total))
                *reinterpret_cast<uint32_t*>(raw + oa) = *reinterpret_cast<const uint32_t*>(gA + oa);
            if (o >= 16 && ob >= delta && ob + 4 <= total && hi16 != lo16)
                *reinterpret_cast<uint32_t*>(raw + ob) = *reinterpret_cast<const uint32_t*>(gA + ob);
        }
        for (int i = tid; i < ntile + T; i += 256) erw[i] = a.er[x0 + i];
    };
    // two consecutive tiles, straight-line code (a run-time loop over the workgroup's tiles measured
    // slower: copy 170 vs 144 us, and an unrolled loop for 2 / 3 / 4 tiles 145 / 149 / 155 us;
    // profiles/r05/headline/r05zt_*, r05zv_*)
    const int64_t xa = static_cast<int64_t>(blockIdx.x) * 2 * a.TP, xb = xa + a.TP;
    const int na = static_cast<int>(min<int64_t>(a.TP, a.Pout - xa));
    const int nb = static_cast<int>(max<int64_t>(0, min<int64_t>(a.TP, a.Pout - xb)));
    const int da = static_cast<int>(reinterpret_cast<uintptr_t>(a.cw + xa * CW) & 15);
    const int db = static_cast<int>(reinterpret_cast<uintptr_t>(a.cw + xb * CW) & 15);
    load(xa, na, da);
    land(xa, na, da);
    __syncthreads();
    if (nb > 0) load(xb, nb, db);  // in flight while tile A is converted and stored
    copy_tile_convert<K, NP>(a, xa, na, da, raw, xo, clen, erw);
    if (nb <= 0) return;
    __syncthreads();  // tile A's stage, lengths and flags are read
    land(xb, nb, db);
    __syncthreads();
    copy_tile_convert<K, NP>(a, xb, nb, db, raw, xo, clen, erw);
}

const void* fec_copy_pair_kernel_for(int k, int np);

#define FEC_COPY_FAST_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(1, 10) X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)

#define FEC_COPY_FAST_INST(K, NP) \
    template __global__ void fec_copy_fast_kernel<K, NP>(CopyFastArgs); \
    template __global__ void fec_copy_pair_kernel<K, NP>(CopyFastArgs);
FEC_COPY_FAST_LIST(FEC_COPY_FAST_INST)

const void* fec_copy_pair_kernel_for(int k, int np) {
#define FEC_COPY_PAIR_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_copy_pair_kernel<K, NP>);
    FEC_COPY_FAST_LIST(FEC_COPY_PAIR_CASE)
#undef FEC_COPY_PAIR_CASE
    return nullptr;
}

const void* fec_copy_fast_kernel_for(int k, int np) {
#define FEC_COPY_FAST_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_copy_fast_kernel<K, NP>);
    FEC_COPY_FAST_LIST(FEC_COPY_FAST_CASE)
#undef FEC_COPY_FAST_CASE
    return nullptr;
}

}  // namespace fec
