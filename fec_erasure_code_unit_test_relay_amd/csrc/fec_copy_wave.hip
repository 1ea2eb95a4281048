// fec_copy_wave.hip -- decode of received packets without LDS staging or barriers, specialised
// on (k, n-k).
//
// The reference outputs a received packet's systematic bytes (fast path, Decoder.cpp:77-108; the
// slow path returns the same bytes for received packets, its length clamped to max_payload,
// :148-149).  In the codeword each sub-stream s is [k systematic | n-k parity]; the payload is the
// systematic bytes with the 2-byte length header removed.
//
// A wave walks a contiguous run of packets, SPW = 64 / NS4 packets per step, one lane per (packet,
// group g of 4 sub-streams), the next step's loads issued before the current step is converted:
//   * the lane's 4n codeword bytes come straight from HBM (buffer loads of n+1 dwords from the
//     dword below, realigned with v_alignbyte; reads past the batch come back as zero);
//   * the 4k systematic bytes are picked with constant-selector v_perm_b32 (gather4), shifted by
//     the header's 2 bytes: output dword m of the group = bytes 2.. of word m, plus the first two
//     bytes of the next group's (ds_bpermute from lane + 1), so every lane stores k whole dwords of
//     its own row -- payload rows are dword aligned (max_payload % 4 == 0) and no store touches
//     another packet's row;
//   * the packet's length (header bytes, slow-path clamp from the erasure flags x..x+T) is formed
//     on lane g = 0 and broadcast; erased packets are skipped entirely (fec_recover_kernel writes
//     their rows), so this kernel can run concurrently with the recovery.
#include "fec_device.h"
#include "fec_kernels.h"

namespace fec {
namespace {

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x3a __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef uint32_t v3u32 __attribute__((ext_vector_type(3)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

// NW consecutive dwords at byte offset o (dword aligned) of resource rs
template <int NW>
__device__ __forceinline__ void load_words(uint32_t (&D)[NW], __amdgpu_buffer_rsrc_t rs, int o) {
#pragma unroll
    for (int c = 0; c < NW; c += 4) {
        if (c + 4 <= NW) {
            const u32x4a v = __builtin_bit_cast(u32x4a, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 4 * c, 0, 0));
            D[c] = v.x;
            D[c + 1] = v.y;
            D[c + 2] = v.z;
            D[c + 3] = v.w;
        } else if (c + 3 == NW) {
            const u32x3a v = __builtin_bit_cast(u32x3a, __builtin_amdgcn_raw_buffer_load_b96(rs, o + 4 * c, 0, 0));
            D[c] = v.x;
            D[c + 1] = v.y;
            D[c + 2] = v.z;
        } else if (c + 2 == NW) {
            const u32x2a v = __builtin_bit_cast(u32x2a, __builtin_amdgcn_raw_buffer_load_b64(rs, o + 4 * c, 0, 0));
            D[c] = v.x;
            D[c + 1] = v.y;
        } else {
            D[c] = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4 * c, 0, 0);
        }
    }
}

// W[0..cnt) (cnt <= NW, cnt wave-divergent) as dwords at byte offset o (dword aligned)
template <int NW>
__device__ __forceinline__ void store_words_n(__amdgpu_buffer_rsrc_t rc, int o, const uint32_t (&W)[NW], int cnt) {
    if (cnt >= NW) {
#pragma unroll
        for (int c = 0; c < NW; c += 4) {
            if (c + 4 <= NW) {
                u32x4a v = {W[c], W[c + 1], W[c + 2], W[c + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), rc, o + 4 * c, 0, 0);
            } else if (c + 3 == NW) {
                u32x3a v = {W[c], W[c + 1], W[c + 2]};
                __builtin_amdgcn_raw_buffer_store_b96(__builtin_bit_cast(v3u32, v), rc, o + 4 * c, 0, 0);
            } else if (c + 2 == NW) {
                u32x2a v = {W[c], W[c + 1]};
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, v), rc, o + 4 * c, 0, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(W[c], rc, o + 4 * c, 0, 0);
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < NW; ++q)
            if (q < cnt) __builtin_amdgcn_raw_buffer_store_b32(W[q], rc, o + 4 * q, 0, 0);
    }
}

}  // namespace

template <int K, int NP>
__global__ __launch_bounds__(256) void fec_copy_wave_kernel(CopyWaveArgs a) {
    constexpr int n = K + NP;
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NS4 = a.NS4, SPW = a.SPW, L = a.L, CW = a.CW, T = a.T;
    const int p = lane / NS4;
    const int g = lane - p * NS4;
    const bool live_lane = p < SPW;
    const int64_t step0 = static_cast<int64_t>(wave) * a.steps_per_wave;
    const int64_t step_end = min<int64_t>(step0 + a.steps_per_wave, a.nsteps);
    if (step0 >= step_end) return;

    // resources: codewords [0, P*CW), erasure flags [0, P), payload rows [0, Pout*L)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.cw), 0, a.cw_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
    const int rowdw = L >> 2;                       // payload dwords per row
    const int ndw = min(K, rowdw - K * g);          // this group's output dwords (<= 0: none)
    const int right = (g + 1 < NS4) ? lane + 1 : lane;  // the next group of the same packet
    const uint64_t pmask = ((NS4 >= 64) ? ~0ull : ((1ull << NS4) - 1ull)) << (p < SPW ? p * NS4 : 0);

    // Everything a step needs from memory -- the codeword words and the erasure flags x..x+T (4
    // per lane at most: T < 4*NS4, host check) -- is loaded one step ahead: vmcnt waits are in
    // issue order, so a load issued after the prefetch would wait for the prefetch too.
    const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.er), 0, a.er_bytes, 0x00020000);
    uint32_t D[n + 1];
    uint32_t E[4];
    auto issue = [&](int64_t step) __attribute__((always_inline)) {
        const int64_t x = step * SPW + p;
        const int o = static_cast<int>(x * CW) + 4 * n * g;
        load_words<n + 1>(D, rs, o & ~3);
        const bool pv = live_lane && x < a.Pout;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = g + j * NS4;
            // past T (or an invalid lane): an offset beyond the resource, which reads as zero
            const int eo = (pv && d <= T) ? static_cast<int>(x) + d : a.er_bytes;
            E[j] = __builtin_amdgcn_raw_buffer_load_b8(re, eo, 0, 0);
        }
    };
    issue(step0);
    for (int64_t step = step0; step < step_end; ++step) {
        const int64_t x = step * SPW + p;
        const bool valid = live_lane && x < a.Pout;
        const int sh = static_cast<int>((x * CW + 4 * n * g) & 3);
        uint32_t S[n];
#pragma unroll
        for (int m = 0; m < n; ++m) S[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], sh);
        // erasure flags x..x+T of the packet, spread over its lanes; x+T < P for x < Pout
        const bool own = g == 0 && E[0] != 0;
        const bool any = (E[0] | E[1] | E[2] | E[3]) != 0;
        if (step + 1 < step_end) issue(step + 1);
        const uint64_t bal_any = __ballot(any);
        const uint64_t bal_own = __ballot(own);
        const bool erased = (bal_own & pmask) != 0;
        const bool slow = (bal_any & pmask) != 0;
        // header bytes 0, 1 of data_with_header: sub-stream 0 position 0, and position 1 (k > 1) or
        // sub-stream 1 position 0 (k = 1) -- group 0's bytes 0 and (1/k)*n + 1%k
        constexpr int h1 = (1 / K) * n + 1 % K;
        const int hdr0 = static_cast<int>(S[0] & 0xff) * 256 + static_cast<int>((S[h1 / 4] >> (8 * (h1 % 4))) & 0xff);
        const int hdr = __builtin_amdgcn_ds_bpermute((lane - g) << 2, hdr0);
        const int ln = erased ? 0 : (slow ? min(hdr, L) : hdr);
        const int cl = min(ln, L);

        uint32_t W[K + 1];
#pragma unroll
        for (int m = 0; m < K; ++m) {
            const int i0 = 4 * m, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3;
            W[m] = gather4(S, (i0 / K) * n + i0 % K, (i1 / K) * n + i1 % K, (i2 / K) * n + i2 % K,
                           (i3 / K) * n + i3 % K);
        }
        W[K] = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(right << 2, static_cast<int>(W[0])));
        if (valid && !erased) {
            uint32_t O[K];
            const int b0 = 4 * K * g;  // payload byte of output dword 0
#pragma unroll
            for (int m = 0; m < K; ++m)
                O[m] = __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & keep_bytes(cl - (b0 + 4 * m));
            if (ndw > 0) store_words_n<K>(rc, static_cast<int>(x * L) + b0, O, ndw);
            if (g == 0) a.out_len[x] = ln;
        }
    }
}

#define FEC_COPY_WAVE_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(1, 10) X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)

#define FEC_COPY_WAVE_INST(K, NP) template __global__ void fec_copy_wave_kernel<K, NP>(CopyWaveArgs);
FEC_COPY_WAVE_LIST(FEC_COPY_WAVE_INST)

const void* fec_copy_wave_kernel_for(int k, int np) {
#define FEC_COPY_WAVE_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_copy_wave_kernel<K, NP>);
    FEC_COPY_WAVE_LIST(FEC_COPY_WAVE_CASE)
#undef FEC_COPY_WAVE_CASE
    return nullptr;
}

}  // namespace fec
