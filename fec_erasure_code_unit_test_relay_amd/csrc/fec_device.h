// fec_device.h -- device helpers shared by the specialised (k, n-k) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fec {

// Buffer resources' num_records cap: the kernels read "zero" through the out-of-range offset
// 0x7ffffff0 (a 16-byte load), which must lie wholly past the range even when the buffer is 2 GiB
// or more (num_records 0x7fffffff would leave its first 15 bytes in range).
constexpr int64_t kRsrcMax = 0x7fffffe0;

// GF(2^8) product of four packed bytes by one constant c (c*x is XOR-linear: three register
// tables indexed per byte by v_perm_b32).  tab[0..1] = c*{0..7}, tab[2..3] = c*({0..7}<<3),
// tab[4] = c*({0..3}<<6).
__device__ __forceinline__ uint32_t gf_mul4x(const uint32_t* tab, uint32_t x) {
    const uint32_t g0 = x & 0x07070707u;
    const uint32_t g1 = (x >> 3) & 0x07070707u;
    const uint32_t g2 = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_perm(tab[1], tab[0], g0) ^ __builtin_amdgcn_perm(tab[3], tab[2], g1) ^
           __builtin_amdgcn_perm(tab[4], tab[4], g2);
}

// selector of v_perm_b32(hi, lo, sel): byte codes 0-3 = lo bytes, 4-7 = hi bytes, 12 = 0x00
constexpr uint32_t sel4(int b0, int b1, int b2, int b3) {
    return uint32_t(b0) | (uint32_t(b1) << 8) | (uint32_t(b2) << 16) | (uint32_t(b3) << 24);
}

// The dword whose byte q is byte i_q of the concatenated words src[] (word c/4, byte c%4);
// indices are compile-time constants after unrolling: two v_perm_b32 + one v_or_b32.
template <int NW>
__device__ __forceinline__ uint32_t gather4(const uint32_t (&src)[NW], int i0, int i1, int i2, int i3) {
    const uint32_t lo = __builtin_amdgcn_perm(src[i1 >> 2], src[i0 >> 2],
                                              sel4(i0 & 3, 4 + (i1 & 3), 12, 12));
    const uint32_t hi = __builtin_amdgcn_perm(src[i3 >> 2], src[i2 >> 2],
                                              sel4(12, 12, i2 & 3, 4 + (i3 & 3)));
    return lo | hi;
}

// 1 + the index of the last non-zero byte of row[0, n) (0 if all are zero), row anywhere in LDS or
// memory with row - 16 readable: 16 bytes per step from the end as four aligned dwords, bytes
// outside the row masked off (a byte loop took CW dependent reads per all-zero row: the adaptive
// relay's zero-length gap rows made its encoders 2.3 - 3.6x slower, profiles/r06/enc_rl_probe.txt).
__device__ __forceinline__ int last_nonzero_end(const uint8_t* row, int n) {
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(row), s1 = s0 + static_cast<uintptr_t>(n);
    uintptr_t a = (s1 + 3) & ~uintptr_t(3);  // one past the last dword touching the row
    while (a > s0) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = *reinterpret_cast<const uint32_t*>(a - 4 * (q + 1));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uintptr_t d = a - 4 * (q + 1);  // the dword's first byte
            uint32_t v = w[q];
            if (d + 4 > s1) v &= 0xffffffffu >> (8 * static_cast<int>(d + 4 - s1));  // bytes past the row
            if (d < s0) v = d + 4 <= s0 ? 0u : v & ~((1u << (8 * static_cast<int>(s0 - d))) - 1u);  // before it
            if (v) return static_cast<int>(static_cast<intptr_t>(d - s0)) + (31 - __builtin_clz(v)) / 8 + 1;
        }
        a -= 16;
    }
    return 0;
}

__device__ __forceinline__ uint32_t keep_bytes(int c) {  // mask of the low c bytes (c clamped)
    return c <= 0 ? 0u : (c >= 4 ? 0xffffffffu : ((1u << (8 * c)) - 1u));
}

// Non-temporal (streaming) 16-byte global load / store: data touched once, kept out of the way
// of the caches' other users.
typedef uint32_t nt_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load16(const void* p) {
    const nt_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store16(void* p, uint4 v) {
    const nt_u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<nt_u32x4*>(p));
}

// Copy global bytes [gbase + delta, gbase + total) into lds[delta, total) (same offsets).  gbase
// is 16-byte aligned, delta and total are multiples of 4.  Interior 16-byte chunks use dwordx4
// loads, BATCH of them in flight per thread before the LDS writes; the two edge chunks use dword
// loads so nothing outside the range is read.
template <int BATCH, bool NT = false>
__device__ __forceinline__ void stage_to_lds(uint8_t* lds, const uint8_t* gbase, int delta, int total,
                                             int tid, int nthreads) {
    const int nchunks = (total + 15) >> 4;
    for (int c0 = 0; c0 < nchunks; c0 += nthreads * BATCH) {
        uint4 v[BATCH];
#pragma unroll
        for (int q = 0; q < BATCH; ++q) {
            const int lo = (c0 + q * nthreads + tid) << 4;
            const bool full = lo >= delta && lo + 16 <= total;
            if constexpr (NT) {
                v[q] = full ? nt_load16(gbase + lo) : make_uint4(0, 0, 0, 0);
            } else {
                v[q] = full ? *reinterpret_cast<const uint4*>(gbase + lo) : make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int q = 0; q < BATCH; ++q) {
            const int lo = (c0 + q * nthreads + tid) << 4;
            if (lo >= delta && lo + 16 <= total) *reinterpret_cast<uint4*>(lds + lo) = v[q];
        }
    }
    // bytes of a range that does not start or end on a dword (a row at an odd / 2-mod-4 offset:
    // the continuing decode starts mid-buffer), byte by byte
    if (tid == 0) {
        for (int b = delta; b < total && (b & 3); ++b) lds[b] = gbase[b];
        for (int b = total & ~3; b < total && b >= ((delta + 3) & ~3); ++b) lds[b] = gbase[b];
    }
    // the (at most two) partial chunks at the ends, dword by dword
    for (int o = tid * 4; o < 32; o += nthreads * 4) {
        const int lo16 = delta & ~15, hi16 = total & ~15;
        const int oa = lo16 + o, ob = hi16 + (o - 16);
        if (o < 16 && oa >= delta && oa + 4 <= total && !(lo16 >= delta && lo16 + 16 <= total))
            *reinterpret_cast<uint32_t*>(lds + oa) = *reinterpret_cast<const uint32_t*>(gbase + oa);
        if (o >= 16 && ob >= delta && ob + 4 <= total && hi16 != lo16)
            *reinterpret_cast<uint32_t*>(lds + ob) = *reinterpret_cast<const uint32_t*>(gbase + ob);
    }
}

// Diagnostic phase stamp (s_memtime, shader clock) of workgroup `wg`, slot `k` of 8; only when a
// stamp buffer is given.  Stamps never feed an output.
__device__ __forceinline__ void phase_stamp(uint64_t* stamps, int wg, int k) {
    if (stamps && threadIdx.x == 0) stamps[static_cast<int64_t>(wg) * 8 + k] = __builtin_amdgcn_s_memtime();
}

}  // namespace fec
