// fec_vr_cf.h -- the closed-form encode of the variable-rate schedule's leftover codewords, as a
// device function: fec_vr_encode_cf_kernel (fec_vr_kernels.hip) is this body over its grid, and the
// multi-tuple tile encoder (fec_encode_tile.hip) runs it in the workgroups after its segments'.
#pragma once
#include <hip/hip_runtime.h>

#include "fec_device.h"
#include "fec_host.h"
#include "fec_vr.h"

namespace fec {

// The same codewords in closed form, a workgroup per codeword and a thread per output dword: byte
// q = (sub-stream s = q / n, position j = q % n) is X_seq[s][j] (j < k) or XOR_i G[i][j] *
// X_{seq-(j-i)}[s][i] (rows before the instance's first call are zero).  The workgroup first brings
// the n rows X_{seq-n+1..seq} ([len_hi, len_lo, payload, zero pad], one round of dword loads) and
// the tuple's gf_mul4 tables into LDS.  No ring and no chain from codeword to codeword: for the few
// codewords of tuples without a tile geometry (k <= 3 in config 4, 2 188 of 360 010), whose ring
// walk (fec_vr_encode_kernel) was one wave's dependent chain per two codewords (65.5 us beside the
// tile encoder).
// The trimmed size is the workgroup's max of the last non-zero byte + 1.
__device__ __forceinline__ void vr_encode_cf_body(const VrEncodeArgs& a, uint8_t* smem, int bid, int nblk) {
    __shared__ int s_nz[4];
    const int tid = threadIdx.x, L = a.L;
    const int XS = (L + 2 + kMaxK + 3) & ~3;  // LDS row: [hdr, payload, zero pad] (S*k <= L+2+k-1)
    uint32_t* tab = reinterpret_cast<uint32_t*>(smem);          // [k*(n-k)][8]
    uint8_t* xr = smem + a.tab_bytes;                            // [n_max][XS]: rows seq-n+1 .. seq
    const int64_t total = a.cum[a.nenc];
    for (int64_t c = bid; c < total; c += nblk) {
        int lo = 0, hi = a.nenc - 1;  // last e with cum[e] <= c
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a.cum[mid] <= c) lo = mid; else hi = mid - 1;
        }
        const int e = lo;
        const int k = a.inst[4 * e], n = a.inst[4 * e + 1], CW = a.inst[4 * e + 2], np = n - k;
        const uint32_t* gt = a.gtab + a.inst[4 * e + 3];
        const int64_t first = a.span[2 * e], sw = a.span[2 * e + 1];
        const int64_t seq = first + (c - a.cum[e]);
        const int64_t r0 = seq - (n - 1);
        for (int i = tid; i < k * np * 8; i += 256) tab[i] = gt[i];
        // rows: dword d of row rr holds X bytes [4d, 4d+4) = header (d = 0: bytes 0, 1) + payload
        const int nw = XS >> 2;
        for (int d = tid; d < n * nw; d += 256) {
            const int rr = d / nw, w = d - rr * nw;
            const int64_t r = r0 + rr;
            uint32_t v = 0;
            if (r >= first) {
                int ln = a.len ? a.len[r] : L;
                ln = ln < 0 ? 0 : (ln > L ? L : ln);
                const uint8_t* src = a.payload + r * L;
                // X bytes 4w..4w+3 = payload bytes 4w-2 .. 4w+1 (header for 4w-2, 4w-1 < 0)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int p = 4 * w + b - 2;
                    uint32_t x;
                    if (p == -2) x = static_cast<uint32_t>(ln >> 8);
                    else if (p == -1) x = static_cast<uint32_t>(ln & 0xff);
                    else x = p < ln ? src[p] : 0u;
                    v |= x << (8 * b);
                }
            }
            reinterpret_cast<uint32_t*>(xr + rr * XS)[w] = v;
        }
        __syncthreads();
        const bool to_old = seq >= sw;
        const int64_t CWp = (CW + 15) & ~15;
        uint8_t* row = to_old ? a.old + a.base[2 * e + 1] + (seq - sw) * CWp : a.cur + a.base[2 * e] + (seq - first) * CWp;
        const uint8_t* xs = xr + (n - 1) * XS;  // row seq; row seq - d at xs - d * XS
        int last_nz = -1;
        for (int w = tid; 4 * w < CWp; w += 256) {
            uint32_t v = 0;
            int q = 4 * w, s = q / n, j = q - s * n;
#pragma unroll
            for (int b = 0; b < 4; ++b, ++q) {
                uint32_t x = 0;
                if (q < CW) {
                    if (j < k) {
                        x = xs[s * k + j];
                    } else {
                        for (int i = 0; i < k; ++i) {
                            const uint32_t* t = tab + (i * np + (j - k)) * 8;
                            x ^= gf_mul4x(t, xs[s * k + i - (j - i) * XS]) & 0xff;
                        }
                    }
                    if (x) last_nz = q;
                }
                v |= x << (8 * b);
                if (++j == n) {
                    j = 0;
                    ++s;
                }
            }
            if ((reinterpret_cast<uintptr_t>(row) & 3) == 0) {
                *reinterpret_cast<uint32_t*>(row + 4 * w) = v;
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b) row[4 * w + b] = static_cast<uint8_t>(v >> (8 * b));
            }
        }
        for (int o = 32; o > 0; o >>= 1) last_nz = max(last_nz, __shfl_xor(last_nz, o));
        if ((tid & 63) == 0) s_nz[tid >> 6] = last_nz;
        __syncthreads();
        if (tid == 0)
            (to_old ? a.len_old : a.len_cur)[seq] = max(max(s_nz[0], s_nz[1]), max(s_nz[2], s_nz[3])) + 1;
        __syncthreads();  // the rows, tables and s_nz are read before the next codeword's
    }
}

}  // namespace fec
