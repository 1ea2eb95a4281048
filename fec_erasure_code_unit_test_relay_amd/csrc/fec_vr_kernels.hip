// fec_vr_kernels.hip -- the byte work of a variable-rate schedule (fec_vr.h) in a few launches:
// encode = per (T,B,N) tuple, gather its instances' payload rows (n-1 all-zero rows in front of
// each: X_{t'<first} = 0) -> the tuple's encode kernel -> scatter into the frames' arrays;
// decode = one copy launch for every received packet (each in its decoder's geometry) + one
// recovery launch over the host plan's coefficient rows.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fec_amd.h"
#include "fec_vr.h"

namespace fec {
namespace {

// One wave per packet row.
__global__ __launch_bounds__(256) void fec_vr_frame_kernel(VrFrameArgs a) {
    const int lane = threadIdx.x & 63;
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); r < a.rows;
         r += static_cast<int64_t>(gridDim.x) * 4) {
        const int lc = a.len_cur[r], lo = a.len_old[r];
        uint8_t* o = a.packets + r * a.stride;
        const uint8_t* c = a.cur + r * a.W;
        const uint8_t* d = a.old + r * a.W;
        if (lane < 10) {
            const int32_t* h = a.hdr + 4 * r;
            uint8_t v;
            switch (lane) {
                case 0: v = static_cast<uint8_t>((r >> 24) & 0xff); break;
                case 1: v = static_cast<uint8_t>((r >> 16) & 0xff); break;
                case 2: v = static_cast<uint8_t>((r >> 8) & 0xff); break;
                case 3: v = static_cast<uint8_t>(r & 0xff); break;
                case 8: v = static_cast<uint8_t>((lc - lc % 256) / 256); break;
                case 9: v = static_cast<uint8_t>(lc % 256); break;
                default: v = static_cast<uint8_t>(h[lane - 4]); break;
            }
            o[lane] = v;
        }
        for (int b = lane; b < lc; b += 64) o[10 + b] = c[b];
        for (int b = lane; b < lo; b += 64) o[10 + lc + b] = d[b];
        if (lane == 0) a.packet_len[r] = 10 + lc + lo;
    }
}

__global__ __launch_bounds__(256) void fec_vr_parse_kernel(VrParseArgs a) {
    const int lane = threadIdx.x & 63;
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); r < a.rows;
         r += static_cast<int64_t>(gridDim.x) * 4) {
        const uint8_t* p = a.packets + r * a.stride;
        const int plen = a.packet_len[r];
        const int lc = plen >= 10 ? p[8] * 256 + p[9] : 0;
        const int64_t lo = plen - 10 - lc;
        uint8_t* c = a.cur + r * a.W;
        uint8_t* d = a.old + r * a.W;
        for (int64_t b = lane; b < a.W; b += 64) {
            c[b] = b < lc ? p[10 + b] : 0;
            d[b] = b < lo ? p[10 + lc + b] : 0;
        }
        if (a.hdr && lane == 0) {
            int32_t* h = a.hdr + 5 * r;
            h[0] = (p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3];
            h[1] = p[4];
            h[2] = p[5];
            h[3] = p[6];
            h[4] = p[7];
        }
    }
}

__global__ __launch_bounds__(256) void fec_vr_gather_kernel(VrGatherArgs a) {
    const int L4 = a.L >> 2;
    const int64_t total = a.nrows * L4;
    for (int64_t f = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; f < total;
         f += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t r = f / L4;
        const int b = static_cast<int>(f - r * L4) * 4;
        const int64_t src = a.rows[r];
        uint32_t v = 0;
        if (src >= 0) v = *reinterpret_cast<const uint32_t*>(a.payload + src * a.L + b);
        *reinterpret_cast<uint32_t*>(a.out + r * a.L + b) = v;
        if (b == 0) a.out_len[r] = src < 0 ? 0 : (a.len ? a.len[src] : a.L);
    }
}

__global__ __launch_bounds__(256) void fec_vr_scatter_kernel(VrScatterArgs a) {
    const int CW = a.CW;
    const int64_t total = a.nrows * CW;
    for (int64_t f = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; f < total;
         f += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t r = f / CW;
        const int b = static_cast<int>(f - r * CW);
        const int64_t d = a.dst[r];
        if (d < 0) continue;
        uint8_t* base = (d & 1) ? a.old : a.cur;
        base[(d >> 1) * a.W + b] = a.cw[r * CW + b];
        if (b == 0) ((d & 1) ? a.len_old : a.len_cur)[d >> 1] = a.cw_len[r];
    }
}

// One thread per 4 output bytes.  Header at symbols 0 and 1 of sub-stream 0 (k = 1: position 0 of
// sub-streams 0 and 1), Decoder.cpp:89-96; the slow path clamps the length (:148-149).
__global__ __launch_bounds__(256) void fec_vr_copy_kernel(VrCopyArgs a) {
    const int L = a.L, L4 = (L + 3) >> 2;
    const int64_t total = a.P * L4;
    for (int64_t f = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; f < total;
         f += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t x = f / L4;
        const int b0 = static_cast<int>(f - x * L4) * 4;
        const uint8_t fate = a.fate[x];
        if (fate == 2) continue;  // recovered: fec_vr_recover_kernel
        uint32_t v = 0;
        int ln = 0;
        if (fate == 1) {
            const int* g = a.inst + 4 * a.pk_dec[x];
            const int k = g[0], n = g[1];
            const uint8_t* src = a.cur + x * a.W;
            const int hdr = src[0] * 256 + src[k > 1 ? 1 : n];
            ln = a.slow[x] ? min(hdr, L) : hdr;
            const int cp = min(ln, L);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int b = b0 + e, h = b + 2;
                if (b < cp) v |= static_cast<uint32_t>(src[(h / k) * n + h % k]) << (8 * e);
            }
        }
        uint8_t* o = a.out + x * L + b0;
        if (b0 + 4 <= L && (L & 3) == 0) {
            *reinterpret_cast<uint32_t*>(o) = v;
        } else {
            for (int e = 0; e < 4 && b0 + e < L; ++e) o[e] = static_cast<uint8_t>(v >> (8 * e));
        }
        if (b0 == 0) a.out_len[x] = ln;
    }
}

// One wave per recovered packet (as fec_recover_kernel): byte h = (sub-stream h/k, position i =
// h%k) = XOR_q coef[i][q] * symbol q of packet x-i+q, read from the reporting decoder's input.
__global__ __launch_bounds__(256) void fec_vr_recover_kernel(VrRecArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t lcf[4][kVrCoefStride];
    const int tid = threadIdx.x;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int lane = tid & 63, wl = tid >> 6;
    const int L = a.L;
    uint8_t* lc = lcf[wl];
    for (int r = blockIdx.x * 4 + wl; r < a.nrec; r += gridDim.x * 4) {
        const int64_t x = a.rec_x[r];
        const int j = a.rec_dec[r];
        const int k = a.inst[4 * j], n = a.inst[4 * j + 1];
        const int64_t sw = a.inst_switch[j];
        for (int i = lane; i < k * n; i += 64) {
            const uint8_t c = a.rec_coef[static_cast<int64_t>(r) * kVrCoefStride + i];
            lc[i] = c ? glog[c] : 255;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        int ln = 0;
        for (int h0 = 0; h0 < L + 2; h0 += 64) {
            const int h = h0 + lane;
            uint8_t acc = 0;
            if (h < L + 2) {
                const int s = h / k, i = h - s * k;
                for (int q = 0; q < n; ++q) {
                    const int lq = lc[i * n + q];
                    const int64_t row = x - i + q;
                    if (lq == 255 || row < 0 || row >= a.rows) continue;
                    const uint8_t v = (row < sw ? a.cur : a.old)[row * a.W + s * n + q];
                    if (v) acc ^= gexp[lq + glog[v]];
                }
            }
            if (h0 == 0) {
                const int hi = __builtin_amdgcn_readlane(static_cast<int>(acc), 0);
                const int lo = __builtin_amdgcn_readlane(static_cast<int>(acc), 1);
                ln = min(hi * 256 + lo, L);
            }
            const int b = h - 2;
            if (b >= 0 && b < L) a.out[x * L + b] = b < ln ? acc : 0;
        }
        if (lane == 0) a.out_len[x] = ln;
        __builtin_amdgcn_wave_barrier();
    }
}

unsigned grid_for(int64_t work) { return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 8192))); }

}  // namespace

int vr_launch_frames(const VrFrameArgs& a, void* s) {
    if (a.rows <= 0) return FEC_OK;
    const int64_t blocks = std::min<int64_t>((a.rows + 3) / 4, 16384);
    hipLaunchKernelGGL(fec_vr_frame_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int vr_launch_parse(const VrParseArgs& a, void* s) {
    if (a.rows <= 0) return FEC_OK;
    const int64_t blocks = std::min<int64_t>((a.rows + 3) / 4, 16384);
    hipLaunchKernelGGL(fec_vr_parse_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int vr_launch_gather(const VrGatherArgs& a, void* s) {
    if (a.nrows <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_gather_kernel, dim3(grid_for(a.nrows * (a.L >> 2))), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_scatter(const VrScatterArgs& a, void* s) {
    if (a.nrows <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_scatter_kernel, dim3(grid_for(a.nrows * a.CW)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_copy(const VrCopyArgs& a, void* s) {
    if (a.P <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_copy_kernel, dim3(grid_for(a.P * ((a.L + 3) >> 2))), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_recover(const VrRecArgs& a, void* s) {
    if (a.nrec <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_recover_kernel, dim3(1024), dim3(256), 0, static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // namespace fec
