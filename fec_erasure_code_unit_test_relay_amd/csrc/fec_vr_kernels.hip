// fec_vr_kernels.hip -- the byte work of a variable-rate schedule (fec_vr.h) in three launches:
// encode = one launch over every encoder instance of every (T,B,N) tuple, straight from the
// payload rows into the frames' arrays; decode = one copy launch for every received packet (each
// in its decoder's geometry) + one recovery launch over the host plan's coefficient rows.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fec_amd.h"
#include "fec_device.h"
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

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Each wave encodes a contiguous run of the codeword list, closed form of the diagonal
// interleaving (as fec_encode_kernel) with the instance's geometry at run time: byte p =
// (sub-stream s = p / n, position j = p % n) is X_seq[s][j] for j < k, else
// XOR_i G[i][j] * X_{seq-(j-i)}[s][i] over the instance's own packets (X before its first call =
// 0).  X_r = [len_hi, len_lo, payload, zero pad] (byte s*k+i = X_r[s][i]).  The wave keeps the
// last n rows X_r in an LDS ring (slot r % n) and loads one new row per codeword while it stays
// in one instance.  Lanes own the output row's 4-byte-aligned words (dword stores inside the row,
// bytes at its two ends); the trimmed size is the last non-zero byte + 1 (FEC_Encoder.cpp:55-60).
__global__ __launch_bounds__(256) void fec_vr_encode_kernel(VrEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* gexp = smem;          // 512
    uint8_t* glg = smem + 512;     // 256
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint8_t* glw = smem + 768 + wv * 512;           // the instance's parity-coefficient logs
    uint8_t* ring = smem + 768 + 4 * 512 + wv * a.ring_bytes;  // n_max slots of slot_bytes
    for (int i = tid; i < 768; i += 256) smem[i] = a.gf[i];
    __syncthreads();
    const int L = a.L;
    const int64_t total = a.cum[a.nenc];
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
    const int64_t chunk = (total + nwaves - 1) / nwaves;
    const int64_t c0 = (static_cast<int64_t>(blockIdx.x) * 4 + wv) * chunk;
    const int64_t c1 = min(total, c0 + chunk);
    if (c0 >= c1) return;
    int lo = 0, hi = a.nenc - 1;  // last e with cum[e] <= c0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.cum[mid] <= c0) lo = mid; else hi = mid - 1;
    }
    int e = lo, k = 0, n = 0, CW = 0, SK4 = 0;
    float rn = 1.0f;
    int64_t first = 0, sw = 0, next_row = 0;  // next_row: first row not yet in the ring
    const bool words = (L & 3) == 0 && (reinterpret_cast<uintptr_t>(a.payload) & 3) == 0;
    auto load_row = [&](int64_t r) {  // X_r -> slot r % n (all-zero before the instance's first call)
        uint8_t* slot = ring + static_cast<int>(((r % n) + n) % n) * a.slot_bytes;  // X byte q at slot[q + 2]
        int ln = 0;
        if (r >= first) {
            ln = a.len ? a.len[r] : L;
            ln = ln < 0 ? 0 : (ln > L ? L : ln);
        }
        if (lane == 0)
            *reinterpret_cast<uint16_t*>(slot + 2) =
                static_cast<uint16_t>((ln >> 8) | ((ln & 0xff) << 8));
        const uint8_t* src = a.payload + r * L;
        if (words) {
            for (int w = lane; w < SK4; w += 64) {  // payload bytes 4w..4w+3 at slot[4 + 4w]
                uint32_t v = 0;
                if (4 * w < ln) v = *reinterpret_cast<const uint32_t*>(src + 4 * w) & keep_bytes(ln - 4 * w);
                *reinterpret_cast<uint32_t*>(slot + 4 + 4 * w) = v;
            }
        } else {
            for (int b = lane; b < 4 * SK4; b += 64) slot[4 + b] = b < ln ? src[b] : 0;
        }
    };
    for (int64_t c = c0; c < c1; ++c) {
        bool fresh = c == c0;
        while (a.cum[e + 1] <= c) {
            ++e;
            fresh = true;
        }
        if (fresh) {
            k = a.inst[4 * e];
            n = a.inst[4 * e + 1];
            CW = a.inst[4 * e + 2];
            rn = 1.0f / static_cast<float>(n);
            SK4 = (((CW / n) * k - 2) + 3) >> 2;  // payload-region words of a row
            first = a.span[2 * e];
            sw = a.span[2 * e + 1];
        }
        const int64_t seq = first + (c - a.cum[e]);
        wave_sync();  // earlier reads of the ring are done
        if (fresh) {
            const uint8_t* gl = a.glog + a.inst[4 * e + 3];
            for (int i = lane; i < k * (n - k); i += 64) glw[i] = gl[i];
            for (int64_t r = seq - (n - 1); r <= seq; ++r) load_row(r);
        } else {
            for (int64_t r = next_row; r <= seq; ++r) load_row(r);
        }
        next_row = seq + 1;
        wave_sync();
        const bool to_old = seq >= sw;
        uint8_t* row = (to_old ? a.old : a.cur) + seq * a.W;
        const int head = static_cast<int>(reinterpret_cast<uintptr_t>(row) & 3);
        const int nw = (head + CW + 3) >> 2;
        const int slot_seq = static_cast<int>(seq % n);
        int last_nz = -1;
        for (int w = lane; w < nw; w += 64) {
            uint32_t v = 0;
            int valid = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int p = 4 * w + b - head;
                if (p < 0 || p >= CW) continue;
                valid |= 1 << b;
                const int s = static_cast<int>((static_cast<float>(p) + 0.5f) * rn), j = p - s * n;
                uint32_t byte;
                if (j < k) {
                    byte = ring[slot_seq * a.slot_bytes + s * k + j + 2];
                } else {
                    uint32_t acc = 0;
                    for (int i = 0; i < k; ++i) {
                        const int lg = glw[i * (n - k) + (j - k)];
                        if (lg == 255) continue;
                        int sl = slot_seq - (j - i);
                        sl += sl < 0 ? n : 0;
                        const uint32_t x = ring[sl * a.slot_bytes + s * k + i + 2];
                        if (x) acc ^= gexp[lg + glg[x]];
                    }
                    byte = acc;
                }
                if (byte) last_nz = p;
                v |= byte << (8 * b);
            }
            uint8_t* dst = row - head + 4 * w;
            if (valid == 15) {
                *reinterpret_cast<uint32_t*>(dst) = v;
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (valid & (1 << b)) dst[b] = static_cast<uint8_t>(v >> (8 * b));
            }
        }
        for (int o = 32; o > 0; o >>= 1) last_nz = max(last_nz, __shfl_xor(last_nz, o));
        if (lane == 0) (to_old ? a.len_old : a.len_cur)[seq] = last_nz + 1;
    }
}

// One wave per packet, lanes over its output words.  Header at symbols 0 and 1 of sub-stream 0
// (k = 1: position 0 of sub-streams 0 and 1), Decoder.cpp:89-96; the slow path clamps the length
// (:148-149).  Payload byte b is codeword byte (h / k) * n + h % k, h = b + 2.
__global__ __launch_bounds__(256) void fec_vr_copy_kernel(VrCopyArgs a) {
    const int L = a.L, L4 = (L + 3) >> 2, lane = threadIdx.x & 63;
    for (int64_t xx = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); xx < a.P;
         xx += static_cast<int64_t>(gridDim.x) * 4) {
        const int64_t x = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(xx)));
        const uint8_t fate = a.fate[x];
        if (fate == 2) continue;  // recovered: fec_vr_recover_kernel
        int ln = 0, cp = 0, k = 1, n = 1;
        const uint8_t* src = a.cur + x * a.W;
        if (fate == 1) {
            const int* g = a.inst + 4 * a.pk_dec[x];
            k = g[0];
            n = g[1];
            const int hdr = src[0] * 256 + src[k > 1 ? 1 : n];
            ln = a.slow[x] ? min(hdr, L) : hdr;
            cp = min(ln, L);
        }
        const float rk = 1.0f / static_cast<float>(k);
        uint8_t* o = a.out + x * L;
        for (int w = lane; w < L4; w += 64) {
            const int b0 = 4 * w;
            uint32_t v = 0;
            if (b0 < cp) {
                int h = b0 + 2;
                int sidx = static_cast<int>((static_cast<float>(h) + 0.5f) * rk);
                int i = h - sidx * k;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (b0 + e < cp) v |= static_cast<uint32_t>(src[sidx * n + i]) << (8 * e);
                    if (++i == k) {
                        i = 0;
                        ++sidx;
                    }
                }
            }
            if (b0 + 4 <= L && (L & 3) == 0) {
                *reinterpret_cast<uint32_t*>(o + b0) = v;
            } else {
                for (int e = 0; e < 4 && b0 + e < L; ++e) o[b0 + e] = static_cast<uint8_t>(v >> (8 * e));
            }
        }
        if (lane == 0) a.out_len[x] = ln;
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

int vr_launch_encode(const VrEncodeArgs& a, void* s) {
    if (a.nenc <= 0) return FEC_OK;
    const size_t lds = 768 + 4 * 512 + 4 * static_cast<size_t>(a.ring_bytes);
    if (lds > 64 * 1024) return FEC_ERR_ARG;
    const int64_t total = a.cum_host_total;
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((total + 63) / 64, 4096)));
    hipLaunchKernelGGL(fec_vr_encode_kernel, dim3(grid), dim3(256), lds, static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_copy(const VrCopyArgs& a, void* s) {
    if (a.P <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_copy_kernel, dim3(static_cast<unsigned>(std::min<int64_t>((a.P + 3) / 4, 16384))), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_recover(const VrRecArgs& a, void* s) {
    if (a.nrec <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_recover_kernel, dim3(1024), dim3(256), 0, static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // namespace fec
