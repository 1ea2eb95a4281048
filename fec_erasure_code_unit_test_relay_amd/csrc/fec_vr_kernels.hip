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
// interleaving (as fec_encode_kernel) with the instance's geometry at run time:
//     cw_seq[s*n + j] = X_seq[s][j]                                  j <  k
//     cw_seq[s*n + j] = XOR_{i<k} G[i][j] * X_{seq-(j-i)}[s][i]      j >= k
// over the instance's own packets (X before its first call = 0), X_r[s][i] = byte s*k+i of
// [len_hi, len_lo, payload, zero pad].  The wave keeps the last n rows in an LDS ring (slot
// r % n), each transposed to k planes of ceil(S/4) words (word g of plane i = X_r[4g..4g+3][i]),
// and loads one new row per codeword while it stays in one instance.  One lane task = (position j,
// group g of 4 sub-streams): a plane word, or k packed gf_mul4 products with the instance's
// register tables (staged in LDS per instance); its 4 bytes go to the LDS output row, which
// leaves as dword stores (bytes at the row's two ends).  The trimmed size is the last non-zero
// byte + 1 (FEC_Encoder.cpp:55-60), a wave max.
__global__ __launch_bounds__(256) void fec_vr_encode_kernel(VrEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint8_t* base = smem + wv * a.wave_bytes;
    uint32_t* tabw = reinterpret_cast<uint32_t*>(base);              // [k*(n-k)][8]
    uint8_t* outb = base + a.tab_bytes;                               // output row at offset head
    uint8_t* ring = outb + a.out_bytes;                               // n_max slots
    const int L = a.L;
    const int64_t total = a.cum[a.nenc];
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (blockDim.x >> 6);
    const int64_t chunk = (total + nwaves - 1) / nwaves;
    const int64_t c0 = (static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + wv) * chunk;
    const int64_t c1 = min(total, c0 + chunk);
    if (c0 >= c1) return;
    int lo = 0, hi = a.nenc - 1;  // last e with cum[e] <= c0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.cum[mid] <= c0) lo = mid; else hi = mid - 1;
    }
    int e = lo, k = 0, n = 0, CW = 0, S = 0, NSG = 0, PL = 0, SB = 0;
    float rk = 1.0f;
    int64_t first = 0, sw = 0, next_row = 0;  // next_row: first row not yet in the ring
    const bool words = (L & 3) == 0 && (reinterpret_cast<uintptr_t>(a.payload) & 3) == 0;
    auto put = [&](uint8_t* slot, int q, uint32_t v) {  // X byte q -> plane q % k, column q / k
        const int sidx = static_cast<int>((static_cast<float>(q) + 0.5f) * rk);
        slot[(q - sidx * k) * PL + sidx] = static_cast<uint8_t>(v);
    };
    auto load_row = [&](int64_t r) {
        uint8_t* slot = ring + static_cast<int>(((r % n) + n) % n) * SB;
        for (int d = lane; d < k * NSG; d += 64) reinterpret_cast<uint32_t*>(slot)[d] = 0;
        if (r < first) return;  // all-zero row before the instance's first call
        int ln = a.len ? a.len[r] : L;
        ln = ln < 0 ? 0 : (ln > L ? L : ln);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            put(slot, 0, static_cast<uint32_t>(ln >> 8));
            put(slot, 1, static_cast<uint32_t>(ln & 0xff));
        }
        const uint8_t* src = a.payload + r * L;
        if (words) {
            for (int w = lane; 4 * w < ln; w += 64) {
                const uint32_t v = *reinterpret_cast<const uint32_t*>(src + 4 * w);
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (4 * w + b < ln) put(slot, 4 * w + b + 2, v >> (8 * b));
            }
        } else {
            for (int b = lane; b < ln; b += 64) put(slot, b + 2, src[b]);
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
            S = CW / n;
            NSG = (S + 3) >> 2;
            PL = 4 * NSG;
            SB = k * PL;
            rk = 1.0f / static_cast<float>(k);
            first = a.span[2 * e];
            sw = a.span[2 * e + 1];
        }
        const int64_t seq = first + (c - a.cum[e]);
        wave_sync();  // earlier reads of the ring, tables and output row are done
        if (fresh) {
            const uint32_t* gt = a.gtab + a.inst[4 * e + 3];
            for (int i = lane; i < k * (n - k) * 8; i += 64) tabw[i] = gt[i];
            for (int64_t r = seq - (n - 1); r <= seq; ++r) load_row(r);
        } else {
            for (int64_t r = next_row; r <= seq; ++r) load_row(r);
        }
        next_row = seq + 1;
        const bool to_old = seq >= sw;
        uint8_t* row = (to_old ? a.old : a.cur) + seq * a.W;
        const int head = static_cast<int>(reinterpret_cast<uintptr_t>(row) & 3);
        wave_sync();
        const int slot_seq = static_cast<int>(seq % n);
        const float rg = 1.0f / static_cast<float>(NSG);
        for (int task = lane; task < n * NSG; task += 64) {
            const int j = static_cast<int>((static_cast<float>(task) + 0.5f) * rg);
            const int g = task - j * NSG;
            uint32_t v;
            if (j < k) {
                v = reinterpret_cast<const uint32_t*>(ring + slot_seq * SB + j * PL)[g];
            } else {
                v = 0;
                for (int i = 0; i < k; ++i) {
                    const uint32_t* t = tabw + (i * (n - k) + (j - k)) * 8;
                    if (!t[5]) continue;
                    int sl = slot_seq - (j - i);
                    sl += sl < 0 ? n : 0;
                    v ^= gf_mul4x(t, reinterpret_cast<const uint32_t*>(ring + sl * SB + i * PL)[g]);
                }
            }
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (4 * g + b < S) outb[head + (4 * g + b) * n + j] = static_cast<uint8_t>(v >> (8 * b));
        }
        wave_sync();
        const int nw = (head + CW + 3) >> 2;
        int last_nz = -1;
        for (int w = lane; w < nw; w += 64) {
            const uint32_t v = reinterpret_cast<const uint32_t*>(outb)[w];
            uint8_t* dst = row - head + 4 * w;
            const int p0 = 4 * w - head;  // row byte of word byte 0
            if (p0 >= 0 && p0 + 4 <= CW) {
                *reinterpret_cast<uint32_t*>(dst) = v;
                if (v) last_nz = p0 + 3 - (__builtin_clz(v) >> 3);
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int p = p0 + b;
                    if (p < 0 || p >= CW) continue;
                    const uint8_t x = static_cast<uint8_t>(v >> (8 * b));
                    dst[b] = x;
                    if (x) last_nz = p;
                }
            }
        }
        for (int o = 32; o > 0; o >>= 1) last_nz = max(last_nz, __shfl_xor(last_nz, o));
        if (lane == 0) (to_old ? a.len_old : a.len_cur)[seq] = last_nz + 1;
    }
}

// The copy's per-packet word, one thread per packet: geo[x] = k | n << 8 | fate << 16 | slow << 24
// in the reporting decoder's geometry (fate != 1: fate << 16 only).  Paying the chain fate ->
// decoder -> geometry once here, with a thread per packet, leaves the copy one level of dependent
// loads (its word) in front of the row bytes.
__global__ __launch_bounds__(256) void fec_vr_geo_kernel(VrCopyArgs a) {
    const int64_t x = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (x >= a.P) return;
    const uint32_t f = a.fate[x];
    uint32_t g = f << 16;
    if (f == 1) {
        const int j = a.pk_dec[x];
        g |= static_cast<uint32_t>(a.inst[4 * j]) | static_cast<uint32_t>(a.inst[4 * j + 1]) << 8 |
             (a.slow[x] ? 1u << 24 : 0u);
    }
    a.geo[x] = g;
}

// One thread per output dword of kVrCopyU packets: a workgroup covers kVrCopyU * a.ppb consecutive
// packets, thread t takes word t % L4 of packets u * ppb + t / L4 (u < kVrCopyU).  Per packet: its
// word (fec_vr_geo_kernel), then the header and the word's 4 bytes together (the byte positions
// depend only on k and n; the bytes past the copied length are masked afterwards), then the store.
// (The chain fate -> decoder -> geometry -> header -> bytes in this kernel: 220 us per 360 000
// packets, r03z.)  Payload byte b is codeword byte (h / k) * n + h % k of the reporting decoder's
// geometry, h = b + 2; the header is at symbols 0 and 1 of sub-stream 0 (k = 1: position 0 of
// sub-streams 0 and 1), Decoder.cpp:89-96; the slow path clamps the length (:148-149).
constexpr int kVrCopyU = 4;
__global__ __launch_bounds__(256) void fec_vr_copy_kernel(VrCopyArgs a) {
    const int L = a.L, L4 = (L + 3) >> 2;
    const int pl = static_cast<int>(threadIdx.x) / L4;
    const int w = static_cast<int>(threadIdx.x) - pl * L4;
    if (pl >= a.ppb) return;
    const int64_t wmax = a.W - 1;
    int64_t x[kVrCopyU];
    uint32_t g[kVrCopyU];
#pragma unroll
    for (int u = 0; u < kVrCopyU; ++u) {
        x[u] = (static_cast<int64_t>(blockIdx.x) * kVrCopyU + u) * a.ppb + pl;
        g[u] = x[u] < a.P ? a.geo[x[u]] : 2u << 16;  // 2: recovered (fec_vr_recover_kernel) or none
    }
    int k[kVrCopyU], n[kVrCopyU], cp[kVrCopyU], ln[kVrCopyU];
    const uint8_t* src[kVrCopyU];
    uint32_t h0[kVrCopyU], h1[kVrCopyU];
#pragma unroll
    for (int u = 0; u < kVrCopyU; ++u) {
        const bool rx = (g[u] >> 16 & 0xff) == 1;
        k[u] = rx ? static_cast<int>(g[u] & 0xff) : 1;
        n[u] = rx ? static_cast<int>(g[u] >> 8 & 0xff) : 1;
        src[u] = a.cur + (rx ? x[u] : 0) * a.W;
        h0[u] = rx ? src[u][0] : 0u;
        h1[u] = rx ? src[u][k[u] > 1 ? 1 : n[u]] : 0u;
    }
    for (int ww = w; ww < L4; ww += 256) {  // one pass unless L > 1024 (then ppb = 1)
        const int b0 = 4 * ww;
        uint32_t byte[kVrCopyU][4];
#pragma unroll
        for (int u = 0; u < kVrCopyU; ++u) {
            const bool rx = (g[u] >> 16 & 0xff) == 1;
            const int h = b0 + 2;
            int sidx = static_cast<int>((static_cast<float>(h) + 0.5f) / static_cast<float>(k[u]));
            int i = h - sidx * k[u];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t pos = min<int64_t>(static_cast<int64_t>(sidx) * n[u] + i, wmax);
                byte[u][e] = rx ? src[u][pos] : 0u;
                if (++i == k[u]) {
                    i = 0;
                    ++sidx;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kVrCopyU; ++u) {
            const uint32_t f = g[u] >> 16 & 0xff;
            if (f == 2) continue;
            if (ww == w) {
                const int hdr = static_cast<int>(h0[u] * 256 + h1[u]);
                ln[u] = f == 1 ? ((g[u] >> 24) ? min(hdr, L) : hdr) : 0;
                cp[u] = min(ln[u], L);
            }
            uint32_t v = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) v |= (b0 + e < cp[u] ? byte[u][e] : 0u) << (8 * e);
            uint8_t* o = a.out + x[u] * L;
            if (b0 + 4 <= L && (L & 3) == 0) {
                *reinterpret_cast<uint32_t*>(o + b0) = v;
            } else {
                for (int e = 0; e < 4 && b0 + e < L; ++e) o[b0 + e] = static_cast<uint8_t>(v >> (8 * e));
            }
            if (ww == 0) a.out_len[x[u]] = ln[u];
        }
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
    const int wpb = std::min(4, 65536 / std::max(1, a.wave_bytes));
    if (wpb < 1) return FEC_ERR_ARG;
    // A wave walks its codewords one after another (a chain of dependent loads per codeword):
    // as many waves as the chip holds before the walks get longer than 2 codewords.
    const int64_t waves = std::max<int64_t>(1, std::min<int64_t>((a.cum_host_total + 1) / 2, 16384));
    const unsigned grid = static_cast<unsigned>((waves + wpb - 1) / wpb);
    hipLaunchKernelGGL(fec_vr_encode_kernel, dim3(grid), dim3(64 * wpb), static_cast<size_t>(wpb) * a.wave_bytes,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_copy(const VrCopyArgs& a, void* s) {
    if (a.P <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_geo_kernel, dim3(static_cast<unsigned>((a.P + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    const int64_t per_wg = static_cast<int64_t>(kVrCopyU) * a.ppb;
    hipLaunchKernelGGL(fec_vr_copy_kernel, dim3(static_cast<unsigned>((a.P + per_wg - 1) / per_wg)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_recover(const VrRecArgs& a, void* s) {
    if (a.nrec <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_recover_kernel, dim3(1024), dim3(256), 0, static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // namespace fec
