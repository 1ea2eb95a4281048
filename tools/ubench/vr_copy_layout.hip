// vr_copy_layout.hip -- config 4's decode copy under two row layouts (experiment, not product).
//
// 360 000 received packets, each with its decoder geometry read per packet at run time (k = 8,
// n = 11 here: CW = 418), copied to 300-byte payload rows:
//   A  one thread per output dword of 4 packets, byte gathers from HBM (the r03 kernel), rows at
//      stride W;
//   B  a wave stages 4 rows in LDS (16-byte loads), then gathers from LDS, rows at stride W;
//   E  a workgroup stages a tile of 32 consecutive rows (one contiguous span when W = 432) and
//      writes the tile's 32 payload rows as one contiguous run.
// W = 3328 (the plan's cw_max stride, set by k = 1) and W = 432 (compact rows, CW rounded to 16).
//   hipcc -O3 --offload-arch=gfx950 -o vr_copy_layout vr_copy_layout.hip && ./vr_copy_layout
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int L = 300, L4 = 75;

__global__ __launch_bounds__(256) void copy_a(const uint8_t* cur, long W, const uint32_t* geo, long P, uint8_t* out) {
    const int ppb = 256 / L4;
    const int pl = threadIdx.x / L4, w = threadIdx.x - pl * L4;
    if (pl >= ppb) return;
    for (int u = 0; u < 4; ++u) {
        const long x = (static_cast<long>(blockIdx.x) * 4 + u) * ppb + pl;
        if (x >= P) return;
        const uint32_t g = geo[x];
        const int k = g & 0xff, n = g >> 8 & 0xff;
        const uint8_t* src = cur + x * W;
        const int h = 4 * w + 2;
        int sidx = static_cast<int>((h + 0.5f) / k), i = h - sidx * k;
        uint32_t v = 0;
        for (int e = 0; e < 4; ++e) {
            v |= static_cast<uint32_t>(src[sidx * n + i]) << (8 * e);
            if (++i == k) {
                i = 0;
                ++sidx;
            }
        }
        reinterpret_cast<uint32_t*>(out + x * L)[w] = v;
    }
}

__global__ __launch_bounds__(256) void copy_b(const uint8_t* cur, long W, const uint32_t* geo, long P, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[4][4][1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long stride = static_cast<long>(gridDim.x) * 16;
    for (long base = (static_cast<long>(blockIdx.x) * 4 + wv) * 4; base < P; base += stride) {
        uint4 v[4];
        int need[4];
        uint32_t g[4];
        for (int u = 0; u < 4; ++u) {
            const long x = base + u;
            g[u] = x < P ? geo[x] : 0x0101;
            const int k = g[u] & 0xff, n = g[u] >> 8 & 0xff;
            need[u] = x < P ? ((L + 1) / k) * n + (L + 1) % k + 1 : 0;
            if (16 * lane < need[u]) v[u] = *reinterpret_cast<const uint4*>(cur + x * W + 16 * lane);
        }
        for (int u = 0; u < 4; ++u)
            if (16 * lane < need[u]) *reinterpret_cast<uint4*>(&stage[wv][u][16 * lane]) = v[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int u = 0; u < 4; ++u) {
            const long x = base + u;
            if (x >= P) break;
            const int k = g[u] & 0xff, n = g[u] >> 8 & 0xff;
            for (int w = lane; w < L4; w += 64) {
                const int h = 4 * w + 2;
                int sidx = static_cast<int>((h + 0.5f) / k), i = h - sidx * k;
                uint32_t val = 0;
                for (int e = 0; e < 4; ++e) {
                    val |= static_cast<uint32_t>(stage[wv][u][sidx * n + i]) << (8 * e);
                    if (++i == k) {
                        i = 0;
                        ++sidx;
                    }
                }
                reinterpret_cast<uint32_t*>(out + x * L)[w] = val;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// a tile of TP consecutive rows: the rows' span [x0*W, (x0+TP)*W) staged whole when W is small
template <int TP>
__global__ __launch_bounds__(256) void copy_e(const uint8_t* cur, long W, const uint32_t* geo, long P, uint8_t* out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    const int tid = threadIdx.x;
    const long ntiles = (P + TP - 1) / TP;
    for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const long x0 = tile * TP;
        const int np = static_cast<int>(min<long>(TP, P - x0));
        const int span = static_cast<int>(np * W);
        const uint4* src = reinterpret_cast<const uint4*>(cur + x0 * W);
        for (int c = tid; 16 * c < span; c += 256) reinterpret_cast<uint4*>(sm)[c] = src[c];
        __syncthreads();
        for (int d = tid; d < np * L4; d += 256) {
            const int p = d / L4, w = d - p * L4;
            const uint32_t g = geo[x0 + p];
            const int k = g & 0xff, n = g >> 8 & 0xff;
            const int h = 4 * w + 2;
            int sidx = static_cast<int>((h + 0.5f) / k), i = h - sidx * k;
            uint32_t val = 0;
            const uint8_t* row = sm + p * W;
            for (int e = 0; e < 4; ++e) {
                val |= static_cast<uint32_t>(row[sidx * n + i]) << (8 * e);
                if (++i == k) {
                    i = 0;
                    ++sidx;
                }
            }
            reinterpret_cast<uint32_t*>(out + x0 * L)[d] = val;
        }
        __syncthreads();
    }
}

int main() {
    const long P = 360000;
    const int k = 8, n = 11;
    std::vector<uint32_t> hg(P, static_cast<uint32_t>(k | n << 8 | 1 << 16));
    uint32_t* geo;
    CHECK(hipMalloc(&geo, P * 4));
    CHECK(hipMemcpy(geo, hg.data(), P * 4, hipMemcpyHostToDevice));
    uint8_t *cur, *out;
    CHECK(hipMalloc(&cur, P * 3328));
    CHECK(hipMalloc(&out, P * L));
    CHECK(hipMemset(cur, 7, P * 3328));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, long W, auto launch) {
        float best = 1e9f;
        for (int r = 0; r < 20; ++r) {
            CHECK(hipEventRecord(e0));
            launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2 && ms < best) best = ms;
        }
        const double bytes = P * (418.0 + 4 + L);
        std::printf("%-28s W=%4ld  %7.1f us  %6.2f TB/s (read 418 + geo 4 + write 300 B/pkt)\n", name, W, best * 1e3,
                    bytes / (best * 1e-3) / 1e12);
    };
    for (long W : {3328L, 432L}) {
        timeit("A byte gathers", W, [&] {
            const int ppb = 256 / L4;
            hipLaunchKernelGGL(copy_a, dim3((P + 4 * ppb - 1) / (4 * ppb)), dim3(256), 0, 0, cur, W, geo, P, out);
        });
        timeit("B wave LDS stage", W, [&] {
            hipLaunchKernelGGL(copy_b, dim3(4096), dim3(256), 0, 0, cur, W, geo, P, out);
        });
        timeit("B wave LDS stage (grid P/16)", W, [&] {
            hipLaunchKernelGGL(copy_b, dim3((P + 15) / 16), dim3(256), 0, 0, cur, W, geo, P, out);
        });
        if (W * 32 <= 64 * 1024) {
            timeit("E tile 32 rows", W, [&] {
                hipLaunchKernelGGL(copy_e<32>, dim3(2048), dim3(256), 32 * W, 0, cur, W, geo, P, out);
            });
            timeit("E tile 32 rows (grid ntiles)", W, [&] {
                hipLaunchKernelGGL(copy_e<32>, dim3((P + 31) / 32), dim3(256), 32 * W, 0, cur, W, geo, P, out);
            });
            timeit("E tile 64 rows", W, [&] {
                hipLaunchKernelGGL(copy_e<64>, dim3((P + 63) / 64), dim3(256), 64 * W, 0, cur, W, geo, P, out);
            });
        }
    }
    CHECK(hipGetLastError());
    return 0;
}
