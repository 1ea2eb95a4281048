// queue_share.hip -- does a spinning kernel on one stream delay kernels on other streams?
// (experiment, not product).  A "server" kernel spins for `spin_ms` on stream 0; then a trivial kernel
// is launched on each of the other streams and its completion time is measured from the host.
// Streams created plainly (hipStreamCreateWithFlags) share the process's GPU_MAX_HW_QUEUES hardware
// queues; streams created with a CU mask (hipExtStreamCreateWithCUMask, all CUs set) are tested for a
// queue of their own.
//   hipcc -O3 --offload-arch=gfx950 -o queue_share queue_share.hip && ./queue_share
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
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

__global__ void spin(long long cycles) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
}
__global__ void tiny(int* p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

int main() {
    const int NS = 12;
    int* d;
    CHECK(hipMalloc(&d, 4096));
    int dev;
    CHECK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, dev));
    const int ncu = prop.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0);
    for (int c = 0; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
    const long long spin_ticks = 100LL * 1000 * 50;  // 50 ms of the 100 MHz wall clock
    for (int mode = 0; mode < 2; ++mode) {
        std::vector<hipStream_t> s(NS);
        for (int i = 0; i < NS; ++i) {
            if (mode == 0) CHECK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
            else CHECK(hipExtStreamCreateWithCUMask(&s[i], static_cast<uint32_t>(mask.size()), mask.data()));
        }
        for (int i = 0; i < NS; ++i) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s[i], d);
        CHECK(hipDeviceSynchronize());
        double worst = 0, sum = 0;
        for (int srv = 0; srv < 2; ++srv) {
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[srv], spin_ticks);
            for (int i = 0; i < NS; ++i) {
                if (i == srv) continue;
                const auto t0 = std::chrono::steady_clock::now();
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s[i], d);
                CHECK(hipStreamSynchronize(s[i]));
                const double us =
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                worst = us > worst ? us : worst;
                sum += us;
                std::printf("%s spinner on stream %d: stream %2d tiny kernel %9.1f us\n",
                            mode ? "cu-mask" : "plain  ", srv, i, us);
            }
            CHECK(hipDeviceSynchronize());
        }
        std::printf("%s streams: worst %.1f us, mean %.1f us over %d launches\n", mode ? "cu-mask" : "plain  ", worst,
                    sum / (2 * (NS - 1)), 2 * (NS - 1));
        for (auto x : s) CHECK(hipStreamDestroy(x));
    }
    // mode 3: one CU-masked "server" stream created first, then NS plain streams; the spinner runs
    // on the masked stream: does any plain stream land on its queue?
    {
        hipStream_t srv;
        CHECK(hipExtStreamCreateWithCUMask(&srv, static_cast<uint32_t>(mask.size()), mask.data()));
        std::vector<hipStream_t> s(NS);
        for (int i = 0; i < NS; ++i) CHECK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
        for (int i = 0; i < NS; ++i) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s[i], d);
        CHECK(hipDeviceSynchronize());
        double worst = 0;
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, srv, spin_ticks);
        for (int i = 0; i < NS; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s[i], d);
            CHECK(hipStreamSynchronize(s[i]));
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            worst = us > worst ? us : worst;
        }
        CHECK(hipDeviceSynchronize());
        std::printf("masked server first, then %d plain streams: worst %.1f us\n", NS, worst);
        for (auto x : s) CHECK(hipStreamDestroy(x));
        CHECK(hipStreamDestroy(srv));
    }
    return 0;
}
