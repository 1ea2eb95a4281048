// queue_prio.hip -- does a long-running kernel on a HIGH-priority stream hold kernels launched on
// normal-priority streams (and the null stream) behind it?  (experiment, not product; the resident
// per-packet servers of fec_server.hip are such kernels.)  A "server" kernel spins for 50 ms on the
// high-priority stream; a tiny kernel is then launched on each of NS normal streams and on the null
// stream, and its completion time is measured from the host.  Run for the server stream created
// before and after the normal streams, and with plain streams for comparison.
//   hipcc -O3 --offload-arch=gfx950 -o queue_prio queue_prio.hip && ./queue_prio
#include <hip/hip_runtime.h>

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

static double run(const char* name, hipStream_t srv, std::vector<hipStream_t>& s, int* d, bool null_too) {
    const long long spin_ticks = 100LL * 1000 * 50;  // 50 ms of the 100 MHz wall clock
    for (auto x : s) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, x, d);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, srv, spin_ticks);
    double worst = 0;
    int over = 0;
    for (size_t i = 0; i <= s.size(); ++i) {
        if (i == s.size() && !null_too) break;
        hipStream_t x = i < s.size() ? s[i] : nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, x, d);
        CHECK(hipStreamSynchronize(x));
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        worst = us > worst ? us : worst;
        over += us > 5000 ? 1 : 0;
    }
    CHECK(hipDeviceSynchronize());
    std::printf("%-44s worst %9.1f us, %d of %zu launches over 5 ms\n", name, worst, over, s.size() + (null_too ? 1 : 0));
    return worst;
}

int main() {
    const int NS = 12;
    int* d;
    CHECK(hipMalloc(&d, 4096));
    int lo = 0, hi = 0;
    CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    std::printf("stream priority range: least %d, greatest %d\n", lo, hi);
    for (int rep = 0; rep < 2; ++rep) {
        {  // plain server stream among plain streams (the hazard)
            hipStream_t srv;
            CHECK(hipStreamCreateWithFlags(&srv, hipStreamNonBlocking));
            std::vector<hipStream_t> s(NS);
            for (auto& x : s) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
            run("plain server, 12 plain streams", srv, s, d, false);
            for (auto x : s) CHECK(hipStreamDestroy(x));
            CHECK(hipStreamDestroy(srv));
        }
        {  // high-priority server created first
            hipStream_t srv;
            CHECK(hipStreamCreateWithPriority(&srv, hipStreamNonBlocking, hi));
            std::vector<hipStream_t> s(NS);
            for (auto& x : s) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
            run("high-priority server first, 12 plain + null", srv, s, d, true);
            for (auto x : s) CHECK(hipStreamDestroy(x));
            CHECK(hipStreamDestroy(srv));
        }
        {  // high-priority server created after the plain streams
            std::vector<hipStream_t> s(NS);
            for (auto& x : s) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
            hipStream_t srv;
            CHECK(hipStreamCreateWithPriority(&srv, hipStreamNonBlocking, hi));
            run("high-priority server last, 12 plain + null", srv, s, d, true);
            for (auto x : s) CHECK(hipStreamDestroy(x));
            CHECK(hipStreamDestroy(srv));
        }
        {  // plain streams created with the least priority explicitly, server greatest
            hipStream_t srv;
            CHECK(hipStreamCreateWithPriority(&srv, hipStreamNonBlocking, hi));
            std::vector<hipStream_t> s(NS);
            for (auto& x : s) CHECK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, lo));
            run("high-priority server, 12 least-priority", srv, s, d, true);
            for (auto x : s) CHECK(hipStreamDestroy(x));
            CHECK(hipStreamDestroy(srv));
        }
    }
    return 0;
}
