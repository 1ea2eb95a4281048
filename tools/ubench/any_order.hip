// any_order.hip -- do kernels launched on one stream with hipExtAnyOrderLaunch run concurrently on
// gfx950?  (experiment, not product)  Four launches of a kernel that keeps 64 workgroups busy for
// `us` microseconds: serial in-order launches take ~4x, concurrent ones ~1x; compared with the same
// launches forked over four streams with events.
//   hipcc -O3 --offload-arch=gfx950 -o any_order any_order.hip && ./any_order
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

__global__ void busy(long long ticks, int* sink) {
    const long long t0 = wall_clock64();
    int v = 0;
    while (wall_clock64() - t0 < ticks) v += threadIdx.x;
    if (v == 12345) sink[0] = v;
}

int main() {
    int* sink;
    CHECK(hipMalloc(&sink, 4));
    hipStream_t s[4];
    for (auto& x : s) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipEvent_t fork, join[4], e0, e1;
    CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    for (auto& j : join) CHECK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const long long ticks = 100 * 50;  // 50 us of the 100 MHz wall clock
    long long tk = ticks;
    void* args[] = {&tk, &sink};
    auto run = [&](const char* name, int mode) {
        float best = 1e9f;
        for (int r = 0; r < 20; ++r) {
            CHECK(hipEventRecord(e0, s[0]));
            if (mode == 0) {  // in order, one stream
                for (int i = 0; i < 4; ++i)
                    CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&busy), dim3(64), dim3(64), args, 0, s[0],
                                             nullptr, nullptr, 0));
            } else if (mode == 1) {  // any order, one stream
                for (int i = 0; i < 4; ++i)
                    CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&busy), dim3(64), dim3(64), args, 0, s[0],
                                             nullptr, nullptr, hipExtAnyOrderLaunch));
            } else {  // forked over four streams
                CHECK(hipEventRecord(fork, s[0]));
                for (int i = 1; i < 4; ++i) CHECK(hipStreamWaitEvent(s[i], fork, 0));
                for (int i = 0; i < 4; ++i)
                    CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&busy), dim3(64), dim3(64), args, 0, s[i],
                                             nullptr, nullptr, 0));
                for (int i = 1; i < 4; ++i) {
                    CHECK(hipEventRecord(join[i], s[i]));
                    CHECK(hipStreamWaitEvent(s[0], join[i], 0));
                }
            }
            // an in-order launch after: waits for everything before it
            CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&busy), dim3(1), dim3(64), args, 0, s[0], nullptr,
                                     nullptr, 0));
            CHECK(hipEventRecord(e1, s[0]));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3 && ms < best) best = ms;
        }
        std::printf("%-28s %8.1f us for 4 x 50 us + 1 x 50 us\n", name, best * 1e3);
    };
    run("in order, one stream", 0);
    run("any order, one stream", 1);
    run("forked over 4 streams", 2);
    return 0;
}
