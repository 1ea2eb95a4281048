// Which in-process timing of one kernel launch agrees with rocprofv3's kernel duration?
//   (a) hipEventRecord before and after the launch on its stream
//   (b) hipExtLaunchKernel with a start and a stop event bound to the dispatch
//   (c) hipExtLaunchKernel with only a start event bound, then hipEventRecord(stop)
//   (d) the kernel's own s_memrealtime stamps (first workgroup start, last workgroup end; 100 MHz)
// Each launch is a grid-stride 16-byte copy of 418 MB -> 300 MB-ish traffic like the codec's
// kernels, with a second kernel between launches (like the step's encoder -> copy).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/event_timing tools/ubench/event_timing.hip
// Run:   rocprofv3 --kernel-trace --stats -d gpurun_out/evt -- tools/ubench/event_timing
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int M>
__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                   int64_t n, unsigned long long* stamps) {
    if (stamps && threadIdx.x == 0) atomicMin(&stamps[0], (unsigned long long)wall_clock64());
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = in[i];
    if (stamps) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(&stamps[1], (unsigned long long)wall_clock64());
    }
}

__global__ void other_kernel(uint4* __restrict__ buf, int64_t n) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        uint4 v = buf[i];
        v.x ^= 1u;
        buf[i] = v;
    }
}

int main() {
    const int64_t in_bytes = 418000000, out_bytes = 418000000;
    const int64_t n = out_bytes / 16;
    uint4 *in, *out, *other;
    unsigned long long* stamps;
    CK(hipMalloc(&in, in_bytes));
    CK(hipMalloc(&out, out_bytes));
    CK(hipMalloc(&other, 64 << 20));
    CK(hipMalloc(&stamps, 16));
    CK(hipMemset(in, 1, in_bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned grid = cus * 8;
    const int N = 50;
    unsigned long long* nul = nullptr;
    auto other_launch = [&]() { hipLaunchKernelGGL(other_kernel, dim3(1024), dim3(256), 0, s, other, (int64_t)(64 << 20) / 16); };
    // warm up
    for (int i = 0; i < 20; ++i) {
        hipLaunchKernelGGL(copy_kernel<9>, dim3(grid), dim3(256), 0, s, in, out, n, nul);
        other_launch();
    }
    CK(hipStreamSynchronize(s));
    std::vector<hipEvent_t> a(N), b(N);
    for (int i = 0; i < N; ++i) { CK(hipEventCreate(&a[i])); CK(hipEventCreate(&b[i])); }
    const char* names[3] = {"(a) record around", "(b) ext start+stop", "(c) ext start + record stop"};
    for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 3; ++m) {
        for (int i = 0; i < N; ++i) {
            void* args[] = {&in, &out, (void*)&n, &nul};
            const void* fn = m == 0 ? (const void*)copy_kernel<0> : m == 1 ? (const void*)copy_kernel<1> : (const void*)copy_kernel<2>;
            if (m == 0) {
                CK(hipEventRecord(a[i], s));
                CK(hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s));
                CK(hipEventRecord(b[i], s));
            } else if (m == 1) {
                CK(hipExtLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s, a[i], b[i], 0));
            } else {
                CK(hipExtLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s, a[i], nullptr, 0));
                CK(hipEventRecord(b[i], s));
            }
            other_launch();
        }
        CK(hipStreamSynchronize(s));
        double tot = 0, mn = 1e9, mx = 0;
        for (int i = 0; i < N; ++i) {
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a[i], b[i]));
            tot += ms; mn = ms < mn ? ms : mn; mx = ms > mx ? ms : mx;
        }
        std::printf("%-30s avg %.2f us  min %.2f  max %.2f\n", names[m], tot / N * 1e3, mn * 1e3, mx * 1e3);
    }
    // (d) in-kernel stamps
    double tot = 0;
    for (int i = 0; i < N; ++i) {
        unsigned long long init[2] = {~0ull, 0ull};
        CK(hipMemcpyAsync(stamps, init, 16, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(copy_kernel<3>, dim3(grid), dim3(256), 0, s, in, out, n, stamps);
        unsigned long long got[2];
        CK(hipMemcpyAsync(got, stamps, 16, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        other_launch();
        tot += (double)(got[1] - got[0]) / 100.0;  // 100 MHz
    }
    std::printf("%-30s avg %.2f us\n", "(d) in-kernel wall clock", tot / N);
    std::printf("rocprof: copy_kernel<M> for method M (0..2: %d launches each, 3: (d)), <9>: warm-up\n", 2 * N);
    return 0;
}
