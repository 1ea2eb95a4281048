// Micro-benchmark: issue rate of v_perm_b32, v_bitop3_b32, v_xor_b32, v_alignbyte_b32 (wave64,
// 8 independent chains per lane) measured with s_memtime; prints cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ void kern(uint32_t* out, uint64_t* cyc, int iters) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 2654435761u + i;
    uint32_t s0 = out[0] | 0x03020100u, s1 = out[1] | 0x07060504u;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (OP == 0) a[i] = __builtin_amdgcn_perm(a[i], s0, a[(i + 1) & 7]);
                if (OP == 1) a[i] = __builtin_amdgcn_bitop3_b32(a[i], s0, a[(i + 1) & 7], 0x96);
                if (OP == 2) a[i] = a[i] ^ a[(i + 1) & 7];
                if (OP == 3) a[i] = __builtin_amdgcn_alignbyte(a[i], a[(i + 1) & 7], 2);
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x ^= a[i];
    out[2 + blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    uint32_t* out; uint64_t* cyc;
    hipMalloc(&out, 64 << 20); hipMalloc(&cyc, 1 << 20);
    hipMemset(out, 0, 64 << 20);
    const int iters = 200;
    const char* names[] = {"v_perm_b32", "v_bitop3_b32", "v_xor_b32", "v_alignbyte_b32"};
    for (int wps : {1, 2, 4, 8}) {          // waves per SIMD: blocks of 64*4*wps threads, one per CU
        for (int op = 0; op < 4; ++op) {
            dim3 grid(256), block(256 * wps > 1024 ? 1024 : 256 * wps);
            auto launch = [&]() {
                if (op == 0) hipLaunchKernelGGL(kern<0>, grid, block, 0, 0, out, cyc, iters);
                if (op == 1) hipLaunchKernelGGL(kern<1>, grid, block, 0, 0, out, cyc, iters);
                if (op == 2) hipLaunchKernelGGL(kern<2>, grid, block, 0, 0, out, cyc, iters);
                if (op == 3) hipLaunchKernelGGL(kern<3>, grid, block, 0, 0, out, cyc, iters);
            };
            launch(); hipDeviceSynchronize();
            launch(); hipDeviceSynchronize();
            uint64_t c[256]; hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
            double avg = 0; for (int i = 0; i < 256; ++i) avg += c[i]; avg /= 256;
            const double instr = double(iters) * 16 * 8;   // per wave
            const int waves_per_simd = (block.x / 64) / 4;
            printf("%-16s waves/SIMD %d: %.2f cycles per wave-instr per SIMD (%.2f per wave)\n", names[op],
                   waves_per_simd, avg / (instr * waves_per_simd), avg / instr);
        }
    }
    return 0;
}
