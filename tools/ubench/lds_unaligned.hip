// Does ds_write_b32 / ds_write_b64 / ds_write_b128 at a byte-unaligned LDS address store all its
// bytes there (unaligned LDS access mode)?  Prints the LDS bytes after each store.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(uint8_t* out, int off) {
    __shared__ __attribute__((aligned(16))) uint8_t s[64];
    if (threadIdx.x == 0) {
        for (int i = 0; i < 64; ++i) s[i] = 0;
        *reinterpret_cast<uint32_t*>(s + off) = 0x44332211u;
        *reinterpret_cast<uint2*>(s + 16 + off) = make_uint2(0x44332211u, 0x88776655u);
        *reinterpret_cast<uint4*>(s + 32 + off) = make_uint4(0x44332211u, 0x88776655u, 0xccbbaa99u, 0x00ffeeddu);
        for (int i = 0; i < 64; ++i) out[i] = s[i];
    }
}

int main() {
    uint8_t* d;
    hipMalloc(&d, 64);
    uint8_t h[64];
    for (int off : {0, 1, 2, 3}) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, off);
        hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
        printf("off %d:", off);
        for (int i = 0; i < 64; ++i) printf("%s%02x", (i % 16) ? "" : " | ", h[i]);
        printf("\n");
    }
    return 0;
}
