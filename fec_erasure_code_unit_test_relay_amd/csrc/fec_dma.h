// fec_dma.h -- LDS-DMA (buffer_load ... lds) and vmcnt helpers for the pipelined kernels.
//
// A wave streams HBM rows into LDS without holding them in registers: buffer_load_dword{,x4} with
// the lds bit writes lane i's bytes at M0 + SIZE*i.  The loads are issued from inline asm so that
// hipcc does not treat every later LDS access as a possible read of the DMA's destination (it would
// wait vmcnt(0) in front of each and drain the prefetch); completion is counted by hand with
// wait_vm (vmcnt decrements in issue order).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fec {
namespace dma {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_void_ptr;

// s_waitcnt vmcnt(n) (expcnt, lgkmcnt: no wait); n is a run-time value (0..63), the immediate is not
__device__ __forceinline__ void wait_vm(int n) {
#define FEC_DMA_VM_CASE(N) \
    case (N): __builtin_amdgcn_s_waitcnt(((N) & 15) | (7 << 4) | (15 << 8) | (((N) >> 4) << 14)); break;
#define FEC_DMA_VM_CASE8(B) \
    FEC_DMA_VM_CASE(B) FEC_DMA_VM_CASE(B + 1) FEC_DMA_VM_CASE(B + 2) FEC_DMA_VM_CASE(B + 3) \
    FEC_DMA_VM_CASE(B + 4) FEC_DMA_VM_CASE(B + 5) FEC_DMA_VM_CASE(B + 6) FEC_DMA_VM_CASE(B + 7)
    switch (n < 0 ? 0 : n) {
        FEC_DMA_VM_CASE8(0) FEC_DMA_VM_CASE8(8) FEC_DMA_VM_CASE8(16) FEC_DMA_VM_CASE8(24)
        FEC_DMA_VM_CASE8(32) FEC_DMA_VM_CASE8(40) FEC_DMA_VM_CASE8(48)
        FEC_DMA_VM_CASE(56) FEC_DMA_VM_CASE(57) FEC_DMA_VM_CASE(58) FEC_DMA_VM_CASE(59) FEC_DMA_VM_CASE(60)
        FEC_DMA_VM_CASE(61) FEC_DMA_VM_CASE(62)
        default: FEC_DMA_VM_CASE(63)
    }
#undef FEC_DMA_VM_CASE8
#undef FEC_DMA_VM_CASE
}

// Raw buffer descriptor as four SGPRs (stride 0, num_records bytes; gfx950 dword 3 flags).
__device__ __forceinline__ v4u raw_rsrc(const void* base, int num_records) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    return v4u{static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(b & 0xffffffffu))),
               static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>((b >> 32) & 0xffffu))),
               static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(num_records)), 0x00020000u};
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_ptr)(p)));
}

// lane i's 16 bytes at byte voff of the buffer -> LDS byte lds + 16*i (M0 saved and restored)
__device__ __forceinline__ void dma16(v4u rsrc, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds) : "memory");
}
// the same with the non-temporal policy (data read once)
__device__ __forceinline__ void dma16_nt(v4u rsrc, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds) : "memory");
}
// lane i's 4 bytes -> LDS byte lds + 4*i
__device__ __forceinline__ void dma4(v4u rsrc, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds) : "memory");
}

}  // namespace dma
}  // namespace fec
