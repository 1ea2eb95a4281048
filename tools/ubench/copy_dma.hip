// copy_dma.hip -- the headline decode copy (fec_copy_fast_kernel<8,3>) against a persistent,
// LDS-DMA double-buffered variant (experiment, not product).
//
// 1 000 000 packets at (10,3,3), L = 300, CW = 418, random codeword bytes, 1.5 % erasures.
//   A  the product kernel (included from csrc/fec_copy_fast.hip): a workgroup per 32-packet tile,
//      stage (16-byte loads into registers, then LDS), header pass, extract, store;
//   B  persistent workgroups walking tiles of TP packets: the next tile's codeword span goes to LDS
//      by buffer_load ... lds (no registers hold it) while the current tile is extracted and
//      stored; VMEM waits from an issue ledger as in fec_encode_tile.hip.
// Outputs (payload rows and lengths) of B are checked against A.
//   hipcc -O3 --offload-arch=gfx950 -I ../../fec_erasure_code_unit_test_relay_amd/csrc \
//       -I ../../include -o copy_dma copy_dma.hip && ./copy_dma
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fec_copy_fast.hip"

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)(p)));
}
__device__ __forceinline__ v4u rsrc(const void* base, uint32_t bytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    return v4u{static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(b & 0xffffffffu))),
               static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>((b >> 32) & 0xffffu))),
               static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(bytes))), 0x00020000u};
}
__device__ __forceinline__ void dma16(v4u r, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(v4u r, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds) : "memory");
}
__device__ __forceinline__ void wait_vm(int n) {
#define VMC(N) \
    case N: __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14)); break;
    switch (n < 0 ? 0 : n) {
        VMC(0) VMC(1) VMC(2) VMC(3) VMC(4) VMC(5) VMC(6) VMC(7) VMC(8) VMC(9) VMC(10) VMC(11) VMC(12)
        VMC(13) VMC(14) VMC(15) VMC(16) VMC(17) VMC(18) VMC(19) VMC(20) VMC(21) VMC(22) VMC(23)
        default: VMC(24)
    }
#undef VMC
}
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));
    __builtin_amdgcn_s_barrier();
}

// TP packets per tile, JN 1 KB DMA pieces per wave per tile (4 * JN KB >= 16 + TP*CW)
template <int K, int NP, int TP, int JN>
__global__ __launch_bounds__(256, 4) void copy_dma(fec::CopyFastArgs a) {
    constexpr int n = K + NP;
    constexpr int RAW = 4 * JN * 1024;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* inb = smem;                          // [2][RAW]
    uint8_t* xo = smem + 2 * RAW;                 // payload tile TP*L
    int32_t* clen = reinterpret_cast<int32_t*>(xo + ((TP * a.L + 15) & ~15));
    uint8_t* erb = reinterpret_cast<uint8_t*>(clen + TP);  // [2][256]: flags [x0, x0+TP+T)
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = a.L, CW = a.CW, NS4 = a.NS4, T = a.T;
    const int64_t ntiles = (a.Pout + TP - 1) / TP;
    const v4u rc = rsrc(a.cw, static_cast<uint32_t>(a.P * CW));
    const v4u re = rsrc(a.er, static_cast<uint32_t>(a.P));
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, static_cast<int>(a.Pout * L), 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(a.out_len, 0, static_cast<int>(a.Pout * 4), 0x00020000);
    uint32_t vm_issued = 0, vm_mark[2] = {0, 0};
    auto issue = [&](int64_t tile, int buf) {
        const int64_t x0 = tile * TP;
        const int64_t g0 = (x0 * CW) & ~int64_t(15);
        const uint32_t dst = lds_addr(inb + buf * RAW);
#pragma unroll
        for (int j = 0; j < JN; ++j) {
            const int c = (j * 4 + wv) * 64 + lane;  // 16-byte chunk of the span
            dma16(rc, static_cast<uint32_t>(g0 + 16 * c), dst + (j * 4 + wv) * 1024);
            ++vm_issued;
        }
        // flags [x0, x0+TP+T): dwords, by wave 0 only (its ledger counts it; the barrier after its
        // wait publishes them)
        if (wv == 0) {
            dma4(re, lane * 4 < TP + T + 3 ? static_cast<uint32_t>(x0 + 4 * lane) : 0x7fffffffu, lds_addr(erb + buf * 256));
            ++vm_issued;
        }
        vm_mark[buf] = vm_issued;
    };
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    issue(tile, 0);
    for (int it = 0; tile < ntiles; ++it, tile += gridDim.x) {
        const int buf = it & 1;
        const int64_t x0 = tile * TP;
        const int ntile = static_cast<int>(min<int64_t>(TP, a.Pout - x0));
        wait_vm(static_cast<int>(vm_issued - vm_mark[buf]));
        lds_barrier();  // tile in LDS everywhere; the other buffer's readers are done
        if (tile + gridDim.x < ntiles) issue(tile + gridDim.x, buf ^ 1);
        const uint8_t* raw = inb + buf * RAW;
        const uint8_t* erw = erb + buf * 256;
        const int delta = static_cast<int>((x0 * CW) & 15);
        for (int t = tid; t < ntile; t += 256) {
            int ln = 0, copy = 0;
            if (!erw[t]) {
                const uint8_t* row = raw + delta + t * CW;
                const int hdr = row[0] * 256 + row[(1 / K) * n + 1 % K];
                bool slow = false;
                for (int d = 0; d <= T; ++d) slow = slow || erw[t + d];
                ln = slow ? min(hdr, L) : hdr;
                copy = min(ln, L);
            }
            clen[t] = copy;
        }
        lds_barrier();
        for (int itm = tid; itm < ntile * NS4; itm += 256) {
            const int g = itm / ntile;
            const int t = itm - g * ntile;
            const int cl = clen[t];
            uint32_t W[K + 1];
            if (cl > 0) {
                const int off = delta + t * CW + 4 * n * g;
                const int a4 = off & ~3;
                uint32_t D[n + 1];
#pragma unroll
                for (int m = 0; m <= n; ++m) D[m] = *reinterpret_cast<const uint32_t*>(raw + a4 + 4 * m);
                uint32_t S[n];
#pragma unroll
                for (int m = 0; m < n; ++m) S[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], off & 3);
#pragma unroll
                for (int m = 0; m < K; ++m) {
                    const int i0 = 4 * m, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3;
                    W[m] = fec::gather4(S, (i0 / K) * n + i0 % K, (i1 / K) * n + i1 % K, (i2 / K) * n + i2 % K,
                                        (i3 / K) * n + i3 % K);
                }
            } else {
#pragma unroll
                for (int m = 0; m < K; ++m) W[m] = 0;
            }
            W[K] = 0;
            uint8_t* orow = xo + t * L;
            const int bh = 4 * g * K - 2;
            if (bh >= 0 && bh < L) *reinterpret_cast<uint16_t*>(orow + bh) = static_cast<uint16_t>(W[0] & fec::keep_bytes(cl - bh));
#pragma unroll
            for (int m = 0; m < K - 1; ++m) {
                const int b = 4 * g * K + 4 * m;
                if (b < L) *reinterpret_cast<uint32_t*>(orow + b) = __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & fec::keep_bytes(cl - b);
            }
            const int bt = 4 * g * K + 4 * K - 4;
            if (bt < L) *reinterpret_cast<uint16_t*>(orow + bt) = static_cast<uint16_t>((W[K - 1] >> 16) & fec::keep_bytes(cl - bt));
        }
        lds_barrier();
        // stores: NSO 16-byte chunks per thread (out of range: dropped), one length per packet
        constexpr int NSO = (TP * 300 / 16 + 255) / 256;
        const int ob = ntile * L;
#pragma unroll
        for (int j = 0; j < NSO; ++j) {
            const int c = (tid + 256 * j) * 16;
            const bool ok = c < ob;
            const uint4 v = *reinterpret_cast<const uint4*>(xo + (ok ? c : 0));
            __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, ro, ok ? static_cast<int>(x0 * L + c) : 0x7ffffff0, 0, 2);
            ++vm_issued;
        }
        const bool own = tid < ntile;
        int lnv = 0;
        if (own && !erw[tid]) {
            const uint8_t* row = raw + delta + tid * CW;
            const int hdr = row[0] * 256 + row[(1 / K) * n + 1 % K];
            bool slow = false;
            for (int d = 0; d <= T; ++d) slow = slow || erw[tid + d];
            lnv = slow ? min(hdr, L) : hdr;
        }
        __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(lnv), rl, own ? static_cast<int>(4 * (x0 + tid)) : 0x7ffffff0, 0, 0);
        ++vm_issued;
    }
    wait_vm(0);
}

}  // namespace

int main() {
    const int64_t Pout = 1000000, T = 10, P = Pout + T;
    const int K = 8, n = 11, L = 300, CW = 418, NS4 = 10;
    std::vector<uint8_t> hcw(static_cast<size_t>(P) * CW), her(static_cast<size_t>(P));
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (auto& c : hcw) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        c = static_cast<uint8_t>(s >> 56);
    }
    for (auto& e : her) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        e = (s >> 40) % 1000 < 15 ? 1 : 0;
    }
    uint8_t *cw, *er, *o1, *o2;
    int32_t *l1, *l2;
    CHECK(hipMalloc(&cw, hcw.size() + 64));
    CHECK(hipMalloc(&er, her.size() + 64));
    CHECK(hipMalloc(&o1, Pout * L));
    CHECK(hipMalloc(&o2, Pout * L));
    CHECK(hipMalloc(&l1, Pout * 4));
    CHECK(hipMalloc(&l2, Pout * 4));
    CHECK(hipMemcpy(cw, hcw.data(), hcw.size(), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(er, her.data(), her.size(), hipMemcpyHostToDevice));
    fec::CopyFastArgs a{};
    a.cw = cw;
    a.er = er;
    a.P = P;
    a.Pout = Pout;
    a.L = L;
    a.CW = CW;
    a.NS4 = NS4;
    a.T = static_cast<int>(T);
    a.stamps = nullptr;
    a.skip_erased = 0;
    a.nt = 1;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        float best = 1e9f, sum = 0;
        for (int r = 0; r < 40; ++r) {
            CHECK(hipEventRecord(e0));
            launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 5) {
                best = ms < best ? ms : best;
                sum += ms;
            }
        }
        std::printf("%-40s best %7.1f us  mean %7.1f us  %5.2f TB/s (719 B/packet)\n", name, best * 1e3, sum / 35 * 1e3,
                    719.0 * Pout / (best * 1e-3) / 1e12);
    };
    // A: the product kernel, TP = 32 as the codec picks at (10,3,3)
    fec::CopyFastArgs aa = a;
    aa.out = o1;
    aa.out_len = l1;
    aa.TP = 32;
    aa.raw_bytes = (16 + 32 * CW + 4 * n + 16 + 15) & ~15;
    aa.out_bytes = (32 * L + 15) & ~15;
    const int lds_a = aa.raw_bytes + aa.out_bytes + 4 * 32 + 32 + 10 + 16;
    const void* ka = reinterpret_cast<const void*>(&fec::fec_copy_fast_kernel<8, 3>);
    CHECK(hipFuncSetAttribute(ka, hipFuncAttributeMaxDynamicSharedMemorySize, lds_a));
    timeit("A product (tile per workgroup, TP 32)", [&] {
        void* args[] = {&aa};
        CHECK(hipLaunchKernel(ka, dim3(static_cast<unsigned>((Pout + 31) / 32)), dim3(256), args, lds_a, 0));
    });
    std::vector<uint8_t> h1(Pout * L), h2(Pout * L);
    std::vector<int32_t> hl1(Pout), hl2(Pout);
    CHECK(hipMemcpy(h1.data(), o1, Pout * L, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hl1.data(), l1, Pout * 4, hipMemcpyDeviceToHost));
    int rc = 0;
    auto variant = [&](const char* name, const void* kb, int TP, int JN, int grid) {
        fec::CopyFastArgs ab = a;
        ab.out = o2;
        ab.out_len = l2;
        ab.TP = TP;
        const int lds = 2 * 4 * JN * 1024 + ((TP * L + 15) & ~15) + 4 * TP + 512;
        CHECK(hipFuncSetAttribute(kb, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        CHECK(hipMemset(o2, 0x55, Pout * L));
        CHECK(hipMemset(l2, 0x55, Pout * 4));
        char nm[96];
        std::snprintf(nm, sizeof nm, "%s grid %d", name, grid);
        timeit(nm, [&] {
            void* args[] = {&ab};
            CHECK(hipLaunchKernel(kb, dim3(static_cast<unsigned>(grid)), dim3(256), args, lds, 0));
        });
        CHECK(hipMemcpy(h2.data(), o2, Pout * L, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hl2.data(), l2, Pout * 4, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t x = 0; x < Pout; ++x)
            if (hl1[x] != hl2[x] || std::memcmp(&h1[x * L], &h2[x * L], L)) ++bad;
        std::printf("    %ld packets differ from A\n", static_cast<long>(bad));
        if (bad) rc = 1;
    };
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const void* b24 = reinterpret_cast<const void*>(&copy_dma<8, 3, 24, 3>);
    const void* b32 = reinterpret_cast<const void*>(&copy_dma<8, 3, 32, 4>);
    for (int w : {3, 4, 5}) variant("B dma TP 24", b24, 24, 3, cus * w);
    for (int w : {3, 4}) variant("B dma TP 32", b32, 32, 4, cus * w);
    return rc;
}
