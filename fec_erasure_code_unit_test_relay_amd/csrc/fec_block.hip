// fec_block.hip -- block-mode coding of many independent code blocks: the batched forms of the
// reference's free functions
//   encodeBlock(data, G, cw, k, n, t = k-1)        (src/codingOperations.cpp:131-147)
//   decodeBlock(cw, G, cw, erasure, k, n, T = n-1, t = 0)   (src/codingOperations.cpp:149-232)
// as Decoder_Symbol_Wise's relay calls them per code block (src/Decoder_Symbol_Wise.cpp:322-328,
// 532-533, 573-575, 610, 643): a full-window decode of one codeword of n symbols, then a
// re-encode.  One thread per block; a workgroup stages 256 consecutive blocks through LDS so that
// the HBM side moves contiguous bytes; GF products go through LDS log/antilog tables.
//
// decodeBlock's outcome for window w = n is a function of the erasure mask alone: the rule table
// built on the host (fec_host.cpp, DecodeRules; the codec's table covers w = n for every T)
// gives, per erased data symbol i, whether the reference recovers it and the coefficients of its
// action-matrix column on the received symbols (zero on erased ones: a zero column is never
// combined into another one by gf256_rref_matrix's column operations).
#include "fec_kernels.h"

namespace fec {

constexpr int kBlkThreads = 256;

__device__ __forceinline__ uint8_t gf_mul_log(const uint8_t* gexp, const uint8_t* glog, int logc, uint8_t x) {
    return x ? gexp[logc + glog[x]] : 0;
}

// Stage `bytes` contiguous bytes from global into LDS (dwords when both sides allow it).
__device__ __forceinline__ void blk_stage_in(uint8_t* dst, const uint8_t* src, int bytes) {
    if (((reinterpret_cast<uintptr_t>(src) | bytes) & 3) == 0) {
        for (int o = threadIdx.x * 4; o < bytes; o += kBlkThreads * 4)
            *reinterpret_cast<uint32_t*>(dst + o) = *reinterpret_cast<const uint32_t*>(src + o);
    } else {
        for (int o = threadIdx.x; o < bytes; o += kBlkThreads) dst[o] = src[o];
    }
}
__device__ __forceinline__ void blk_stage_out(uint8_t* dst, const uint8_t* src, int bytes) {
    if (((reinterpret_cast<uintptr_t>(dst) | bytes) & 3) == 0) {
        for (int o = threadIdx.x * 4; o < bytes; o += kBlkThreads * 4)
            *reinterpret_cast<uint32_t*>(dst + o) = *reinterpret_cast<const uint32_t*>(src + o);
    } else {
        for (int o = threadIdx.x; o < bytes; o += kBlkThreads) dst[o] = src[o];
    }
}

// encodeBlock with t = k-1 for every block: cw = [data, parity], parity j = XOR_i G[i][j] * d[i].
__global__ __launch_bounds__(kBlkThreads) void fec_block_encode_kernel(BlockArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* gexp = smem;                       // 512
    uint8_t* glog = smem + 512;                 // 256
    int16_t* lgc = reinterpret_cast<int16_t*>(smem + 768);  // k*n coefficient logs, -1 = zero
    uint8_t* tin = smem + 768 + 2 * 512;        // 256*k
    uint8_t* tout = tin + kBlkThreads * a.k;    // 256*n
    const int k = a.k, n = a.n;
    for (int i = threadIdx.x; i < 512; i += kBlkThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kBlkThreads) glog[i] = a.gf[512 + i];
    __syncthreads();
    for (int i = threadIdx.x; i < k * n; i += kBlkThreads) {
        const uint8_t c = a.G[i];
        lgc[i] = c ? glog[c] : -1;
    }
    for (int64_t b0 = static_cast<int64_t>(blockIdx.x) * kBlkThreads; b0 < a.nblk;
         b0 += static_cast<int64_t>(gridDim.x) * kBlkThreads) {
        const int nb = static_cast<int>(min<int64_t>(kBlkThreads, a.nblk - b0));
        blk_stage_in(tin, a.in + b0 * k, nb * k);
        __syncthreads();
        if (threadIdx.x < nb) {
            const uint8_t* d = tin + threadIdx.x * k;
            uint8_t* o = tout + threadIdx.x * n;
            for (int i = 0; i < k; ++i) o[i] = d[i];
            for (int j = k; j < n; ++j) {
                uint8_t acc = 0;
                for (int i = 0; i < k; ++i) {
                    const int lc = lgc[i * n + j];
                    if (lc >= 0) acc ^= gf_mul_log(gexp, glog, lc, d[i]);
                }
                o[j] = acc;
            }
        }
        __syncthreads();
        blk_stage_out(a.out + b0 * n, tout, nb * n);
        __syncthreads();
    }
}

// decodeBlock with T = n-1, t = 0 for every block: the full window w = n.  out = the codeword with
// every recovered data symbol written in (Decoder_Symbol_Wise reads the data from it), er_out =
// the updated erasure flags (recovered symbols cleared).
__global__ __launch_bounds__(kBlkThreads) void fec_block_decode_kernel(BlockArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* gexp = smem;
    uint8_t* glog = smem + 512;
    uint8_t* tcw = smem + 768;                  // 256*n
    uint8_t* ter = tcw + kBlkThreads * a.n;     // 256*n
    const int k = a.k, n = a.n;
    for (int i = threadIdx.x; i < 512; i += kBlkThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kBlkThreads) glog[i] = a.gf[512 + i];
    const uint8_t* table = a.rules + a.wbase_n;
    for (int64_t b0 = static_cast<int64_t>(blockIdx.x) * kBlkThreads; b0 < a.nblk;
         b0 += static_cast<int64_t>(gridDim.x) * kBlkThreads) {
        const int nb = static_cast<int>(min<int64_t>(kBlkThreads, a.nblk - b0));
        blk_stage_in(tcw, a.in + b0 * n, nb * n);
        blk_stage_in(ter, a.er + b0 * n, nb * n);
        __syncthreads();
        if (threadIdx.x < nb) {
            uint8_t* cw = tcw + threadIdx.x * n;
            uint8_t* er = ter + threadIdx.x * n;
            uint32_t mask = 0;
            for (int c = 0; c < n; ++c) mask |= (er[c] ? 1u : 0u) << c;
            const uint32_t full = n >= 32 ? 0xffffffffu : ((1u << n) - 1);
            if (mask != 0 && mask != full) {  // nothing erased / window all erased (:181-182)
                const uint8_t* e = table + static_cast<int64_t>(mask) * a.ES;
                uint8_t rec[32];
                uint32_t done = 0;
                for (int i = 0; i < k; ++i) {
                    if (!er[i] || e[i] == 0xFF) continue;
                    const uint8_t* col = e + k + i * n;
                    uint8_t acc = 0;
                    for (int c = 0; c < n; ++c) {
                        const uint8_t cf = col[c];
                        if (cf) acc ^= gf_mul_log(gexp, glog, glog[cf], cw[c]);
                    }
                    rec[i] = acc;
                    done |= 1u << i;
                }
                for (int i = 0; i < k; ++i)  // written after all products: decData is computed
                    if (done & (1u << i)) {  // from the codeword before any symbol is replaced
                        cw[i] = rec[i];
                        er[i] = 0;
                    }
            }
        }
        __syncthreads();
        blk_stage_out(a.out + b0 * n, tcw, nb * n);
        if (a.er_out) blk_stage_out(a.er_out + b0 * n, ter, nb * n);
        __syncthreads();
    }
}

}  // namespace fec
