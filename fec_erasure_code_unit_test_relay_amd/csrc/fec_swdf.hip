// fec_swdf.hip -- the relay's symbol-wise decode-and-forward (SWDF, RELAYING_TYPE 2) and the
// destination's symbol-wise decode, batched over many packets of one relay stream.
//
// Reference: Decoder_Symbol_Wise (src/Decoder_Symbol_Wise.cpp) driven by Variable_Rate_FEC_Decoder
// (relay :950-1601, destination :1603-1879) and the local simulation's relay loop with
// FLAG_FOR_CONSTANT_TRANS = 1 (application_local_simulation.cpp:532-587: one relay frame per seq).
//
// Per seq t the relay keeps a window of the last n1 = T1+1 received source codewords
// (push_current_codeword / rotate_pointers_and_insert_zero_word, :119-176; an erased packet is an
// all-zero slot flagged erased; slots before the first packet are zero and NOT erased) and, per
// code block j < S, takes the diagonal  d[m] = symbol (j, m) of packet t-n1+1+m  (:564-568),
// decodes it with decodeBlock(T = n1-1, t = 0) when 0 < erasures(window) < n1-k+1 (:570-573), and
// forwards the k data symbols reversed, Y_t[j][i] = d[k-1-i] (:577-578).  Its frame for seq t is
// the second hop's diagonal code over Y (:593-618):
//   frame = [size BE16][0, 0][S blocks of n2: Y_t[j][p] (p < k), parity p >= k =
//            XOR_{i<k} G2[i][p] * Y_{t-(p-i)}[j][i]][n2-2 zero bytes],  size = (S+1)*n2
// (the 2 zero bytes are codeword_new_vector's offset-2 start, the trailing ones the extra block
// of codeword_r_d_size, Variable_Rate_FEC_Decoder.cpp:998, 1482-1491).
// The destination keeps the same window over the relay frames and outputs, per seq t2, the
// data_with_header of source packet t2 - (n1 + n2 - k - 1) (symbol_wise_decode_1 + extract_data,
// :621-665): out[j*k + i] = d2[k-1-i] with d2 the decoded hop-2 diagonal.
//
// Every decision depends only on the erasure flags: decodeBlock's outcome for a full window is
// the codec's decode rule for (w = n, erasure mask) (fec_host.cpp DecodeRules).  So the byte work
// is two data-parallel kernels: a diagonal decode (one thread per (packet, block)) used by both
// the relay and the destination, and the relay's re-encode.  Undefined behaviour of the reference
// defined away ("Relay"): n flags (not n-1 plus garbage) reach decodeBlock, slots hold
// zero-padded packets, k2 == k.  The block count is the reference's ceil(max_payload/k)+1 on ints
// (:553, :632; at most S): the blocks past it are not relayed and stay zero, as in the reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <new>

#include "fec_amd.h"
#include "fec_kernels.h"

namespace fec {

constexpr int kSwThreads = 256;

struct SwDecodeArgs {
    const uint8_t* in;      // rows of in_stride bytes; symbol (row, j, m) at in_off + j*n + m
    int64_t in_stride;
    int in_off;
    const uint8_t* er;      // per row: 1 = erased
    int64_t P;
    int k, n, S, blocks;
    const uint8_t* rules;   // window-n rule table (raw coefficients)
    int ES;
    const uint8_t* gf;      // exp[512], log[256]
    uint8_t* out;           // rows of out_stride bytes: out[j*k + i]
    int64_t out_stride;
    uint8_t* flag;          // per row (may be null): erasures >= n-k+1
};

struct SwEncodeArgs {
    const uint8_t* y;       // rows of S*k bytes
    int64_t P;
    int k, n2, S, blocks;
    const uint8_t* G2;      // k x n2
    const uint8_t* gf;
    uint8_t* frames;        // rows of F = 2 + (S+1)*n2 bytes
    int F;
};

__global__ __launch_bounds__(kSwThreads) void fec_swdf_decode_kernel(SwDecodeArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    for (int i = threadIdx.x; i < 512; i += kSwThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kSwThreads) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int k = a.k, n = a.n, S = a.S;
    const int64_t total = a.P * S;
    for (int64_t id = static_cast<int64_t>(blockIdx.x) * kSwThreads + threadIdx.x; id < total;
         id += static_cast<int64_t>(gridDim.x) * kSwThreads) {
        const int64_t t = id / S;
        const int j = static_cast<int>(id - t * S);
        uint8_t* o = a.out + t * a.out_stride + j * k;
        if (j >= a.blocks) {  // not relayed / decoded (:553, :632)
            for (int i = 0; i < k; ++i) o[i] = 0;
            continue;
        }
        uint32_t mask = 0;
        uint8_t d[32];
        for (int m = 0; m < n; ++m) {
            const int64_t r = t - n + 1 + m;
            const bool erased = r >= 0 && a.er[r] != 0;
            mask |= (erased ? 1u : 0u) << m;
            d[m] = (r >= 0 && !erased) ? a.in[r * a.in_stride + a.in_off + j * n + m] : 0;
        }
        const int cnt = __popc(mask);
        if (cnt > 0 && cnt < n - k + 1) {  // decodeBlock(T = n-1, t = 0) on the diagonal
            const uint8_t* e = a.rules + static_cast<int64_t>(mask) * a.ES;
            uint8_t rec[32];
            uint32_t done = 0;
            for (int i = 0; i < k; ++i) {
                if (!((mask >> i) & 1u) || e[i] == 0xFF) continue;
                const uint8_t* col = e + k + i * n;
                uint8_t acc = 0;
                for (int c = 0; c < n; ++c) {
                    const uint8_t cf = col[c];
                    if (cf && d[c]) acc ^= gexp[glog[cf] + glog[d[c]]];
                }
                rec[i] = acc;
                done |= 1u << i;
            }
            for (int i = 0; i < k; ++i)
                if ((done >> i) & 1u) d[i] = rec[i];
        }
        for (int i = 0; i < k; ++i) o[i] = d[k - 1 - i];
        if (a.flag && j == 0) a.flag[t] = cnt >= n - k + 1 ? 1 : 0;
    }
}

__global__ __launch_bounds__(kSwThreads) void fec_swdf_encode_kernel(SwEncodeArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ int16_t lg[32 * 32];  // log of G2[i][p], -1 = zero
    for (int i = threadIdx.x; i < 512; i += kSwThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kSwThreads) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int k = a.k, n2 = a.n2, S = a.S, Sk = a.S * a.k;
    for (int i = threadIdx.x; i < k * n2; i += kSwThreads) lg[i] = a.G2[i] ? glog[a.G2[i]] : -1;
    __syncthreads();
    const int64_t total = a.P * S;
    for (int64_t id = static_cast<int64_t>(blockIdx.x) * kSwThreads + threadIdx.x; id < total;
         id += static_cast<int64_t>(gridDim.x) * kSwThreads) {
        const int64_t t = id / S;
        const int j = static_cast<int>(id - t * S);
        uint8_t* f = a.frames + t * a.F;
        if (j == 0) {
            const int size = (S + 1) * n2;
            f[0] = static_cast<uint8_t>(size >> 8);
            f[1] = static_cast<uint8_t>(size);
            f[2] = 0;
            f[3] = 0;
        }
        if (j == S - 1)
            for (int o = 4 + S * n2; o < a.F; ++o) f[o] = 0;
        uint8_t* blk = f + 4 + j * n2;
        if (j >= a.blocks) {
            for (int p = 0; p < n2; ++p) blk[p] = 0;
            continue;
        }
        const uint8_t* yt = a.y + t * Sk + j * k;
        for (int p = 0; p < k; ++p) blk[p] = yt[p];
        for (int p = k; p < n2; ++p) {
            uint8_t acc = 0;
            for (int i = 0; i < k; ++i) {
                const int64_t r = t - (p - i);
                const int lc = lg[i * n2 + p];
                if (r < 0 || lc < 0) continue;
                const uint8_t v = a.y[r * Sk + j * k + i];
                if (v) acc ^= gexp[lc + glog[v]];
            }
            blk[p] = acc;
        }
    }
}

}  // namespace fec

struct fec_swdf {
    fec_codec* hop1 = nullptr;  // Decoder(n1-1, n1-k, n1-k): the relay's decoder_current
    fec_codec* hop2 = nullptr;  // Encoder(n2-1, n2-k, n2-k) / the destination's decoder_current
    fec::CodecView v1, v2;
    int F = 0;
    int blocks = 0;  // ceil(max_payload / k) + 1 on ints (Decoder_Symbol_Wise.cpp:553, :632)
    ~fec_swdf() {
        if (hop1) fec_codec_destroy(hop1);
        if (hop2) fec_codec_destroy(hop2);
    }
};

namespace {

int grid_for(int64_t items) {
    return static_cast<int>(std::min<int64_t>((items + fec::kSwThreads - 1) / fec::kSwThreads, 8192));
}

int launch_diag_decode(const fec::CodecView& v, int blocks, const uint8_t* in, int64_t in_stride, int in_off,
                       const uint8_t* er, int64_t P, uint8_t* out, int64_t out_stride, uint8_t* flag,
                       hipStream_t s) {
    fec::SwDecodeArgs a;
    a.in = in;
    a.in_stride = in_stride;
    a.in_off = in_off;
    a.er = er;
    a.P = P;
    a.k = v.k;
    a.n = v.n;
    a.S = v.S;
    a.blocks = blocks;
    if (v.wbase_n < 0) return FEC_ERR_ARG;  // n > 17: no window-n rule table
    a.rules = v.rules + v.wbase_n;
    a.ES = v.ES;
    a.gf = v.gf;
    a.out = out;
    a.out_stride = out_stride;
    a.flag = flag;
    hipLaunchKernelGGL(fec::fec_swdf_decode_kernel, dim3(grid_for(P * v.S)), dim3(fec::kSwThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // namespace

extern "C" {

int fec_swdf_create(int max_payload, int T1, int N1, int T2, int N2, fec_swdf** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    if (T1 < 0 || N1 < 0 || T2 < 0 || N2 < 0 || T1 - N1 != T2 - N2 || T1 - N1 + 1 < 1) return FEC_ERR_ARG;
    try {
        std::unique_ptr<fec_swdf> w(new fec_swdf());
        // Variable_Rate_FEC_Decoder.cpp:953-954 / :1608: Decoder(n-1, n-k, n-k), Encoder(n2-1,
        // n2-k2, n2-k2) with n = T+1, k = T-N+1 (Application_Layer_Receiver.cpp: n = T_value+1)
        if (int st = fec_codec_create(max_payload, T1, N1, N1, &w->hop1)) return st;
        if (int st = fec_codec_create(max_payload, T2, N2, N2, &w->hop2)) return st;
        fec::codec_view(w->hop1, &w->v1);
        fec::codec_view(w->hop2, &w->v2);
        if (w->v1.S != w->v2.S || w->v1.n > 32 || w->v2.n > 32) return FEC_ERR_ARG;
        w->F = 2 + (w->v1.S + 1) * w->v2.n;
        w->blocks = max_payload / w->v1.k + 1;
        *out = w.release();
        return FEC_OK;
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}

int fec_swdf_destroy(fec_swdf* w) {
    delete w;
    return FEC_OK;
}

int fec_swdf_geometry(const fec_swdf* w, int* k, int* n1, int* n2, int* S, int* frame_bytes, int* delay) {
    if (!w) return FEC_ERR_ARG;
    if (k) *k = w->v1.k;
    if (n1) *n1 = w->v1.n;
    if (n2) *n2 = w->v2.n;
    if (S) *S = w->v1.S;
    if (frame_bytes) *frame_bytes = w->F;
    if (delay) *delay = w->v1.n + w->v2.n - w->v1.k - 1;
    return FEC_OK;
}

size_t fec_swdf_workspace_bytes(const fec_swdf* w, int64_t P) {
    if (!w || P < 0) return 0;
    return static_cast<size_t>(P) * w->v1.S * w->v1.k;
}

int fec_swdf_relay_batch(fec_swdf* w, const uint8_t* d_cw, int64_t cw_stride, const uint8_t* d_erasure,
                         int64_t P, uint8_t* d_frames, uint8_t* d_flag, void* d_work, size_t work_bytes,
                         void* stream) {
    if (!w || P < 0) return FEC_ERR_ARG;
    if (P == 0) return FEC_OK;
    if (!d_cw || !d_erasure || !d_frames || cw_stride < w->v1.S * w->v1.n) return FEC_ERR_ARG;
    if (!d_work || work_bytes < fec_swdf_workspace_bytes(w, P)) return FEC_ERR_WORKSPACE;
    hipStream_t s = static_cast<hipStream_t>(stream);
    uint8_t* y = static_cast<uint8_t*>(d_work);
    const int Sk = w->v1.S * w->v1.k;
    if (int st = launch_diag_decode(w->v1, w->blocks, d_cw, cw_stride, 0, d_erasure, P, y, Sk, d_flag, s)) return st;
    fec::SwEncodeArgs a;
    a.y = y;
    a.P = P;
    a.k = w->v2.k;
    a.n2 = w->v2.n;
    a.S = w->v2.S;
    a.blocks = w->blocks;
    a.G2 = w->v2.G;
    a.gf = w->v2.gf;
    a.frames = d_frames;
    a.F = w->F;
    hipLaunchKernelGGL(fec::fec_swdf_encode_kernel, dim3(grid_for(P * a.S)), dim3(fec::kSwThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int fec_swdf_destination_batch(fec_swdf* w, const uint8_t* d_frames, const uint8_t* d_erasure, int64_t P,
                               uint8_t* d_out, uint8_t* d_flag, void* stream) {
    if (!w || P < 0) return FEC_ERR_ARG;
    if (P == 0) return FEC_OK;
    if (!d_frames || !d_erasure || !d_out) return FEC_ERR_ARG;
    // frame symbol (j, m) at byte 4 + j*n2 + m (size header + codeword_new_vector's offset 2)
    return launch_diag_decode(w->v2, w->blocks, d_frames, w->F, 4, d_erasure, P, d_out, w->v2.S * w->v2.k, d_flag,
                              static_cast<hipStream_t>(stream));
}

}  // extern "C"
