// fec_copy_pipe.hip -- decode of received packets: one independent LDS-DMA pipeline per wave.
//
// The reference outputs a received packet's systematic bytes (fast path, Decoder.cpp:77-108; the
// slow path returns the same bytes for received packets, its length clamped to max_payload at
// :148-149).  In the codeword each sub-stream s is [k systematic | n-k parity]; the payload is the
// systematic bytes with the 2-byte length header removed.
//
// Each wave (a workgroup of its own: no s_barrier anywhere) walks a contiguous run of tiles of Q
// packets with a three-slot LDS ring:
//   * the tile's codeword rows (one contiguous Q*CW-byte slab) and its erasure flags arrive in LDS
//     by LDS-DMA, issued two tiles ahead; no register holds a load in flight, and the wave waits
//     for exactly the tile it converts (vmcnt counted by hand, fec_dma.h);
//   * the flags x0..x0+Q+T-1 become one 64-bit ballot: erased = bit p, slow path = any of bits
//     p..p+T (Decoder.cpp:80-83);
//   * item (p, g) = packet p, group g of 4 sub-streams: the group's codeword bytes are read as
//     dwords and realigned, its 4k systematic bytes picked with constant-selector v_perm_b32 and
//     shifted by the header's 2 bytes (the 2 bytes past the group come from the next group's first
//     sub-stream), giving the k output dwords [4kg, 4kg+4k) of row p, masked by the packet's
//     length, written to the wave's output tile in LDS;
//   * the output tile (Q*L bytes, 16-byte aligned in HBM) goes out in 16-byte stores, ~1 KB of
//     contiguous payload per wave instruction; lengths are one dword store per packet.
// Erased packets get a zero row and length 0; fec_recover_kernel overwrites the recovered ones.
#include "fec_device.h"
#include "fec_dma.h"
#include "fec_kernels.h"

#include <utility>

namespace fec {
namespace {

template <typename F, int... Is>
__device__ __forceinline__ void pfor_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void pfor(F&& f) {
    pfor_impl(f, std::make_integer_sequence<int, N>{});
}

// The dword whose byte q is byte I_q of src[] (compile-time indices): a plain copy when the four
// bytes are one word in place, one v_perm_b32 when they come from at most two words, else two and
// an OR.
template <int NW, int I0, int I1, int I2, int I3>
__device__ __forceinline__ uint32_t pgather4(const uint32_t (&src)[NW]) {
    constexpr int w0 = I0 >> 2, w1 = I1 >> 2, w2 = I2 >> 2, w3 = I3 >> 2;
    if constexpr (w0 == w1 && w1 == w2 && w2 == w3 && (I0 & 3) == 0 && (I1 & 3) == 1 && (I2 & 3) == 2 &&
                  (I3 & 3) == 3) {
        return src[w0];
    } else {
        constexpr int a = w0;
        constexpr int b = (w1 != a) ? w1 : (w2 != a) ? w2 : w3;
        if constexpr ((w1 == a || w1 == b) && (w2 == a || w2 == b) && (w3 == a || w3 == b)) {
            constexpr auto code = [](int w, int i) constexpr { return w == a ? (i & 3) : 4 + (i & 3); };
            constexpr uint32_t sel = sel4(code(w0, I0), code(w1, I1), code(w2, I2), code(w3, I3));
            return __builtin_amdgcn_perm(src[b], src[a], sel);
        } else {
            return gather4(src, I0, I1, I2, I3);
        }
    }
}

// codeword byte (relative to group g's first byte 4*n*g) of data_with_header byte d of the group
template <int K, int N>
constexpr int grp_src(int d) {
    return (d / K) * N + d % K;
}

}  // namespace

template <int K, int NP>
__global__ __launch_bounds__(64) void fec_copy_pipe_kernel(CopyPipeArgs a) {
    constexpr int n = K + NP;
    constexpr int SMAX = grp_src<K, n>(4 * K + 1);  // last source byte an item reads
    constexpr int NSRC = SMAX / 4 + 1;              // realigned source words
    constexpr int ND = NSRC + 1;                    // LDS dwords read
    constexpr int H1 = (1 / K) * n + 1 % K;         // codeword byte of header byte 1
    extern __shared__ __attribute__((aligned(16))) uint8_t psmem[];

    const int lane = threadIdx.x;
    const int64_t s_first = static_cast<int64_t>(blockIdx.x) * a.steps_per_wave;
    const int nw = static_cast<int>(min<int64_t>(a.steps_per_wave, a.nsteps - s_first));
    if (nw <= 0) return;
    const int Q = a.Q, L = a.L, CW = a.CW, T = a.T, NS4 = a.NS4;
    const int delta = a.delta, edelta = a.edelta;
    const int slot_stride = a.slot_bytes + 256;
    const int nd = a.nd, npass = a.npass, ns = a.ns;
    const int SO = npass + ns;  // stores per step
    const int ND1 = nd + 1;     // loads per issue
    const int64_t Pout = a.Pout;

    const dma::v4u rs = dma::raw_rsrc(a.cw_base, a.cw_records);
    const dma::v4u re = dma::raw_rsrc(a.er_base, a.er_records);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_records, 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(a.out_len, 0, a.len_records, 0x00020000);
    const uint32_t lds0 = dma::lds_addr(psmem);
    uint8_t* stage = psmem + 3 * slot_stride;

    auto issue = [&](int sidx) __attribute__((always_inline)) {
        const int x0 = static_cast<int>((s_first + sidx) * Q);
        const uint32_t slot = lds0 + (sidx % 3) * slot_stride;
        const uint32_t gb = static_cast<uint32_t>(x0) * static_cast<uint32_t>(CW);  // 16-aligned (Q*CW % 16 == 0)
        for (int j = 0; j < nd; ++j) {
            const int c = j * 64 + lane;
            if (c * 16 < a.slot_bytes) {
                if (a.nt)
                    dma::dma16_nt(rs, gb + 16u * c, slot + j * 1024);
                else
                    dma::dma16(rs, gb + 16u * c, slot + j * 1024);
            }
        }
        dma::dma4(re, static_cast<uint32_t>(x0 + 4 * lane), slot + a.slot_bytes);
    };

    issue(0);
    if (nw > 1) issue(1);
    for (int s = 0; s < nw; ++s) {
        if (s + 2 < nw) issue(s + 2);
        {
            // VMEM instructions issued after tile s's loads: its successors' loads and the stores of
            // the two steps before (exact counts: every instruction below is issued unconditionally)
            int after = 0;
            if (s >= 2) after += SO;
            if (s + 1 < nw) after += ND1;
            if (s >= 1) after += SO;
            if (s + 2 < nw) after += ND1;
            dma::wait_vm(after);
        }
        const uint8_t* sl = psmem + (s % 3) * slot_stride;
        const int64_t x0 = (s_first + s) * Q;
        const int nval = static_cast<int>(min<int64_t>(Q, Pout - x0));
        const uint8_t fv = lane < Q + T ? sl[a.slot_bytes + edelta + lane] : 0;
        const uint64_t fmask = __ballot(fv != 0);
        const uint64_t wmask = (T >= 63) ? ~0ull : ((2ull << T) - 1ull);

        for (int pass = 0; pass < npass; ++pass) {
            const int it = pass * 64 + lane;
            const int p = static_cast<int>(__umulhi(static_cast<uint32_t>(it), a.ns4magic));
            const int g = it - p * NS4;
            const bool active = p < nval;  // it < Q*NS4 follows: p < Q
            const int pp = active ? p : 0;
            const int rowb = delta + pp * CW;
            const int hdr = static_cast<int>(sl[rowb]) * 256 + static_cast<int>(sl[rowb + H1]);
            const bool erased = ((fmask >> pp) & 1ull) != 0;
            const bool slow = ((fmask >> pp) & wmask) != 0;
            const int ln = erased ? 0 : (slow ? min(hdr, L) : hdr);
            const int cl = min(ln, L);
            __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(ln), rl,
                                                  (active && g == 0) ? static_cast<int>(4 * (x0 + p)) : 0x7ffffff0, 0, 0);

            const int b0 = rowb + 4 * n * g;
            const int a4 = b0 & ~3, sh = b0 & 3;
            uint32_t D[ND];
#pragma unroll
            for (int m = 0; m < ND; ++m) D[m] = *reinterpret_cast<const uint32_t*>(sl + a4 + 4 * m);
            uint32_t S[NSRC];
#pragma unroll
            for (int m = 0; m < NSRC; ++m) S[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], sh);
            uint32_t W[K + 1];
            pfor<K>([&](auto mc) __attribute__((always_inline)) {
                constexpr int m = decltype(mc)::value;
                W[m] = pgather4<NSRC, grp_src<K, n>(4 * m), grp_src<K, n>(4 * m + 1), grp_src<K, n>(4 * m + 2),
                                grp_src<K, n>(4 * m + 3)>(S);
            });
            W[K] = pgather4<NSRC, grp_src<K, n>(4 * K), grp_src<K, n>(4 * K + 1), grp_src<K, n>(4 * K + 1),
                            grp_src<K, n>(4 * K + 1)>(S);  // bytes 0, 1 used
            const int ob = 4 * K * g;  // output byte of dword 0
            uint32_t* orow = reinterpret_cast<uint32_t*>(stage + pp * L + ob);
#pragma unroll
            for (int m = 0; m < K; ++m) {
                const uint32_t v = __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & keep_bytes(cl - (ob + 4 * m));
                if (active && ob + 4 * m < L) orow[m] = v;
            }
        }

        // output tile -> HBM: 16-byte pieces, the ones past the batch end dropped by the range check
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        const int tb = Q * L, vb = nval * L;
        for (int k = 0; k < ns; ++k) {
            const int c = (k * 64 + lane) * 16;
            const v4 v = c < tb ? *reinterpret_cast<const v4*>(stage + c) : v4{0, 0, 0, 0};
            const int off = c < vb ? static_cast<int>(x0 * L) + c : 0x7ffffff0;
            if (a.nt)
                __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 0);
        }
    }
    dma::wait_vm(0);
}

#define FEC_COPY_PIPE_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(1, 10) X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)

#define FEC_COPY_PIPE_INST(K, NP) template __global__ void fec_copy_pipe_kernel<K, NP>(CopyPipeArgs);
FEC_COPY_PIPE_LIST(FEC_COPY_PIPE_INST)

const void* fec_copy_pipe_kernel_for(int k, int np) {
#define FEC_COPY_PIPE_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_copy_pipe_kernel<K, NP>);
    FEC_COPY_PIPE_LIST(FEC_COPY_PIPE_CASE)
#undef FEC_COPY_PIPE_CASE
    return nullptr;
}

}  // namespace fec
