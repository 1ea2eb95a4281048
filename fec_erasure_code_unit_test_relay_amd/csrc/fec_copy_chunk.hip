// fec_copy_chunk.hip -- decode of received packets, one lane per 16-byte piece of output.
//
// The reference outputs a received packet's systematic bytes (fast path, Decoder.cpp:77-108; the
// slow path returns the same bytes for received packets, its length clamped to max_payload at
// :148-149).  Output byte b of packet t is data_with_header byte b+2, i.e. position (b+2) % k of
// sub-stream (b+2) / k, which sits at codeword byte ((b+2)/k)*n + (b+2)%k.
//
// Lane i owns output chunk j = i % C of packet t = i / C (C = ceil(L/16)): bytes [16j, 16j+16) of
// row t.  For k dividing 16 the chunk starts at the same sub-stream phase for every j, so the
// chunk's source bytes are a compile-time pattern relative to sub-stream 16j/k: the lane loads the
// few dwords covering them straight from HBM (buffer loads at the dword below, realigned with one
// v_alignbyte per dword), picks the 16 bytes with constant-selector v_perm_b32 and stores them with
// one 16-byte store.  Consecutive lanes store consecutive 16-byte pieces of the payload slab: every
// store instruction writes ~1 KB of contiguous output, and every codeword byte is loaded by the one
// or two lanes whose chunk needs it.  No LDS, no barrier: the waves are independent, and a grid of
// resident waves walks the chunks with two chunks' loads in flight per lane.
//
// Per lane also: the erasure flags t..t+T (one 16-byte load at the dword below t: T <= 12) and the
// length header (bytes 0 and 1 of the codeword), both shared by the C lanes of the packet.  Erased
// packets get a zero row and length 0 here; fec_recover_kernel overwrites the recovered ones after.
#include "fec_device.h"
#include "fec_kernels.h"

#include <utility>

namespace fec {
namespace {

typedef uint32_t cc_v4u __attribute__((ext_vector_type(4)));
typedef uint32_t cc_v3u __attribute__((ext_vector_type(3)));
typedef uint32_t cc_v2u __attribute__((ext_vector_type(2)));

template <typename F, int... Is>
__device__ __forceinline__ void cfor_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void cfor(F&& f) {
    cfor_impl(f, std::make_integer_sequence<int, N>{});
}

// codeword byte of output byte b of a chunk, relative to the chunk's first sub-stream
template <int K, int N>
constexpr int src_rel(int b) {
    return ((2 + b) / K) * N + (2 + b) % K;
}

// The dword whose byte q is byte I_q of src[] (compile-time indices): one v_perm_b32 when the four
// bytes come from at most two words, else two and an OR.
template <int NW, int I0, int I1, int I2, int I3>
__device__ __forceinline__ uint32_t cgather4(const uint32_t (&src)[NW]) {
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

template <int K, int NP>
struct ChunkGeom {
    static constexpr int n = K + NP;
    static constexpr int lo = src_rel<K, n>(0);
    static constexpr int hi = src_rel<K, n>(15);
    static constexpr int NS = (hi - lo) / 4 + 1;  // realigned source words
    static constexpr int NW = NS + 1;             // loaded words (one more for the realignment)
};

// Everything one chunk needs from memory, loaded before any of it is used.
template <int NW>
struct ChunkLoads {
    uint32_t D[NW];
    cc_v4u E;       // erasure flags at the dword below t
    cc_v2u H;       // codeword bytes at the dword below the row start (length header)
};

template <int NW>
__device__ __forceinline__ void load_dwords(uint32_t (&D)[NW], __amdgpu_buffer_rsrc_t rs, int o, int aux) {
#pragma unroll
    for (int c = 0; c < NW; c += 4) {
        if (c + 4 <= NW) {
            const cc_v4u v = aux ? __builtin_amdgcn_raw_buffer_load_b128(rs, o + 4 * c, 0, 2)
                                 : __builtin_amdgcn_raw_buffer_load_b128(rs, o + 4 * c, 0, 0);
            D[c] = v.x;
            D[c + 1] = v.y;
            D[c + 2] = v.z;
            D[c + 3] = v.w;
        } else if (c + 3 == NW) {
            const cc_v3u v = aux ? __builtin_amdgcn_raw_buffer_load_b96(rs, o + 4 * c, 0, 2)
                                 : __builtin_amdgcn_raw_buffer_load_b96(rs, o + 4 * c, 0, 0);
            D[c] = v.x;
            D[c + 1] = v.y;
            D[c + 2] = v.z;
        } else if (c + 2 == NW) {
            const cc_v2u v = aux ? __builtin_amdgcn_raw_buffer_load_b64(rs, o + 4 * c, 0, 2)
                                 : __builtin_amdgcn_raw_buffer_load_b64(rs, o + 4 * c, 0, 0);
            D[c] = v.x;
            D[c + 1] = v.y;
        } else {
            D[c] = aux ? __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4 * c, 0, 2)
                       : __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4 * c, 0, 0);
        }
    }
}

}  // namespace

template <int K, int NP>
__global__ __launch_bounds__(256) void fec_copy_chunk_kernel(CopyChunkArgs a) {
    using G = ChunkGeom<K, NP>;
    constexpr int n = G::n;
    static_assert(16 % K == 0, "the chunk's source pattern is the same for every chunk only when k | 16");
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.cw), 0, a.cw_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.er), 0, a.er_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.out_bytes, 0x00020000);
    const int L = a.L, CW = a.CW, T = a.T, C = a.C;
    const int nt = a.nt;
    const int stride = gridDim.x * blockDim.x;
    const int nchunks = a.nchunks;

    // masks of the flags t..t+T: bytes 0..min(T,7) of the first word, 0..T-8 of the second
    // (T <= 12, host check)
    const uint64_t m_lo = T >= 7 ? ~0ull : ((1ull << (8 * T + 8)) - 1ull);
    const uint64_t m_hi = T >= 8 ? ((1ull << (8 * (T - 7))) - 1ull) : 0ull;

    auto locate = [&](int i, int& t, int& j) __attribute__((always_inline)) {
        int q = static_cast<int>(__umulhi(static_cast<uint32_t>(i), a.cmagic));
        if ((q + 1) * C <= i) ++q;  // the magic may be one short
        t = q;
        j = i - q * C;
    };
    auto issue = [&](int i, ChunkLoads<G::NW>& ld) __attribute__((always_inline)) {
        int t, j;
        locate(i, t, j);
        const bool ok = i < nchunks;
        const int row = t * CW;
        const int src = row + (16 / K) * j * n + G::lo;
        load_dwords<G::NW>(ld.D, rs, ok ? (src & ~3) : 0x7ffffff0, nt);
        const bool fh = ok && !(a.dbg & 4);
        ld.E = __builtin_amdgcn_raw_buffer_load_b128(re, fh ? (t & ~3) : 0x7ffffff0, 0, 0);
        ld.H = __builtin_amdgcn_raw_buffer_load_b64(rs, fh ? (row & ~3) : 0x7ffffff0, 0, 0);
    };
    auto finish = [&](int i, const ChunkLoads<G::NW>& ld) __attribute__((always_inline)) {
        if (i >= nchunks) return;
        int t, j;
        locate(i, t, j);
        const int row = t * CW;
        const int sh = (row + (16 / K) * j * n + G::lo) & 3;
        // flags t..t+T: erased = flag t, slow = any of them (Decoder.cpp:80-83)
        const uint64_t e_lo = static_cast<uint64_t>(ld.E.x) | (static_cast<uint64_t>(ld.E.y) << 32);
        const uint64_t e_hi = static_cast<uint64_t>(ld.E.z) | (static_cast<uint64_t>(ld.E.w) << 32);
        const int s8 = 8 * (t & 3);
        const uint64_t f0 = s8 ? ((e_lo >> s8) | (e_hi << (64 - s8))) : e_lo;  // flags t..t+7
        const uint64_t f1 = e_hi >> s8;                                         // flags t+8..
        const bool erased = (f0 & 0xff) != 0;
        const bool slow = ((f0 & m_lo) | (f1 & m_hi)) != 0;
        // length header: data_with_header bytes 0 and 1 = sub-stream 0 positions 0 and 1 (k > 1)
        const uint64_t h64 = (static_cast<uint64_t>(ld.H.x) | (static_cast<uint64_t>(ld.H.y) << 32)) >> (8 * (row & 3));
        constexpr int h1 = (1 / K) * n + 1 % K;
        const int hdr = static_cast<int>(h64 & 0xff) * 256 + static_cast<int>((h64 >> (8 * h1)) & 0xff);
        const int ln = erased ? 0 : (slow ? min(hdr, L) : hdr);
        const int cl = min(ln, L);
        if (j == 0) a.out_len[t] = ln;

        uint32_t S[G::NS];
#pragma unroll
        for (int m = 0; m < G::NS; ++m) S[m] = __builtin_amdgcn_alignbyte(ld.D[m + 1], ld.D[m], sh);
        uint32_t O[4];
        cfor<4>([&](auto qc) __attribute__((always_inline)) {
            constexpr int qq = decltype(qc)::value;
            O[qq] = cgather4<G::NS, src_rel<K, n>(4 * qq) - G::lo, src_rel<K, n>(4 * qq + 1) - G::lo,
                             src_rel<K, n>(4 * qq + 2) - G::lo, src_rel<K, n>(4 * qq + 3) - G::lo>(S);
        });
        const int b0 = 16 * j;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) O[qq] &= keep_bytes(cl - (b0 + 4 * qq));
        const int o = (a.dbg & 2) ? 0x7ffffff0 : ((a.dbg & 1) ? ((t * L + b0) & ~15) : t * L + b0);
        const int rem = L - b0;  // >= 4, a multiple of 4
        if (rem >= 16) {
            const cc_v4u v = {O[0], O[1], O[2], O[3]};
            if (nt)
                __builtin_amdgcn_raw_buffer_store_b128(v, ro, o, 0, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b128(v, ro, o, 0, 0);
        } else if (rem == 12) {
            // the row's last piece (L % 16 == 12 at L = 300): no store touches the next row
            const cc_v3u v = {O[0], O[1], O[2]};
            if (nt)
                __builtin_amdgcn_raw_buffer_store_b96(v, ro, o, 0, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b96(v, ro, o, 0, 0);
        } else if (rem == 8) {
            const cc_v2u v = {O[0], O[1]};
            if (nt)
                __builtin_amdgcn_raw_buffer_store_b64(v, ro, o, 0, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b64(v, ro, o, 0, 0);
        } else {
            if (nt)
                __builtin_amdgcn_raw_buffer_store_b32(O[0], ro, o, 0, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b32(O[0], ro, o, 0, 0);
        }
    };

    // two chunks per lane per round, both chunks' loads issued before either is finished
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nchunks; i += 2 * stride) {
        ChunkLoads<G::NW> l0, l1;
        issue(i, l0);
        issue(i + stride, l1);
        finish(i, l0);
        finish(i + stride, l1);
    }
}

#define FEC_COPY_CHUNK_LIST(X) X(8, 3) X(8, 4) X(4, 7)

#define FEC_COPY_CHUNK_INST(K, NP) template __global__ void fec_copy_chunk_kernel<K, NP>(CopyChunkArgs);
FEC_COPY_CHUNK_LIST(FEC_COPY_CHUNK_INST)

const void* fec_copy_chunk_kernel_for(int k, int np) {
#define FEC_COPY_CHUNK_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_copy_chunk_kernel<K, NP>);
    FEC_COPY_CHUNK_LIST(FEC_COPY_CHUNK_CASE)
#undef FEC_COPY_CHUNK_CASE
    return nullptr;
}

}  // namespace fec
