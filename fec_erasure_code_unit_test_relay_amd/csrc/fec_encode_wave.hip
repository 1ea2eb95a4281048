// fec_encode_wave.hip -- encode kernel with wave-private packet sequences, specialised on (k, n-k).
//
// Same closed form as every encode kernel here (fec_kernels.hip): for packet t, sub-stream s,
//     cw_t[s*n + j] = X_t[s][j]                                   j <  k
//     cw_t[s*n + j] = XOR_i G[i][j] * X_{t-(j-i)}[s][i]           j >= k
// with X_t[s] = bytes [s*k, s*k+k) of [len_hi, len_lo, payload, zero pad] (Encoder.cpp:65-98,
// Encoder_Basic.cpp:48-74, codingOperations.cpp:131-147).
//
// Organisation (no workgroup barrier after the one that publishes the coefficient tables):
//   * a lane owns one group of 4 sub-streams (g) of one packet SEQUENCE (M consecutive packets);
//     a wave holds 64 / NS4 sequences side by side and walks them in lockstep, one packet per
//     step, so the waves of a CU interleave freely and hide each other's memory latency;
//   * a lane reads its k+1 payload dwords of the packet straight from HBM (buffer loads: rows
//     before the stream start come back as zero, the encoder-creation semantics), prefetched one
//     packet pair ahead, and transposes them into k "position words" (byte e = position i of
//     sub-stream 4g+e) with constant-selector v_perm_b32;
//   * parity is accumulated FORWARD: position word i of packet t contributes G[i][k+jj] * word to
//     parity jj of packet t+(k+jj-i), i.e. into an (n-1)-slot register ring of accumulators; the
//     loop body is unrolled over n-1 packets so every ring index is a compile-time register;
//     a packet's parity is complete when its slot comes round.  GF products are gf_mul4x
//     (three v_perm_b32 table lookups, tables in LDS read as wave-wide broadcasts, one read per
//     coefficient per packet pair);
//   * the n codeword words of the group are re-interleaved with constant selectors and stored
//     straight to HBM (dword-aligned 16-byte stores: when a codeword row starts at a = t*CW mod 4
//     != 0 the words are shifted by a bytes and each lane takes its first a bytes from the lane to
//     its left, ds_bpermute; a sequence's lane 0 takes them from the previous packet's last lane);
//   * each sequence starts with an (n-1)-packet warm-up over the packets in front of it (no stores).
#include "fec_device.h"
#include "fec_kernels.h"

#include <utility>

namespace fec {
namespace {

constexpr int kWaveThreads = 256;
#ifndef FEC_TAB_AHEAD
#define FEC_TAB_AHEAD 2
#endif
constexpr int kTabAhead = FEC_TAB_AHEAD;  // coefficient tables are read this many (word, parity) items early

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x3a __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef uint32_t v3u32 __attribute__((ext_vector_type(3)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>), unrolled at compile time
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Materialise v here: stops the compiler from sinking its computation towards a far-away use
// (the accumulator ring is only read a whole block later), which would keep every table and
// selector of the block live at once.
__device__ __forceinline__ void pin(uint32_t& v) { asm volatile("" : "+v"(v)); }

struct Sel3 {
    uint32_t s0, s1, s2;
};
__device__ __forceinline__ Sel3 split_sel(uint32_t x) {
    return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}
// acc ^ c*x for the packed bytes of x (selectors s), c's tables t (0..3) and t4.  Both XORs are
// bitop3 intrinsics on purpose: plain XOR chains get reassociated across the whole unrolled block,
// which keeps every product of the block live at once.
__device__ __forceinline__ uint32_t mul_acc(uint32_t acc, const uint4& t, uint32_t t4, const Sel3& s) {
    uint32_t a = xor3(acc, __builtin_amdgcn_perm(t.y, t.x, s.s0), __builtin_amdgcn_perm(t.w, t.z, s.s1));
    pin(a);
    return a ^ __builtin_amdgcn_perm(t4, t4, s.s2);  // VOP2: half the issue cost of a bitop3
}

__device__ __forceinline__ uint32_t bperm(int src_lane, uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src_lane << 2, static_cast<int>(v)));
}

// payload dwords of one (packet, group): D[0] = dword gK-1 (the header slot for g = 0), D[1..K] =
// dwords gK .. gK+K-1 of the payload row
template <int K>
struct RowIn {
    uint32_t D[K + 1];
    int ln;  // payload length (0 = the packet does not exist: before the stream start)
};

template <int K>
__device__ __forceinline__ void load_row(RowIn<K>& r, __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rl,
                                         bool has_len, int voff_row, int lane_off, int row_rel, bool exists,
                                         int L) {
    const int o = voff_row + lane_off;  // byte offset of dword gK
    r.D[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, o - 4, 0, 0);
#pragma unroll
    for (int c = 0; c < K; c += 4) {
        if (c + 4 <= K) {
            const u32x4a v = __builtin_bit_cast(u32x4a, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 4 * c, 0, 0));
            r.D[1 + c] = v.x;
            r.D[2 + c] = v.y;
            r.D[3 + c] = v.z;
            r.D[4 + c] = v.w;
        } else if (c + 3 == K) {
            const u32x3a v = __builtin_bit_cast(u32x3a, __builtin_amdgcn_raw_buffer_load_b96(rs, o + 4 * c, 0, 0));
            r.D[1 + c] = v.x;
            r.D[2 + c] = v.y;
            r.D[3 + c] = v.z;
        } else if (c + 2 == K) {
            const u32x2a v = __builtin_bit_cast(u32x2a, __builtin_amdgcn_raw_buffer_load_b64(rs, o + 4 * c, 0, 0));
            r.D[1 + c] = v.x;
            r.D[2 + c] = v.y;
        } else {
            r.D[1 + c] = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4 * c, 0, 0);
        }
    }
    if (has_len) {
        const int v = static_cast<int>(__builtin_amdgcn_raw_buffer_load_b32(rl, row_rel * 4, 0, 0));
        r.ln = v < 0 ? 0 : (v > L ? L : v);
    } else {
        r.ln = exists ? L : 0;
    }
}

// Header, length mask and position words of one (packet, group).  H[m] = dword m of the group's
// 4K-byte window of [len_hi, len_lo, payload, 0 pad]; P[i] = position word i.  nvalid = payload
// dwords of the row from dword gK on (L/4 - gK): the dwords past the row end, which belong to the
// next packet, are zeroed (the window's zero pad).
template <int K>
__device__ __forceinline__ void row_words(const RowIn<K>& r, int g, int L, int nvalid, uint32_t (&H)[K],
                                          uint32_t (&P)[K]) {
    const uint32_t hdr = (static_cast<uint32_t>(r.ln & 0xff) << 24) | (static_cast<uint32_t>((r.ln >> 8) & 0xff) << 16);
    uint32_t D[K + 1];
    D[0] = g == 0 ? hdr : r.D[0];
#pragma unroll
    for (int m = 0; m < K; ++m) D[m + 1] = m < nvalid ? r.D[m + 1] : 0u;
#pragma unroll
    for (int m = 0; m < K; ++m) H[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], 2);
    if (r.ln == L) {
    } else if (r.ln > 0) {  // short packet: bytes at payload offsets >= ln are zero
        const int lim = r.ln + 2 - 4 * K * g;
#pragma unroll
        for (int m = 0; m < K; ++m) H[m] &= keep_bytes(lim - 4 * m);
    } else {  // empty or not-yet-existing packet: all zero, header included
#pragma unroll
        for (int m = 0; m < K; ++m) H[m] = 0;
    }
#pragma unroll
    for (int i = 0; i < K; ++i) P[i] = gather4(H, i, K + i, 2 * K + i, 3 * K + i);
}

// Codeword words of the group: bytes [e*n, e*n+n) = sub-stream 4g+e: K systematic bytes, NP parity.
template <int K, int NP>
__device__ __forceinline__ void group_words(const uint32_t (&H)[K], const uint32_t (&Q)[NP > 0 ? NP : 1],
                                            uint32_t (&X)[K + NP]) {
    constexpr int n = K + NP;
    uint32_t src[n];
#pragma unroll
    for (int m = 0; m < K; ++m) src[m] = H[m];
#pragma unroll
    for (int jj = 0; jj < NP; ++jj) src[K + jj] = Q[jj];
    auto idx = [](int b) {  // byte b of the group -> source byte index (word*4 + byte)
        const int e = b / n, j = b % n;
        return j < K ? (e * K + j) : (4 * (K + j - K) + e);
    };
#pragma unroll
    for (int q = 0; q < n; ++q) X[q] = gather4(src, idx(4 * q), idx(4 * q + 1), idx(4 * q + 2), idx(4 * q + 3));
}

// Last 4 valid bytes of the group's words (bytes [vb-4, vb)), vb = n * rem for the last group.
template <int n, int REM>
__device__ __forceinline__ uint32_t tail_word_rem(const uint32_t (&X)[n]) {
    constexpr int b = n * REM - 4;
    if constexpr (b < 0) {
        return X[0] << (8 * (4 - n * REM));
    } else if constexpr (b % 4 == 0) {
        return X[b / 4];
    } else {
        return __builtin_amdgcn_alignbyte(X[b / 4 + 1], X[b / 4], b % 4);
    }
}

// W[idx] for a runtime idx without indexing registers (idx >= n -> 0)
template <int n>
__device__ __forceinline__ uint32_t word_at(const uint32_t (&W)[n], int idx) {
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < n; ++q) r = q == idx ? W[q] : r;
    return r;
}

// Store `cnt` words W[0..cnt) at byte offset o (dword aligned) of the codeword resource.
template <int n>
__device__ __forceinline__ void store_words(__amdgpu_buffer_rsrc_t rc, int o, const uint32_t (&W)[n], int cnt) {
#pragma unroll
    for (int c = 0; c < n; c += 4) {
        const int w = (n - c) < 4 ? (n - c) : 4;
        if (c + w <= cnt) {
            if (w == 4) {
                u32x4a v = {W[c], W[c + 1 < n ? c + 1 : c], W[c + 2 < n ? c + 2 : c], W[c + 3 < n ? c + 3 : c]};
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), rc, o + 4 * c, 0, 0);
            } else if (w == 3) {
                u32x3a v = {W[c], W[c + 1 < n ? c + 1 : c], W[c + 2 < n ? c + 2 : c]};
                __builtin_amdgcn_raw_buffer_store_b96(__builtin_bit_cast(v3u32, v), rc, o + 4 * c, 0, 0);
            } else if (w == 2) {
                u32x2a v = {W[c], W[c + 1 < n ? c + 1 : c]};
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, v), rc, o + 4 * c, 0, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(W[c], rc, o + 4 * c, 0, 0);
            }
        } else {
#pragma unroll
            for (int q = c; q < c + w; ++q)
                if (q < cnt) __builtin_amdgcn_raw_buffer_store_b32(W[q], rc, o + 4 * q, 0, 0);
        }
    }
}

// Rare path (a codeword whose last byte is zero): trimmed size = 1 + position of the last non-zero
// byte over the sequence's lanes, reduced towards lane g = 0, which stores it.
template <int n>
__device__ __forceinline__ void slow_trim(const uint32_t (&X)[n], int g, int lane, int NS4, int last_g,
                                                    bool need, bool alive, __amdgpu_buffer_rsrc_t rw, int off,
                                                    uint32_t* lslot) {
    int z = -1;
#pragma unroll
    for (int q = n - 1; q >= 0; --q)
        if (z < 0 && X[q] != 0) z = 4 * q + 3 - (__builtin_clz(X[q]) >> 3);
    int best = z < 0 ? 0 : 4 * n * g + z + 1;
    for (int d = 1; d < NS4; d <<= 1) {
        const int src = (g + d < NS4) ? lane + d : lane;
        const int o = static_cast<int>(bperm(src, static_cast<uint32_t>(best)));
        best = o > best ? o : best;
    }
    const bool need0 = bperm(lane + last_g, need ? 1u : 0u) != 0;  // lane 0 asks its last lane
    if (alive && g == 0 && need0) {
        if (lslot)
            *lslot = static_cast<uint32_t>(best);
        else
            __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(best), rw, off, 0, 0);
    }
}

}  // namespace

template <int K, int NP>
__global__ __launch_bounds__(kWaveThreads, 4) void fec_encode_wave_kernel(EncWaveArgs a) {
    constexpr int n = K + NP;
    constexpr int W = n - 1;            // parity reaches back n-1 packets
    constexpr int NPA = NP > 0 ? NP : 1;
    __shared__ uint4 tabs[(K * NP > 0 ? K * NP : 1) * 2];
    for (int q = threadIdx.x; q < K * NP * 2; q += blockDim.x)
        tabs[q] = reinterpret_cast<const uint4*>(a.ptab)[q];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * (kWaveThreads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NS4 = a.NS4, SPW = a.SPW, M = a.M, L = a.L, CW = a.CW, P = a.P, hist = a.history;
    const int seq0 = wave * SPW;        // first sequence of the wave
    if (seq0 >= a.nseq) return;
    const int sq = lane / NS4;
    const int g = lane - sq * NS4;
    const bool alive = sq < SPW && seq0 + sq < a.nseq;
    const int r0 = (seq0 + sq) * M;     // first packet of the lane's sequence (batch-relative)
    const int last_g = NS4 - 1;

    // buffer resources built from kernel arguments only (provably wave-uniform).  Payload rows
    // [-history, P): rows outside read as zero -- the packets before the encoder's first one.
    // Codeword rows [0, P): stores outside are dropped.
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.payload_base), 0, a.payload_bytes, 0x00020000);
    const bool has_len = a.len_base != nullptr;
    const __amdgpu_buffer_rsrc_t rl =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(a.len_base), 0, a.len_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(a.cw, 0, a.cw_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(a.cw_len, 0, 4 * P, 0x00020000);
    const int lane_off = 4 * K * g;      // byte offset of dword gK in a payload row

    const int nvalid = (L >> 2) - K * g;  // payload dwords of the row from dword gK on

    // lane holding the group to the left (lane 0: the last group, i.e. the previous packet's tail)
    const int left = g == 0 ? lane + last_g : lane - 1;

    uint32_t acc[W][NPA];
#pragma unroll
    for (int u = 0; u < W; ++u)
#pragma unroll
        for (int jj = 0; jj < NPA; ++jj) acc[u][jj] = 0;
    uint32_t tsave = 0;  // lane 0 of a sequence: previous packet's tail word

    // W warm-up packets, the sequence's M packets, then at least one more: its lane 0 completes the
    // last packet's final partial dword (batch end)
    const int nblk = (M + W + 1 + W - 1) / W;

    auto load = [&](RowIn<K>& r, int s) __attribute__((always_inline)) {
        const int t = r0 - W + s;
        const int rel = t + hist;  // row index in the payload / length resources
        load_row<K>(r, rs, rl, has_len, rel * L, lane_off, rel, t >= -hist && t < P, L);
        if (t == P - 1 && 4 * (g * K + K) > L) {  // chunks straddling the buffer end: dword loads
            const int o = rel * L + lane_off;
#pragma unroll
            for (int m = 0; m < K; ++m) r.D[1 + m] = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4 * m, 0, 0);
        }
    };

    // one packet: its parity Q is complete; codeword words, stores, trimmed wire size
    // Output staging: each sequence's codewords form one contiguous byte stream in HBM, assembled
    // in a per-sequence LDS ring (absolute byte x at ring offset x & rmask) and flushed in
    // 16-byte aligned chunks; the chunks shared with the neighbouring sequences go out as dwords.
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int rmask = a.ring_bytes - 1;
    // Ring of sequence j of this wave.  Lane g of sequence j writes dword q of its group at bank
    // (A_j/4 + n*g + q) mod 64, and A_j - A_0 = j*M*CW.  With padding, sequence j is shifted so that
    // its lanes continue sequence j-1's bank run: lane (j, g) lands where lane NS4*j + g of one long
    // sequence would, and for odd n the 64 lanes then hit 64 different banks.
    const int wbase = (threadIdx.x >> 6) * (SPW + 1);  // first ring of this wave
    const int ring_stride = a.ring_bytes + (a.ring_pad ? 256 : 0);
    const int mcw64 = (((M & 255) * (CW & 255)) & 255) >> 2;  // (M*CW/4) mod 64 (M*CW % 4 == 0)
    auto ring_of = [&](int j) __attribute__((always_inline)) {
        const int pad = a.ring_pad ? ((NS4 * n * j - j * mcw64) & 63) : 0;
        return smem + (wbase + j) * ring_stride + pad * 4;
    };
    uint8_t* ring = ring_of(sq < SPW ? sq : SPW);
    // Trimmed sizes: a 32-entry LDS ring per sequence (slot t & 31), flushed to HBM one 64-byte
    // line of 16 packets at a time -- one size per packet stored straight to HBM would be one
    // partial-line write per packet (~32 MB of extra write traffic per 1M packets).
    const bool len_lds = !(a.dbg & 16);
    auto lring_of = [&](int j) __attribute__((always_inline)) {
        return reinterpret_cast<uint32_t*>(smem + 4 * (SPW + 1) * ring_stride + (wbase + j) * 128);
    };
    uint32_t* lring = lring_of(sq < SPW ? sq : SPW);
    const int A0 = r0 * CW;                                    // sequence start (4-byte aligned)
    int fl = A0;                                               // next byte to flush

    auto emit = [&](int s, const uint32_t (&H)[K], const uint32_t (&Q)[NPA]) __attribute__((always_inline)) {
        uint32_t X[n];
        group_words<K, NP>(H, Q, X);
        uint32_t tw = X[n - 1];
        if (g == last_g) {
            switch (a.rem) {
                case 1: tw = tail_word_rem<n, 1>(X); break;
                case 2: tw = tail_word_rem<n, 2>(X); break;
                case 3: tw = tail_word_rem<n, 3>(X); break;
                default: break;
            }
        }
        const uint32_t lv = bperm(left, tw);
        const uint32_t prev = g == 0 ? tsave : lv;
        tsave = lv;
        const int t = r0 - W + s;
        const int A = t * CW;
        // t % 4 = (s - W) % 4 for every lane: the alignment is wave-uniform
        const int al = (((s - W) & 3) * CW) & 3;
        const int o = A + 4 * n * g - al;  // dword-aligned; the lane covers [o, o + 4n)
        uint32_t Z[n];
        if (al == 0) {
#pragma unroll
            for (int q = 0; q < n; ++q) Z[q] = X[q];
        } else {
            const int sh = 4 - al;
            Z[0] = __builtin_amdgcn_alignbyte(X[0], prev, sh);
#pragma unroll
            for (int q = 1; q < n; ++q) Z[q] = __builtin_amdgcn_alignbyte(X[q], X[q - 1], sh);
        }
        // all n words, also past the row end for the last group: the next packet's words overwrite
        // them before they are flushed
#pragma unroll
        for (int q = 0; q < n; ++q) *reinterpret_cast<uint32_t*>(ring + ((o + 4 * q) & rmask)) = Z[q];
        // trimmed wire size (FEC_Encoder.cpp:55-60): fast path = the codeword's last byte is set
        const bool store = alive && s >= W && s < W + M && !(a.dbg & 1);  // s bounds are wave-uniform
        uint32_t lw = X[n - 1];
        switch (a.rem) {
            case 1: lw = tail_word_rem<n, 1>(X); break;
            case 2: lw = tail_word_rem<n, 2>(X); break;
            case 3: lw = tail_word_rem<n, 3>(X); break;
            default: break;
        }
        const bool full = (lw >> 24) != 0;
        if (store && g == last_g && full) {
            if (len_lds)
                lring[t & 31] = static_cast<uint32_t>(CW);
            else
                __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(CW), rw, 4 * t, 0, 0);
        }
        const bool need = store && g == last_g && !full;
        if (__builtin_amdgcn_ballot_w64(need))
            slow_trim<n>(X, g, lane, NS4, last_g, need, alive, rw, 4 * t, len_lds ? &lring[t & 31] : nullptr);
    };

    // Flush every sequence's final bytes below row srow (relative to the sequence start): all 64
    // lanes store one sequence at a time, so each store instruction covers one contiguous run.
    // The rows' last partial dwords are final only once the next row has been assembled.
    // dprev: rows since the previous flush (2 after a packet pair, 1 after a single packet).
    const int nseq_w = min(SPW, a.nseq - seq0);  // sequences of this wave (uniform)
    const int r0_last = (seq0 + nseq_w - 1) * M;
    const bool fast_fit = 2 * CW + 64 <= 16 * 64;   // a pair's chunks fit one store per sequence
    // Flush boundaries: 64-byte aligned (a line is written by one flush, not split across two
    // whose halves would reach HBM separately), except at the sequence's end.
    const int fmask = (a.dbg & 8) ? ~15 : ~63;
    auto flush_slow = [&](int srow) __attribute__((always_inline)) {
        for (int j = 0; j < nseq_w; ++j) {
            const int r0j = (seq0 + j) * M;
            const int Aendj = min(r0j + M, P) * CW;
            const int hi = min(((r0j + srow) * CW) & ~3, Aendj);
            int flj = __builtin_amdgcn_readlane(fl, j * NS4);
            if (hi <= flj) continue;
            const uint8_t* rj = ring_of(j);
            if (flj & 15) {  // sequence start inside a chunk: its dwords up to the chunk boundary
                const int e = min((flj + 15) & ~15, hi & ~3);
                const int x = flj + 4 * lane;
                if (x + 4 <= e)
                    __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(rj + (x & rmask)), rc, x, 0, 0);
                flj = e;
            }
            const int cend = hi == Aendj ? (hi & ~15) : (hi & fmask);
            for (int c = flj + 16 * lane; c < cend; c += 16 * 64) {
                const v4u32 v = *reinterpret_cast<const v4u32*>(rj + (c & rmask));
                __builtin_amdgcn_raw_buffer_store_b128(v, rc, c, 0, 0);
            }
            flj = max(flj, cend);
            if (hi == Aendj && flj < Aendj) {  // sequence end inside a chunk: dwords, bytes (batch end)
                const int x = flj + 4 * lane;
                if (x + 4 <= Aendj)
                    __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(rj + (x & rmask)), rc, x, 0, 0);
                const int b0 = Aendj & ~3;
                if (lane == 0 && b0 < Aendj) {
                    const uint32_t v = *reinterpret_cast<const uint32_t*>(rj + (b0 & rmask));
                    for (int b = 0; b < Aendj - b0; ++b)
                        __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v >> (8 * b)), rc, b0 + b, 0, 0);
                }
                flj = Aendj;
            }
            if (sq == j) fl = flj;
        }
    };
    // Trimmed sizes of the rows emitted so far: whole 16-packet groups (64-byte lines), and at the
    // sequence's end the rest.  Stateless: the previous flush ended at (r0j + srow - dprev) & ~15.
    auto flush_len = [&](int srow, int dprev) __attribute__((always_inline)) {
        if (!len_lds || (a.dbg & 1)) return;
        for (int j = 0; j < nseq_w; ++j) {
            const int r0j = (seq0 + j) * M;
            const int endj = min(r0j + M, P);
            const int lo = srow - dprev <= 0 ? r0j : max(r0j, (r0j + srow - dprev) & ~15);
            const int hi = r0j + srow >= endj ? endj : max(lo, (r0j + srow) & ~15);
            if (hi <= lo) continue;
            const int row = lo + lane;
            if (row < hi) __builtin_amdgcn_raw_buffer_store_b32(lring_of(j)[row & 31], rw, 4 * row, 0, 0);
        }
    };

    // Steady state (neither a sequence's first flush nor its last): sequence j's window is
    // [(r0j + srow - dprev) * CW & ~15, (r0j + srow) * CW & ~15), 16-byte chunks only, at most one
    // per lane.  Scalar addressing; the LDS reads of four sequences are issued before their stores.
    auto flush = [&](int srow, int dprev) __attribute__((always_inline)) {
        if (a.dbg & 1) return;
        flush_len(srow, dprev);
        if (!(fast_fit && srow - dprev >= 1 && srow < M && r0_last + srow < P)) {
            flush_slow(srow);
            return;
        }
        for (int j0 = 0; j0 < nseq_w; j0 += 4) {
            v4u32 v[4];
            int c[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = j0 + u;
                const int r0j = (seq0 + j) * M;
                const int lo = ((r0j + srow - dprev) * CW) & fmask;
                const int hi = ((r0j + srow) * CW) & fmask;
                c[u] = lo + 16 * lane;
                ok[u] = j < nseq_w && c[u] < hi;
                const uint8_t* rj = ring_of(j);
                v[u] = ok[u] ? *reinterpret_cast<const v4u32*>(rj + (c[u] & rmask)) : v4u32{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (ok[u]) __builtin_amdgcn_raw_buffer_store_b128(v[u], rc, c[u], 0, 0);
        }
        fl = ((r0 + srow) * CW) & fmask;
    };

    // One block = W packets: the accumulator ring comes round once, every slot index below is a
    // compile-time constant.  Packets go in pairs (tables read once per pair).  The first block
    // (WARM) covers the W packets in front of the sequence: it only accumulates the parity terms
    // that land on the sequence's own packets, and builds no codewords.  The walk ends after the
    // flush that reaches row M (uniform).
    bool done = false;
    RowIn<K> ra, rb, na;
    auto run_block = [&](auto warmc, int blk) __attribute__((always_inline)) {
        constexpr bool WARM = decltype(warmc)::value;
        static_for<(W + 1) / 2>([&](auto ic) __attribute__((always_inline)) {
            constexpr int U = 2 * decltype(ic)::value;
            constexpr bool TWO = U + 1 < W;
            if (!WARM && done) return;
            const int s = WARM ? U : blk * W + U;
            uint32_t QA[NPA], QB[NPA];
#pragma unroll
            for (int jj = 0; jj < NPA; ++jj) {
                QA[jj] = acc[U][jj];
                acc[U][jj] = 0;
                QB[jj] = 0;
            }
            // each row's registers are refilled with the packet two ahead as soon as its words are
            // built: (s+2, s+3) after a pair, s+2 after a single
            uint32_t PA[K], PB[K];
            {
                uint32_t HA[K];
                row_words<K>(ra, g, L, nvalid, HA, PA);
#pragma unroll
                for (int i = 0; i < K; ++i) pin(PA[i]);
                if constexpr (TWO) load(ra, s + 2);
                if constexpr (!WARM) emit(s, HA, QA);  // packet s's parity slot was complete before this step
            }
            __builtin_amdgcn_sched_barrier(0);
            uint32_t HB[K];
            if constexpr (TWO) {
                row_words<K>(rb, g, L, nvalid, HB, PB);
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    pin(PB[i]);
                    if constexpr (!WARM) pin(HB[i]);
                }
                load(rb, s + 3);
            } else {
                load(na, s + 2);
            }
            // parity contributions: K*NP (position word, parity) items in the order i = K-1..0,
            // jj = 0..NP-1; each item's tables are read from LDS kTabAhead items early
            if (!(a.dbg & 2)) {
                constexpr int NIT = K * NP;
                constexpr int NB = kTabAhead + 1;
                uint4 tb[NB];
                uint32_t t4b[NB];
                auto tload = [&](auto kc) __attribute__((always_inline)) {
                    constexpr int k = decltype(kc)::value;
                    constexpr int I = K - 1 - k / (NP > 0 ? NP : 1), JJ = k % (NP > 0 ? NP : 1);
#ifdef FEC_VAR_NOZ
                    const int z = 0;
#else
                    int z;
                    asm volatile("s_mov_b32 %0, 0" : "=s"(z));  // keeps the table reads in this step
#endif
                    tb[k % NB] = tabs[z + (I * NP + JJ) * 2];
                    t4b[k % NB] = tabs[z + (I * NP + JJ) * 2 + 1].x;
                };
                static_for<(kTabAhead < NIT ? kTabAhead : NIT)>([&](auto kc) __attribute__((always_inline)) { tload(kc); });
                Sel3 sa{0, 0, 0}, sb{0, 0, 0};
                static_for<NIT>([&](auto kc) __attribute__((always_inline)) {
                    constexpr int k = decltype(kc)::value;
                    constexpr int I = K - 1 - k / (NP > 0 ? NP : 1), JJ = k % (NP > 0 ? NP : 1);
                    // warm-up: only terms reaching packet W (the sequence's first) or later
                    constexpr bool NEEDA = !WARM || U + K + JJ - I >= W;
                    constexpr bool NEEDB = TWO && (!WARM || U + 1 + K + JJ - I >= W);
                    if constexpr (k + kTabAhead < NIT) tload(std::integral_constant<int, k + kTabAhead>{});
                    if constexpr (JJ == 0) {
                        sa = split_sel(PA[I]);
                        if constexpr (TWO) sb = split_sel(PB[I]);
                    }
                    const uint4 t = tb[k % NB];
                    const uint32_t t4 = t4b[k % NB];
                    constexpr int DA = (U + K + JJ - I) % W;
                    if constexpr (NEEDA) {
                        acc[DA][JJ] = mul_acc(acc[DA][JJ], t, t4, sa);
                        pin(acc[DA][JJ]);
                    }
                    if constexpr (TWO && I == K - 1 && JJ == 0) {
                        // packet s+1's slot is complete once packet s's delay-1 term is in
#pragma unroll
                        for (int j2 = 0; j2 < NPA; ++j2) {
                            QB[j2] = acc[(U + 1) % W][j2];
                            acc[(U + 1) % W][j2] = 0;
                        }
                    }
                    if constexpr (NEEDB) {
                        constexpr int DB = (U + 1 + K + JJ - I) % W;
                        acc[DB][JJ] = mul_acc(acc[DB][JJ], t, t4, sb);
                        pin(acc[DB][JJ]);
                    }
                });
            }
            if constexpr (TWO) {
                if constexpr (!WARM) {
                    emit(s + 1, HB, QB);
                    flush(s + 2 - W, 2);
                    done = s + 2 - W >= M;
                }
            } else {  // odd W: the next block's first pair is (s+1, s+2)
                if constexpr (!WARM) {
                    flush(s + 1 - W, 1);
                    done = s + 1 - W >= M;
                }
                ra = rb;
                rb = na;
            }
        });
    };

    load(ra, 0);
    load(rb, 1);
    run_block(std::true_type{}, 0);
    for (int blk = 1; blk < nblk && !done; ++blk) run_block(std::false_type{}, blk);
}

#ifdef FEC_WAVE_ONLY  // quick builds while tuning: -DFEC_WAVE_ONLY
#define FEC_ENC_WAVE_LIST(X) X(8, 3)
#else
#define FEC_ENC_WAVE_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)
#endif

#define FEC_ENC_WAVE_INST(K, NP) template __global__ void fec_encode_wave_kernel<K, NP>(EncWaveArgs);
FEC_ENC_WAVE_LIST(FEC_ENC_WAVE_INST)

const void* fec_encode_wave_kernel_for(int k, int np) {
#define FEC_ENC_WAVE_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_encode_wave_kernel<K, NP>);
    FEC_ENC_WAVE_LIST(FEC_ENC_WAVE_CASE)
#undef FEC_ENC_WAVE_CASE
    return nullptr;
}

}  // namespace fec
