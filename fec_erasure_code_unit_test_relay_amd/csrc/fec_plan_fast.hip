// fec_plan_fast.hip -- the decode planner's per-(episode, diagonal) replay, specialised at compile
// time on k and n-k.
//
// Same algorithm and outputs as fec_plan_kernel (fec_kernels.hip): one wave replays one block
// (diagonal b) of the decoder through one loss episode on coefficient vectors and writes, for
// every symbol of an erased packet, whether it is recovered (sym_ok) and its coefficient row over
// the diagonal (coef).  Differences are in the organisation only:
//   * the block state lives in registers: lane q holds column q of cwc[n][n] and datc[k][n]
//     (the coefficient of round position q in every codeword / data symbol);
//   * decodeBlock (codingOperations.cpp:149-232) applies its precomputed rule with the rule's
//     coefficients in log form (0xff = zero): every term is one LDS exp-table read,
//     exp[log f + log v], with log 0 mapped past the table's non-zero range so that no term
//     branches; the n reads of a row are independent and overlap;
//   * the rule entry arrives in one wave-wide load and is read with constant-index v_readlane.
#include "fec_device.h"
#include "fec_kernels.h"

namespace fec {
namespace {

constexpr int kLogZero = 512;    // log of 0: any sum with it indexes the zero tail of ex[]
constexpr int kExBytes = 1040;   // ex[0..1024]

template <int K, int N>
struct RegReplay {
    const uint8_t* ex;           // LDS: ex[i] = 2^i for i < 512, 0 above
    const uint16_t* lg;          // LDS: lg[v] = log2 v, lg[0] = kLogZero
    const uint8_t* rules;        // log-form rule table
    const int64_t* wbase;
    int ES, T, lane;
    uint32_t er;                 // erased positions (uniform)
    uint32_t memo_key = ~0u;     // (w << 26 | m) of the last rule loaded (uniform)
    bool memo_none = false;      // ... and it recovered nothing
    uint32_t memo_ev = 0;        // ... its entry, one dword per lane
    uint32_t cw[N];              // lane q: cwc[p][q]
    uint32_t dat[K];             // lane q: datc[i][q]

    __device__ __forceinline__ void decode_block(int t) {
        if (t < K && !((er >> t) & 1u)) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i == t) dat[i] = cw[i];
        }
        const int w = min(t + T + 1, N);
        const uint32_t full = (1u << w) - 1u;
        const uint32_t m = er & full;
        if (m == full || !(m & ((1u << K) - 1u))) return;
        // The outcome (which symbols come back) is a function of (w, m) alone: a rule that
        // recovered nothing at (w, m) recovers nothing until the mask changes, and the entry of
        // the last (w, m) is still in ev.  Within a round the k blocks' decodes mostly see one mask,
        // so this saves most of the dependent rule loads of the serial replay.
        const uint32_t key = (static_cast<uint32_t>(w) << 26) | m;
        if (key == memo_key && memo_none) return;
        if (key != memo_key) {
            // entry {sel[K], logcol[K][N]} (K*(N+1) <= 256 bytes for every instantiation)
            const uint32_t* ent = reinterpret_cast<const uint32_t*>(rules + wbase[w] + static_cast<int64_t>(m) * ES);
            memo_ev = (lane < (ES >> 2)) ? ent[lane] : 0u;
            memo_key = key;
        }
        const uint32_t ev = memo_ev;
        uint32_t lv[N];
#pragma unroll
        for (int c = 0; c < N; ++c) lv[c] = lg[cw[c]];
        uint32_t fresh[K];
        uint32_t got = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            fresh[i] = 0;
            if (!((m >> i) & 1u)) continue;
            const uint32_t sel = (__builtin_amdgcn_readlane(ev, i >> 2) >> ((i & 3) * 8)) & 0xffu;
            if (sel == 0xffu) continue;
            uint32_t acc = 0;
#pragma unroll
            for (int c = 0; c < N; ++c) {
                const int idx = K + i * N + c;
                uint32_t lf = (__builtin_amdgcn_readlane(ev, idx >> 2) >> ((idx & 3) * 8)) & 0xffu;
                // columns at or past w are zero in the entry; erased columns never contribute
                lf = (lf == 0xffu || ((m >> c) & 1u)) ? static_cast<uint32_t>(kLogZero) : lf;
                acc ^= ex[lf + lv[c]];
            }
            fresh[i] = acc;
            got |= 1u << i;
        }
        memo_none = got == 0;
        if (!got) return;
#pragma unroll
        for (int i = 0; i < K; ++i)
            if ((got >> i) & 1u) {
                dat[i] = fresh[i];
                cw[i] = fresh[i];
            }
        er &= ~got;
    }

    // Decoder_Block_Code::decodeSymbol (Decoder_Block_Code.cpp:61-78) at position p.
    __device__ __forceinline__ void symbol(int p, bool erased) {
        if (erased) {
            er |= 1u << p;
        } else {
            er &= ~(1u << p);
#pragma unroll
            for (int c = 0; c < N; ++c)
                if (c == p) cw[c] = (lane == p) ? 1u : 0u;
        }
        if (p < T) return;
        const int j0 = p - T;
        const int j1 = (p == N - 1) ? max(K, j0 + 1) : j0 + 1;
        for (int j = j0; j < j1; ++j) decode_block(j);
    }

    __device__ void feed(int64_t time, int b, bool erased) {
        int p = static_cast<int>((time - b) % N);
        if (p < 0) p += N;
        symbol(p, erased);
    }
};

// Erasure flags of 256 consecutive packets, 4 per lane, read with v_readlane.
struct ErWin {
    const uint8_t* er;
    int P;
    int base = 0;
    uint32_t v = 0;
    int lane;
    __device__ void load(int b) {
        base = b;
        const int i = b + lane * 4;
        if (i >= 0 && i + 3 < P && ((reinterpret_cast<uintptr_t>(er + i) & 3) == 0)) {
            v = *reinterpret_cast<const uint32_t*>(er + i);
        } else {
            v = 0;
            for (int e = 0; e < 4; ++e)
                if (i + e >= 0 && i + e < P && er[i + e]) v |= 1u << (8 * e);
        }
    }
    __device__ bool get(int t) const {  // t in [base, base + 256)
        const int d = t - base;
        return ((__builtin_amdgcn_readlane(v, d >> 2) >> ((d & 3) * 8)) & 0xffu) != 0;
    }
};

}  // namespace

template <int K, int NP>
__global__ __launch_bounds__(64) void fec_plan_fast_kernel(PlanArgs a) {
    constexpr int N = K + NP;
    __shared__ uint8_t ex[kExBytes];
    __shared__ uint16_t lg[256];
    const int lane = threadIdx.x, T = a.T;
    for (int i = lane; i < kExBytes; i += 64) ex[i] = (i < 512) ? a.gf[i] : 0;
    for (int v = lane; v < 256; v += 64) lg[v] = v ? a.gf[512 + v] : static_cast<uint16_t>(kLogZero);
    __syncthreads();

    RegReplay<K, N> br;
    br.ex = ex;
    br.lg = lg;
    br.rules = a.rules;
    br.wbase = a.wbase;
    br.ES = a.ES;
    br.T = T;
    br.lane = lane;
    const int Pi = static_cast<int>(a.P), Pouti = static_cast<int>(a.Pout);  // P < 2^31 (host check)
    const int pairs = a.counters[6] * N;
    const int items = pairs + a.counters[7];
    for (int pr = blockIdx.x; pr < items; pr += gridDim.x) {
        if (pr >= pairs) {
            episode_dup_fill(a, pr - pairs, lane);
            continue;
        }
        const int ep = pr / N;
        const int b = pr - ep * N;
        const int tr = a.work[ep];
        if (tr < 0 || tr >= Pi) continue;
        if (tr >= T) {
            // resync at tr (Decoder.cpp:111-133) from the initial state, precomputed per phase
            int phi = (tr - b) % N;
            if (phi < 0) phi += N;
            const uint8_t* st = a.rstate + static_cast<int64_t>(phi) * a.rs_bytes;
            br.er = *reinterpret_cast<const uint32_t*>(st);
            const bool on = lane < N;
#pragma unroll
            for (int p = 0; p < N; ++p) br.cw[p] = on ? st[4 + p * N + lane] : 0u;
#pragma unroll
            for (int i = 0; i < K; ++i) br.dat[i] = on ? st[4 + N * N + i * N + lane] : 0u;
        } else {
            // startup: the replayed slots before packet 0 are empty (NULL); replay explicitly
#pragma unroll
            for (int p = 0; p < N; ++p) br.cw[p] = 0;
#pragma unroll
            for (int i = 0; i < K; ++i) br.dat[i] = 0;
            br.er = 0;
            for (int i = 0; i < N - T; ++i) br.feed(tr + i, b, true);
            for (int i = 0; i < T; ++i)
                if (tr - T + i >= 0) br.feed(tr - T + i, b, false);
        }
        ErWin win;
        win.er = a.er;
        win.P = Pi;
        win.lane = lane;
        win.load((tr - T) & ~3);
        // p = (t - b) mod N: position of packet t in this block's round;
        // ix = (t - T - b) mod N: position (symbol index) of the output packet x = t - T
        int p = (tr - b) % N;
        if (p < 0) p += N;
        int ix = (p - T) % N;
        if (ix < 0) ix += N;
        int latest = -1;
        for (int t = tr; t < Pi; ++t) {
            if (t >= win.base + 256) win.load((t - T) & ~3);
            const bool e = win.get(t);
            if (!e) {
                if (t - latest > T) break;  // Decoder.cpp:80-83: back to the fast path
            } else {
                latest = t;
            }
            br.symbol(p, e);
            const int x = t - T;
            const int i = ix;
            if (++p == N) p = 0;
            if (++ix == N) ix = 0;
            if (x < 0 || x >= Pouti || i >= K || !win.get(x)) continue;
            const bool ok = !((br.er >> i) & 1u);  // Decoder_Basic.cpp:76-79
            if (lane == 0) a.sym_ok[static_cast<int64_t>(x) * K + i] = ok ? 1 : 0;
            if (ok && lane < N) {
                uint32_t v = 0;
#pragma unroll
                for (int ii = 0; ii < K; ++ii) v = (ii == i) ? br.dat[ii] : v;
                a.coef[(static_cast<int64_t>(x) * K + i) * N + lane] = static_cast<uint8_t>(v);
            }
        }
    }
}

#define FEC_PLAN_FAST_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(1, 10) X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)

#define FEC_PLAN_FAST_INST(K, NP) template __global__ void fec_plan_fast_kernel<K, NP>(PlanArgs);
FEC_PLAN_FAST_LIST(FEC_PLAN_FAST_INST)

const void* fec_plan_fast_kernel_for(int k, int np) {
#define FEC_PLAN_FAST_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_plan_fast_kernel<K, NP>);
    FEC_PLAN_FAST_LIST(FEC_PLAN_FAST_CASE)
#undef FEC_PLAN_FAST_CASE
    return nullptr;
}

}  // namespace fec
