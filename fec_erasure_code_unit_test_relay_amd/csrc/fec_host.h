// fec_host.h -- host-side control plane of the MI355X streaming-erasure codec.
//
// Everything here depends only on (T,B,N) and on the erasure pattern, never on payload bytes:
//   * GF(2^8) (poly 0x11d, generator 2 -- the field of Intel ISA-L's ec_base.c that the reference
//     links through gf_mul/gf_inv, src/basicOperations.cpp:18-24);
//   * the k x n systematic generator (gen_G_cauchy, src/codingOperations.cpp:48-95);
//   * DecodeRules: for every (window w, erasure mask) the outcome of the reference's per-symbol
//     decode (decodeBlock, src/codingOperations.cpp:149-232, built on gf256_rref_matrix,
//     src/basicOperations.cpp:43-122): which erased data symbols it declares recovered and with
//     which action-matrix column.  Built once per configuration, uploaded to HBM;
//   * StreamPlanner: a symbolic replica of the reference decoder state machine
//     (Decoder::decodeStream, src/Decoder.cpp:72-175; Decoder_Basic, src/Decoder_Basic.cpp:46-89;
//     Decoder_Block_Code::decodeSymbol, src/Decoder_Block_Code.cpp:61-78) that tracks, instead of
//     bytes, the GF coefficient vector of every stored symbol over the received symbols of its
//     diagonal codeword.  Because every sub-stream sees the same erasure flags
//     (src/Decoder.cpp:117-169), one symbolic run serves all S sub-streams; the GPU then applies
//     the coefficients to the bytes.  The same machine runs per erasure episode on the GPU
//     (fec_plan_kernel in fec_codec.hip); this host copy serves the per-packet drop-in API.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace fec {

constexpr int kMaxK = 16;   // k = T-N+1
constexpr int kMaxN = 32;   // n = k+B (erasure masks are 32-bit)
constexpr int kMaxRuleN = 17;  // decode-rule tables are built for n <= 17 (2^17 masks)

// ------------------------------------------------------------------------------------------
// GF(2^8)
// ------------------------------------------------------------------------------------------
struct Field {
    uint8_t exp[512];  // exp[i] = 2^(i mod 255)
    uint8_t log[256];  // log[0] unused
    uint8_t mt[256][256];  // mt[a][b] = a*b (host planners: one lookup per product)
    Field() {
        unsigned v = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = static_cast<uint8_t>(v);
            log[v] = static_cast<uint8_t>(i);
            v = (v << 1) ^ ((v & 0x80) ? 0x11d : 0);
            v &= 0x1ff;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
        for (int a = 0; a < 256; ++a)
            for (int b = 0; b < 256; ++b) mt[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const {
        return (a && b) ? exp[log[a] + log[b]] : 0;
    }
    uint8_t inv(uint8_t a) const { return a ? exp[255 - log[a]] : 0; }
};

const Field& field();

// ------------------------------------------------------------------------------------------
// Geometry: k, n, S sub-streams of k bytes each, CW = S*n untrimmed codeword bytes
// (Encoder.cpp:31-39, FEC_Encoder.cpp:29-31).
// ------------------------------------------------------------------------------------------
struct Geometry {
    int L = 0, T = 0, B = 0, N = 0, k = 0, n = 0, S = 0, CW = 0;
    static Geometry make(int max_payload, int T, int B, int N) {
        Geometry g;
        g.L = max_payload;
        g.T = T;
        g.B = B;
        g.N = N;
        g.k = T - N + 1;
        g.n = g.k + B;
        if (max_payload < 1 || T < 0 || B < 0 || N < 0 || g.k < 1 || g.k > kMaxK || g.n > kMaxN)
            throw std::invalid_argument("unsupported (max_payload,T,B,N)");
        g.S = (max_payload + 2 + g.k - 1) / g.k;
        g.CW = g.S * g.n;
        return g;
    }
};

// Systematic k x n generator (row-major): Cauchy1 (or the RS matrix for (10,8,4)/(11,5,4)),
// transposed, then the burst-structure zeros of gen_G_cauchy (codingOperations.cpp:48-95).
std::vector<uint8_t> make_generator(int T, int B, int N);

// Per parity coefficient G[i][k+jj] (index i*(n-k)+jj): the three register tables of gf_mul4x
// (fec_device.h) and a non-zero flag, 8 words each.
std::vector<uint32_t> parity_mul_tables(const std::vector<uint8_t>& G, int k, int n);

// ------------------------------------------------------------------------------------------
// Decode rules.  For window w (columns 0..w-1 of the current diagonal codeword) and erasure mask m
// (bit c = column c erased), entry = { sel[k] ; col[k][w] }: sel[i] = column j whose action-matrix
// column recovers erased data symbol i (0xFF = not recoverable), col[i][c] = that column's
// coefficient on codeword symbol c.
// ------------------------------------------------------------------------------------------
struct DecodeRules {
    int k = 0, n = 0, T = 0;
    int w_lo = 0;                      // smallest window that occurs: min(T+1, n)
    int entry_bytes = 0;               // k * (1 + n) rounded up to a multiple of 4
    std::vector<int64_t> w_base;       // byte offset of window w's table (index w; -1: no table)
    std::vector<uint8_t> table;
    // n > kMaxRuleN: no table (2^n masks); each (w, mask) that occurs is computed on first use
    // and kept (the device planner computes its own, fec_kernels.hip wave_rule)
    bool lazy = false;
    std::vector<uint8_t> G;
    // The whole symbolic decoder state right after a resynchronisation at time t >= T
    // (StreamPlanner::resync_at), per phase t mod n: the resync rewrites every symbol of every
    // diagonal block, so the state after it depends only on the phase (the device planner's
    // build_resync_states rests on the same fact).  Filled by build_resync; empty = replay.
    std::vector<uint8_t> resync_full;
    size_t resync_full_bytes = 0;
    void build(const std::vector<uint8_t>& G, int k, int n, int T);
    void build_resync();
    const uint8_t* entry(int w, uint32_t mask) const {
        if (lazy) return lazy_entry(w, mask);
        return table.data() + w_base[w] + static_cast<int64_t>(mask) * entry_bytes;
    }

private:
    const uint8_t* lazy_entry(int w, uint32_t mask) const;
    mutable std::mutex mu_;
    mutable std::unordered_map<uint64_t, std::unique_ptr<uint8_t[]>> cache_;
};

// The rule table of (T,B,N) (G = make_generator(T,B,N)), built once per process and shared by
// every codec, streaming decoder and variable-rate plan of that configuration (thread-safe).
std::shared_ptr<const DecodeRules> shared_decode_rules(int T, int B, int N);

// The rule for one (w, mask), computed directly (used to build the table and by tests).
void decode_rule(const uint8_t* G, int k, int n, int w, uint32_t mask, uint8_t* sel,
                 uint8_t* col /* k*w */);

// ------------------------------------------------------------------------------------------
// StreamPlanner: symbolic decoder.  Output of one step is the fate of packet x = t - T.
// ------------------------------------------------------------------------------------------
enum PacketFate : uint8_t {
    kNone = 0,       // x < 0: nothing to output yet (reference returns payload 0)
    kCopy = 1,       // received: systematic bytes of its own codeword (fast or slow path)
    kRecovered = 2,  // erased and recovered: rows coef[i][q], source = symbol q of packet x-i+q
    kLost = 3,       // erased and not recoverable: payload 0
};

struct StepResult {
    PacketFate fate = kNone;
    int64_t x = -1;
    bool slow = false;               // output produced by the block decoders (payload clamped)
    uint8_t coef[kMaxK * kMaxN];     // k rows of n coefficients (valid for kRecovered)
};

class StreamPlanner {
public:
    StreamPlanner(const Geometry& g, const DecodeRules* rules);
    // Feed packet t (t must increase by one per call starting at 0); erased = packet t missing.
    StepResult step(int64_t t, bool erased);
    int64_t latest_erasure() const { return latest_; }
    // True when a received packet t would take the fast path (Decoder.cpp:77-108): no erasure in
    // the last T packets.  Then every received packet up to the next erasure does too, and
    // skip_received(t, count) stands for count such steps (their outputs are kCopy once t >= T,
    // never slow): the block state is not touched on the fast path, only the flag ring is.
    bool fast_at(int64_t t) const { return latest_ == -1 || t - latest_ > T_; }
    void skip_received(int64_t t, int64_t count) {
        latest_ = -1;
        if (count >= T_ + 1) {
            std::fill(hist_.begin(), hist_.end(), uint8_t(0));
        } else {
            for (int64_t i = 0; i < count; ++i) hist_[(t + i) % (T_ + 1)] = 0;
        }
    }
    // The decoder's resynchronisation at erased packet t (Decoder.cpp:111-133) applied to the
    // current state, and a copy of one block's state (er mask, cwc[n][n], datc[k][n]).
    void resync_at(int64_t t);
    void block_state(int b, uint32_t* er, uint8_t* cwc, uint8_t* datc) const;
    // the block state of every diagonal (er, cwc, datc) as one byte image, and back
    size_t state_bytes() const { return er_.size() * 4 + cwc_.size() + datc_.size(); }
    void save_state(uint8_t* dst) const;
    void load_state(const uint8_t* src);

private:
    void feed(int64_t time, bool erased);
    void decode_symbol(int b, int p, bool erased);
    void decode_blocks(int b, int t0, int t1);
    void recover(int b, int w, uint32_t m);
    uint8_t* cw(int b, int p) { return &cwc_[(b * n_ + p) * n_]; }
    uint8_t* dat(int b, int i) { return &datc_[(b * k_ + i) * n_]; }

    int k_, n_, T_;
    const DecodeRules* rules_;
    std::vector<uint32_t> er_;     // per diagonal block: erased-position mask
    std::vector<uint8_t> cwc_;     // [b][p][q] coefficient of stored codeword symbol p on source q
    std::vector<uint8_t> datc_;    // [b][i][q] same for the recovered/received data symbol i
    std::vector<uint8_t> hist_;    // erasure flags of the last T+1 packets (ring)
    int64_t latest_ = -1;          // Decoder::latest_erasure_seq
    int memo_w_ = -1;              // the last (window, mask) whose decode recovered nothing
    uint32_t memo_m_ = 0;
};

// Post-resync state of one diagonal block for every phase phi = (t_resync - b) mod n, for resyncs
// at t >= T (all T replayed codewords exist), starting from the decoders' initial state.  Layout
// per phase (resync_state_bytes(g) bytes): uint32 er | cwc[n][n] | datc[k][n] | pad to 4.
int resync_state_bytes(const Geometry& g);
std::vector<uint8_t> build_resync_states(const Geometry& g, const DecodeRules& rules);

}  // namespace fec
