// fec_session.hip -- the two-hop adaptive relay session (RELAYING_TYPE 2 / 3 with
// N_INITIAL = N_INITIAL_2 = -1: application_local_simulation.cpp:71-593, FLAG_FOR_CONSTANT_TRANS = 1).
//
// Control plane (host, symbolic).  Every decision of the session -- the sender's split of T_TOT
// over the two hops from the relay's 12-byte feedback (Application_Layer_Sender.cpp:75-198), the
// relay-mode Variable_Rate_FEC_Encoder's switches (Variable_Rate_FEC_Encoder.cpp:74-235), the
// estimators (Parameter_Estimator.cpp:58-186, T = T_TOT in relay mode), the relay's hop-2 code
// (Application_Layer_Receiver.cpp:142-164), the relay's and the destination's
// Variable_Rate_FEC_Decoder state machines (:542-948, :950-1601, :1603-1879) and the state-dependent
// selections (Decoder_Symbol_Wise.cpp:178-546) -- depends on the hop erasure patterns and headers
// only.  SessionPlan replays the loop with Decoder_Symbol_Wise objects whose slots hold references
// (a hop-1 packet's current or old part, a relay packet's part) instead of bytes, and records:
//   * the source's encoder instances (the batched variable-rate encoder, fec_vr.cpp) and the
//     16-byte hop-1 headers;
//   * per relay call a job (the GF symbols it computes from its window) and, per lineage -- an
//     object from its creation (fresh zero rows) through the copy_elements that hands its state to
//     the main object until the next copy replaces it -- the ordered calls that update its
//     codeword_new_vector rows and emit the word's part;
//   * per destination output a job (the main object's extract_data), the processed / flag bytes;
//   * the relay packets' layout (compact, host-known sizes) and their 8-byte headers, size fields
//     and state-dependent header rows.
// Byte work (device): the encoder launches, then three kernels -- ses_apply_kernel (every job's GF
// dot products over its window, data-parallel), ses_lineage_kernel (a workgroup per lineage: the
// codeword_new_vector rows in LDS, shifted per call, the call's symbols placed, the type-2 parity
// re-encoded from the earlier rows, the part stored), ses_prefix_kernel -- and the destination's
// jobs and loss check (calc_missed_chars, Variable_Rate_FEC_Decoder.cpp:2698-2792).
//
// Conventions (identical in oracle/fec_oracle.c or_relay_session_run): a slot holds the rest of
// the received packet from its pointer on, zero beyond; the GF methods use the generator of the
// call's own (k, n) / (k2, n2); the relay's erased-packet word has its full size; the loop runs Q
// seqs inside FLAG_FOR_CONSTANT_TRANS's range; hop-1 seq 0 must arrive; n2 > n selections read
// zero past the diagonal (type 3).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "fec_amd.h"
#include "fec_host.h"
#include "fec_vr.h"
#include "fec_status.h"

namespace fec {
int sd_relay_plan_state(int k, int n, int n2, int sdbo, const uint8_t* er, int* const* header, uint8_t* rec);
int sd_dest_plan_state(int k, int n, int* const* header, uint8_t* rec, bool* flag);

namespace {
constexpr int kST = 10;           // T_TOT (FEC_Macro.h:32)
constexpr int kSHdr = kST + 1;    // header entries per row / header bytes per word part
constexpr int kSSd = 3 * kST;     // codeword_vector_state_dependent rows
constexpr int kSCycle = 1000 / 10;  // ESTIMATION_WINDOW_SIZE / ..._REDUCTION_FACTOR (FEC_Macro.h:54-55)
constexpr int kSRow = 3344;       // an LDS row of codeword_new_vector: >= every part ((302+1)*11 = 3333)
constexpr int kSMaxN = 11;

// One apply job: out[j*ostride + o] = XOR_{p < nin} coef[o*nin + p] * slot(row(o, p))[base + j*bs + p]
// for j < blocks, o < nout, with row(o, p) = ref0 + rb0 - rstep*o + p (the window's rows) and
// slot(r)[x] = the referenced part's byte x - 2 (x >= 2; zero past the part's packet).
struct SesJob {
    int64_t out;
    int32_t ref0, coef;
    int16_t blocks;
    uint8_t nout, nin, bs, base, ostride, rstep;
    int8_t rb0;
    uint8_t pad[7];
};
static_assert(sizeof(SesJob) == 32, "SesJob layout");

// One call of a relay lineage: its symbols at d (blocks x nsym, from its job), the part (the first
// `size` bytes of codeword_new_vector[n2-1]) stored at out.
struct SesCall {
    int64_t d, out;
    int32_t size, g2;  // g2: offset of the type-2 parity coefficients [(n2-k) x k] in the coefficient table
    uint8_t k, n2, type, blocks_lo;
    int32_t blocks;
};
static_assert(sizeof(SesCall) == 32, "SesCall layout");

// Per seq: the relay packet's fixed bytes -- the 8-byte header (Application_Layer_Sender.cpp:317-330),
// the word's size field, and for type 3 the header rows of its parts.
struct SesPrefix {
    int64_t off;        // packet offset in the relay buffer
    int32_t size_first; // the word's BE16 field
    int16_t hdr2_at;    // offset (from the packet) of the second part's header row, 0 = none
    uint8_t type, pad;
    uint8_t hdr8[8];
    uint8_t hdr_a[kSHdr];
    uint8_t hdr_b[kSHdr];
    uint8_t pad2[2];
};
static_assert(sizeof(SesPrefix) == 48, "SesPrefix layout");

struct SymDsw {  // Decoder_Symbol_Wise (include/Decoder_Symbol_Wise.h) with references for bytes
    int64_t cv[kST + 1];
    uint8_t er[kST + 1];
    int64_t sd[kSSd];
    uint8_t sder[kSSd];
    int header[kSSd][kSHdr];
    int32_t lineage = -1;
    SymDsw() {
        for (auto& r : cv) r = -1;
        std::memset(er, 0, sizeof(er));
        for (auto& r : sd) r = -1;
        std::memset(sder, 0, sizeof(sder));
        for (int i = 0; i < kSSd; ++i)
            for (int j = 0; j < kSHdr; ++j) header[i][j] = j + 1;  // :60-62
    }
    void shift(int n) {  // push_current_codeword / rotate_pointers_and_insert_zero_word (:119-176)
        for (int i = 0; i < n - 1; ++i) {
            cv[i] = cv[i + 1];
            er[i] = er[i + 1];
        }
        for (int i = 0; i < kSSd - 1; ++i) {
            sd[i] = sd[i + 1];
            std::memcpy(header[i], header[i + 1], sizeof(int) * kST);  // entry T_TOT stays with its row
            sder[i] = sder[i + 1];
        }
    }
    void push(int64_t ref, int n) {
        shift(n);
        cv[n - 1] = ref;
        er[n - 1] = 0;
    }
    void rotate(int n) {
        shift(n);
        cv[n - 1] = -1;
        er[n - 1] = 1;
    }
};

struct Estimator {  // Parameter_Estimator, relay mode (T = T_TOT at every call, :72-75)
    int T = kST, B = 0, N = 0, N_max = 0, B_cur = 0, N_cur = 0;
    uint8_t erasure[12] = {};
    int64_t prev = -2;
    void estimate(int64_t seq, int msg_T) {
        if (T == 0) return;
        if (prev == -2) {
            T = msg_T;
            prev = seq - 1;
        }
        T = kST;
        if (seq - prev < 1) return;
        for (int64_t s = prev + 1; s <= seq; ++s) {
            for (int i = T; i >= 1; --i) erasure[i] = erasure[i - 1];
            erasure[0] = s < seq ? 1 : 0;
            int sum = 0;
            for (int i = 0; i <= T; ++i) sum += erasure[i] == 1;
            if (sum == T + 1 || sum == 0) continue;
            if (B == 0) B = 1;
            if (N == 0) N = 1;
            if (sum > N_max) N_max = sum;
            int i;
            for (i = 0; i <= T; ++i)
                if (erasure[i]) break;
            const int first = i;
            for (i = T; i >= 0; --i)
                if (erasure[i]) break;
            const int span = i - first + 1;
            if (span == T + 1) {
                if (sum > N) N = B = sum;
            } else {
                const int mbs = std::max(sum, B), mbp = std::max(span, B);
                if ((T - N + 1) * (T - sum + 1 + mbs) >= (T - sum + 1) * (T - N + 1 + mbp)) {
                    if (span > B) B = N = span;
                } else {
                    if (sum > N) N = B = sum;
                    if (N > B) B = N;
                }
            }
            if ((T - N_max + 1) * (T - N + 1 + B) > (T - N + 1) * (T + 1)) B = N = N_max;
        }
        prev = seq;
        if ((T - N_cur + 1) * (T - N + 1 + B) >= (T - N + 1) * (T - N_cur + 1 + B_cur)) {
            B_cur = B;
            N_cur = N;
        }
    }
};

struct VrdState {  // Variable_Rate_FEC_Decoder's relay / destination members
    int64_t seq_start = -1, latest = -1, sdc = -1, sde = -1;
    int T = 0, B = 0, N = 0, dcf = 0;
    int k_old = 0, n_old = 0, k2_old = 0, n2_old = 0, k_last = 0, n_last = 0, k2_last = 0, n2_last = 0;
    std::unique_ptr<SymDsw> main, nw;
    int64_t switches = 0, flags = 0;
};

int rd_size(int L, int k2, int n2) { return ((L + 2 + k2 - 1) / k2 + 1) * n2; }  // :997-999

}  // namespace

struct SessionPlan {
    int R = 2, L = 300;
    int64_t Q = 0;
    // source
    std::vector<VrInstance> enc;
    std::vector<uint8_t> hdr1;  // [Q][16]
    int64_t src_switches = 0;
    float rate1 = 0, rate1_curr = 0, min_rate = 0;
    int64_t rate1_n = 0;
    // relay
    std::vector<SesJob> rjobs;
    std::vector<int64_t> rrefs;   // hop-1 references: seq*2 + part, or -1
    std::vector<SesCall> calls;   // grouped by lineage, in call order
    std::vector<int64_t> lin;     // [nlin+1]: first call of each lineage
    std::vector<std::vector<SesCall>> lin_calls;
    int64_t d_bytes = 0;          // symbols of every relay call
    std::vector<SesPrefix> prefix;
    std::vector<int64_t> rpk_off;  // [Q+1] relay packets, compact
    int64_t relay_switches = 0, relay_flags = 0;
    // destination
    std::vector<SesJob> djobs;
    std::vector<int64_t> parts;   // [2 x parts]: a relay packet part's first byte and its packet's end (buffer offsets)
    std::vector<int32_t> djr;     // the destination jobs' window rows: part index, or -1 (zero row)
    std::vector<uint8_t> proc, dflag;
    int64_t dest_switches = 0, dest_flags = 0;
    float rate2 = 0, rate2_curr = 0;
    int64_t rate2_n = 0;
    // shared coefficient table
    std::vector<uint8_t> coef;
    std::map<std::string, int32_t> coef_ix;
    double control_ms = 0;

    int32_t intern(const uint8_t* c, size_t n) {
        std::string key(reinterpret_cast<const char*>(c), n);
        auto it = coef_ix.find(key);
        if (it != coef_ix.end()) return it->second;
        const int32_t at = static_cast<int32_t>(coef.size());
        coef.insert(coef.end(), c, c + n);
        coef_ix.emplace(std::move(key), at);
        return at;
    }
    void run(int relay_type, int max_payload, int64_t Q_, const uint8_t* e1, int64_t n1, const uint8_t* e2,
             int64_t n2);

private:
    int32_t next_lineage = 0;
    // memos of the per-call planning: a type-2 window's decode rows (by k, n, erasure mask), the
    // type-2 parity coefficients (by k, n2), a state-dependent call's record (by geometry, flags and
    // the header entries the selection reads)
    std::unordered_map<uint64_t, std::pair<int32_t, bool>> rows_memo_;
    std::unordered_map<uint32_t, int32_t> g2_memo_;
    std::unordered_map<std::string, std::pair<int32_t, std::vector<uint8_t>>> sd_memo_;
    std::string key_;
    std::vector<uint8_t> rec_;
    int32_t rows_coef(int k, int n, const uint8_t* er, bool* flag) {
        uint64_t mask = 0;
        for (int i = 0; i < n; ++i) mask |= static_cast<uint64_t>(er[i] ? 1 : 0) << i;
        const uint64_t key = static_cast<uint64_t>(k) | static_cast<uint64_t>(n) << 8 | mask << 16;
        auto it = rows_memo_.find(key);
        if (it == rows_memo_.end()) {
            uint8_t rows[kSMaxN * kSMaxN];
            bool f;
            decode_rows(k, n, er, rows, &f);
            it = rows_memo_.emplace(key, std::make_pair(intern(rows, static_cast<size_t>(k) * n), f)).first;
        }
        *flag = it->second.second;
        return it->second.first;
    }
    int32_t g2_coef(int k, int n2) {
        const uint32_t key = static_cast<uint32_t>(k) | static_cast<uint32_t>(n2) << 8;
        auto it = g2_memo_.find(key);
        if (it != g2_memo_.end()) return it->second;
        // parity position n2-1-delta = XOR_m G2[m][n2-1-delta] * row m+delta (:601-613)
        const std::vector<uint8_t> G2 = make_generator(n2 - 1, n2 - k, n2 - k);
        uint8_t g[kSMaxN * kSMaxN] = {};
        for (int delta = 0; delta < n2 - k; ++delta)
            for (int m = 0; m < k; ++m) g[delta * k + m] = G2[m * n2 + n2 - 1 - delta];
        const int32_t at = intern(g, static_cast<size_t>(std::max(1, (n2 - k) * k)));
        g2_memo_.emplace(key, at);
        return at;
    }
    std::unique_ptr<SymDsw> fresh() {
        std::unique_ptr<SymDsw> d(new SymDsw());
        d->lineage = next_lineage++;
        lin_calls.emplace_back();
        return d;
    }
    // the decode rows of a full-window decode (decodeBlock T = n-1, t = 0) for the window's flags,
    // output i = position k-1-i (symbol_wise_encode_1 :577-578, extract_data of decode_1 :647, :659)
    void decode_rows(int k, int n, const uint8_t* er, uint8_t* out, bool* flag) {
        int cnt = 0;
        uint32_t mask = 0;
        for (int i = 0; i < n; ++i) {
            cnt += er[i] ? 1 : 0;
            mask |= (er[i] ? 1u : 0u) << i;
        }
        *flag = cnt >= n - k + 1;
        uint8_t rows[kSMaxN * kSMaxN] = {};
        for (int q = 0; q < n; ++q) rows[q * n + q] = 1;
        if (cnt > 0 && cnt < n - k + 1) {
            const auto rules = shared_decode_rules(n - 1, n - k, n - k);
            const uint8_t* e = rules->entry(n, mask);
            for (int i = 0; i < k; ++i)
                if (((mask >> i) & 1u) && e[i] != 0xFF) std::memcpy(rows + i * n, e + k + i * n, static_cast<size_t>(n));
        }
        for (int i = 0; i < k; ++i) std::memcpy(out + i * n, rows + (k - 1 - i) * n, static_cast<size_t>(n));
    }
    // one relay object's GF call (symbol_wise_encode_1 / _state_dependent) after its slot update;
    // the part it emits goes to `out` (size bytes); type 3: its header row to *hdr
    int relay_call(SymDsw& o, int k, int n, int k2, int n2, int64_t out, int size, uint8_t* hdr, bool* flag);
    int dest_call(SymDsw& o, int k, int n, int64_t seq, bool* flag);
    int relay_erased(VrdState& d, int64_t seq, int64_t poff);
    int relay_received(VrdState& d, int64_t seq, int mT, int mB, int mN, int counter, int n, int k, int n2, int k2,
                       int64_t poff);
    int dest_received(VrdState& d, int64_t seq, int mT, int mB, int mN, int counter, int n, int k, int64_t poff,
                      int64_t wbytes, const SesPrefix& pf, int size_first);
    void dest_slot(SymDsw& o, int n, int64_t part_p, int64_t part_end, const int* hdr, SymDsw& memset_this);
    int emit(SymDsw& o, int k, int n, int64_t seq);
};

int SessionPlan::relay_call(SymDsw& o, int k, int n, int k2, int n2, int64_t out, int size, uint8_t* hdr,
                            bool* flag) {
    if (k2 != k || n > kSMaxN || n2 > kSMaxN || n2 < k) return FEC_ERR_ARG;
    const int blocks = L / k + 1;  // :553 / :184-185
    SesJob j{};
    j.blocks = static_cast<int16_t>(blocks);
    j.bs = static_cast<uint8_t>(n);
    j.base = 2;
    j.ref0 = static_cast<int32_t>(rrefs.size());
    SesCall c{};
    c.d = d_bytes;
    c.out = out;
    c.size = size;
    c.k = static_cast<uint8_t>(k);
    c.n2 = static_cast<uint8_t>(n2);
    c.type = static_cast<uint8_t>(R);
    c.blocks = blocks;
    if (R == 2) {
        for (int m = 0; m < n; ++m) rrefs.push_back(o.cv[m]);
        j.nout = static_cast<uint8_t>(k);
        j.nin = static_cast<uint8_t>(n);
        j.ostride = static_cast<uint8_t>(k);
        j.coef = rows_coef(k, n, o.er, flag);
        c.g2 = g2_coef(k, n2);
        d_bytes += static_cast<int64_t>(blocks) * k;
    } else {
        *flag = false;  // the relay's flag is never set (:195)
        // the selection reads the window's flags (slots lo..2T) and header rows 0..n2-1 (rows
        // 0..n2-2: entries < n2-1, row n2-1: rewritten entries < n2, the rest carried into the record)
        const int lo = 2 * kST - n + 1 - (n2 - k);
        key_.assign(1, static_cast<char>(k));
        key_.push_back(static_cast<char>(n));
        key_.push_back(static_cast<char>(n2));
        for (int r = lo; r <= 2 * kST; ++r) key_.push_back(static_cast<char>(o.sder[r]));
        for (int r = 0; r < n2; ++r)
            for (int e = 0; e < kSHdr; ++e) key_.push_back(static_cast<char>(o.header[r][e]));
        auto it = sd_memo_.find(key_);
        if (it == sd_memo_.end()) {
            int* rows[kSSd];
            for (int i = 0; i < kSSd; ++i) rows[i] = o.header[i];
            rec_.assign(static_cast<size_t>(kSHdr + n2 * n), 0);
            if (int st = sd_relay_plan_state(k, n, n2, 0, o.sder, rows, rec_.data())) return st;
            const int32_t at = intern(rec_.data() + kSHdr, static_cast<size_t>(n2) * n);
            it = sd_memo_.emplace(key_, std::make_pair(at, std::vector<uint8_t>(rec_.begin(), rec_.begin() + kSHdr)))
                     .first;
        }
        const std::vector<uint8_t>& hrow = it->second.second;
        for (int i = 0; i < n2; ++i) o.header[n2 - 1][i] = hrow[static_cast<size_t>(i)];  // (the planner's write-back)
        std::memcpy(hdr, hrow.data(), kSHdr);
        // window rows: output o, position p reads slot lo + (n2-1-o) + p (p < n - symInd; the
        // coefficients past the partial diagonal are zero, so rows past slot 2*T_TOT are never read)
        for (int r = lo; r < lo + n2 + n - 1; ++r) rrefs.push_back(r <= 2 * kST ? o.sd[r] : -1);
        j.nout = static_cast<uint8_t>(n2);
        j.nin = static_cast<uint8_t>(n);
        j.ostride = static_cast<uint8_t>(n2);
        j.rb0 = static_cast<int8_t>(n2 - 1);  // output o: the diagonal of symInd = k-1-o
        j.rstep = 1;
        j.coef = it->second.first;
        c.g2 = 0;
        d_bytes += static_cast<int64_t>(blocks) * n2;
    }
    j.out = c.d;
    rjobs.push_back(j);
    lin_calls[static_cast<size_t>(o.lineage)].push_back(c);
    return FEC_OK;
}

// :542-948 (constant transmission)
int SessionPlan::relay_erased(VrdState& d, int64_t seq, int64_t poff) {
    const int n = d.n_last, k = d.k_last, n2 = d.n2_last, k2 = d.k2_last;
    if (d.seq_start == -1) return FEC_ERR_ARG;
    bool flag = false;
    if (seq > d.sde && d.dcf == 1) {  // :605-616
        d.dcf = 0;
        *d.main = *d.nw;
        d.n2_old = d.n2_last;
        d.k2_old = d.k2_last;
    }
    if (seq == d.sdc) {  // :619-633
        d.sde = d.sdc + kST;
        d.k_old = d.T - d.N + 1;
        d.n_old = d.T + 1;
        d.T = d.B = d.N = 0;
        d.nw = fresh();
        d.dcf = 1;
        ++d.switches;
    }
    const int hb = R == 3 ? kSHdr : 0;
    SesPrefix& pf = prefix[static_cast<size_t>(seq)];
    const int size_first = rd_size(L, k2, n2);
    int64_t at = poff + 10;
    if (d.dcf == 0) {  // :636-684
        d.main->rotate(n);
        if (R == 3) {
            d.main->sd[2 * kST] = -1;
            d.main->sder[2 * kST] = 1;
        }
        if (int st = relay_call(*d.main, k, n, k2, n2, at + hb, size_first, pf.hdr_a, &flag)) return st;
        d.flags += flag;
        at += hb + size_first;
    } else {  // :685-761
        d.main->rotate(d.n_old);
        if (R == 3) {
            d.main->sd[2 * kST] = -1;
            d.main->sder[2 * kST] = 1;
        }
        const int size_old = rd_size(L, d.k2_old, d.n2_old);
        const int64_t at_old = at + hb + size_first + hb;
        if (int st = relay_call(*d.main, d.k_old, d.n_old, d.k2_old, d.n2_old, at_old, size_old, pf.hdr_b, &flag))
            return st;
        d.flags += flag;
        d.nw->rotate(n);
        if (R == 3) {
            d.main->sd[2 * kST] = -1;  // :702-704: the main object's slot, as written
            d.nw->sder[2 * kST] = 1;
        }
        bool f2;
        if (int st = relay_call(*d.nw, k, n, k2, n2, at + hb, size_first, pf.hdr_a, &f2)) return st;
        pf.hdr2_at = static_cast<int16_t>(10 + hb + size_first);
        at = at_old + size_old;
    }
    pf.size_first = size_first;
    d.latest = seq + 1;
    return static_cast<int>(at - poff);
}

// :950-1601 for a received hop-1 packet in sequence
int SessionPlan::relay_received(VrdState& d, int64_t seq, int mT, int mB, int mN, int counter, int n, int k, int n2,
                                int k2, int64_t poff) {
    if (d.seq_start == -1) {  // :952-967
        d.T = mT;
        d.B = mB;
        d.N = mN;
        d.seq_start = 0;
        d.latest = 0;
        d.n_old = n;
        d.k2_old = k2;
        d.n2_old = n2;
        d.k2_last = k2;
        d.n2_last = n2;
    }
    if (seq != d.latest) return FEC_ERR_SEQUENCE;
    if (d.T != mT || d.B != mB || d.N != mN) d.sdc = seq - counter;  // :975-978
    bool flag = false;
    if (seq > d.sde && d.dcf == 1) {  // :1423-1434
        d.dcf = 0;
        *d.main = *d.nw;
        d.n_old = n;
        d.n2_old = n2;
        d.k2_old = k2;
    }
    if (seq == d.sdc) {  // :1437-1456
        d.sde = d.sdc + kST;
        d.k_old = d.T - d.N + 1;
        d.n_old = d.T + 1;
        if (d.k2_old != d.k_old) {
            d.n2_old = kST - d.N + 1;
            d.k2_old = d.T - d.N + 1;
        }
        d.T = mT;
        d.B = mB;
        d.N = mN;
        d.nw = fresh();
        d.dcf = 1;
        ++d.switches;
    }
    const int hb = R == 3 ? kSHdr : 0;
    SesPrefix& pf = prefix[static_cast<size_t>(seq)];
    const int size_cur = rd_size(L, k2, n2);
    const int64_t ref_cur = seq * 2, ref_old = seq * 2 + 1;
    int64_t at = poff + 10;
    if (d.dcf == 0) {  // :1458-1501
        d.main->push(ref_cur, n);
        if (R == 3) {
            d.main->sd[2 * kST] = ref_cur;
            d.main->sder[2 * kST] = 0;
        }
        if (int st = relay_call(*d.main, k, n, k2, n2, at + hb, size_cur, pf.hdr_a, &flag)) return st;
        d.flags += flag;
        at += hb + size_cur;
    } else {  // :1502-1588
        d.main->push(ref_old, d.n_old);
        if (R == 3) {
            d.main->sd[2 * kST] = ref_old;
            d.main->sder[2 * kST] = 0;
        }
        const int size_old = rd_size(L, d.k2_old, d.n2_old);
        const int64_t at_old = at + hb + size_cur + hb;
        if (int st = relay_call(*d.main, d.k_old, d.n_old, d.k2_old, d.n2_old, at_old, size_old, pf.hdr_b, &flag))
            return st;
        d.flags += flag;
        d.nw->push(ref_cur, n);
        if (R == 3) {
            d.nw->sd[2 * kST] = ref_cur;
            d.nw->sder[2 * kST] = 0;
        }
        bool f2;
        if (int st = relay_call(*d.nw, k, n, k2, n2, at + hb, size_cur, pf.hdr_a, &f2)) return st;
        pf.hdr2_at = static_cast<int16_t>(10 + hb + size_cur);
        at = at_old + size_old;
    }
    pf.size_first = size_cur;
    d.latest = seq + 1;
    d.k_last = k;
    d.n_last = n;
    d.k2_last = k2;
    d.n2_last = n2;
    return static_cast<int>(at - poff);
}

// the destination's slot update for one seq: a received part [part_p, part_end) of a relay
// packet, or none (part_p < 0)
void SessionPlan::dest_slot(SymDsw& o, int n, int64_t part_p, int64_t part_end, const int* hdr, SymDsw& memset_this) {
    if (part_p >= 0) {
        const int64_t ix = static_cast<int64_t>(parts.size() / 2);
        parts.push_back(part_p);
        parts.push_back(part_end);
        o.push(ix, n);
        if (R == 3) {
            for (int i = 0; i < kSHdr; ++i) o.header[kSSd - 1][i] = hdr[i];
            o.sd[kSSd - 1] = ix;
            o.sder[kSSd - 1] = 0;
        }
    } else {
        o.rotate(n);
        if (R == 3) {
            for (int i = 0; i < kSHdr; ++i) o.header[kSSd - 1][i] = 0;
            memset_this.sd[kSSd - 1] = -1;  // :1759 zeroes the main object's slot
            o.sder[kSSd - 1] = 1;
        }
    }
}

// the main object's decode + extract_data (:653-661) for seq: an output row of the destination
int SessionPlan::emit(SymDsw& o, int k, int n, int64_t seq) {
    const int blocks = L / k + 1;  // :632 / :494
    if (blocks * k > 320 || n > kSMaxN) return FEC_ERR_ARG;
    SesJob j{};
    j.blocks = static_cast<int16_t>(blocks);
    j.bs = static_cast<uint8_t>(n);
    j.base = 4;  // symbol (block j, position q) at slot byte 4 + j*n + q (:636-639, :504)
    j.nout = static_cast<uint8_t>(k);
    j.nin = static_cast<uint8_t>(n);
    j.ostride = static_cast<uint8_t>(k);
    j.out = seq * 320;
    j.ref0 = static_cast<int32_t>(djr.size());
    bool flag = false;
    if (R == 2) {
        for (int m = 0; m < n; ++m) djr.push_back(static_cast<int32_t>(o.cv[m]));
        j.coef = rows_coef(k, n, o.er, &flag);
    } else {
        // the decode reads header entries < n of rows lo..3T-1 (:501-508)
        const int lo = kSSd - 1 - (k - 1) - (n - 1);
        key_.assign(1, static_cast<char>(k | 0x40));
        key_.push_back(static_cast<char>(n));
        for (int r = lo; r < kSSd; ++r)
            for (int e = 0; e < n; ++e) key_.push_back(static_cast<char>(o.header[r][e]));
        auto it = sd_memo_.find(key_);
        if (it == sd_memo_.end()) {
            int* rows[kSSd];
            for (int i = 0; i < kSSd; ++i) rows[i] = o.header[i];
            rec_.assign(static_cast<size_t>(k) * n, 0);
            if (int st = sd_dest_plan_state(k, n, rows, rec_.data(), &flag)) return st;
            it = sd_memo_.emplace(key_, std::make_pair(intern(rec_.data(), rec_.size()),
                                                       std::vector<uint8_t>(1, flag ? 1 : 0))).first;
        }
        flag = it->second.second[0] != 0;
        for (int r = lo; r < kSSd; ++r) djr.push_back(static_cast<int32_t>(o.sd[r]));
        j.rb0 = static_cast<int8_t>(k - 1);  // output ks: frames t2-ks-(n-1-q) (:501-508)
        j.rstep = 1;
        j.coef = it->second.first;
    }
    djobs.push_back(j);
    proc[static_cast<size_t>(seq)] = 1;
    dflag[static_cast<size_t>(seq)] = flag ? 1 : 0;
    dest_flags += flag;
    rate2_curr = static_cast<float>(k) / n;  // :1722-1724
    rate2 += static_cast<float>(k) / n;
    ++rate2_n;
    return FEC_OK;
}

// :1603-1879 for a received relay packet at buffer offset poff (wbytes of word after its 8-byte header)
int SessionPlan::dest_received(VrdState& d, int64_t seq, int mT, int mB, int mN, int counter, int n, int k,
                               int64_t poff, int64_t wbytes, const SesPrefix& pf, int size_received) {
    if (d.seq_start == -1) {  // :1607-1621
        d.T = mT;
        d.B = mB;
        d.N = mN;
        d.seq_start = 0;
        d.latest = 0;
        d.k_old = k;
        d.n_old = n;
        d.k_last = k;
        d.n_last = n;
    }
    if (seq < d.latest) return FEC_OK;
    int transition_flag = 0;
    if (d.T != mT || d.B != mB || d.N != mN) {  // :1629-1636
        d.sdc = counter > 128 ? seq - (counter - 255) : seq - counter;
        transition_flag = 1;
    }
    const int hb = R == 3 ? kSHdr : 0;
    const int64_t wend = poff + 8 + wbytes;
    const int64_t cwr = poff + 8 + 2 + hb, cwt = cwr + size_received + hb;
    int new_header[kSHdr], new_header_trans[kSHdr];
    for (int i = 0; i < kSHdr; ++i) {
        new_header[i] = pf.hdr_a[i];  // :1663-1664
        new_header_trans[i] = pf.hdr2_at ? pf.hdr_b[i] : 0;  // :1653-1654 (zero past the word)
    }
    for (int64_t s = d.latest; s < seq; ++s) {  // :1671-1769
        if (s > d.sde && d.dcf == 1) {
            d.dcf = 0;
            *d.main = *d.nw;
            d.n_last = n;
            d.k_last = k;
        }
        if (s == d.sdc) {
            d.sde = d.sdc + kST;
            d.k_old = d.T - d.N + 1;
            d.n_old = d.T + 1;
            d.T = mT;
            d.B = mB;
            d.N = mN;
            transition_flag = 0;
            d.nw.reset(new SymDsw());
            d.dcf = 1;
            ++d.switches;
        }
        if (d.dcf == 0) {
            dest_slot(*d.main, d.n_last, -1, 0, nullptr, *d.main);
            if (int st = emit(*d.main, d.k_last, d.n_last, s)) return st;
        } else {
            dest_slot(*d.main, d.n_old, -1, 0, nullptr, *d.main);
            if (int st = emit(*d.main, d.k_old, d.n_old, s)) return st;
            dest_slot(*d.nw, n, -1, 0, nullptr, *d.main);
        }
    }
    if (seq > d.sde && d.dcf == 1) {  // :1772-1781
        d.dcf = 0;
        *d.main = *d.nw;
        d.n_last = n;
        d.k_last = k;
    }
    if (seq == d.sdc || (seq >= d.sdc && transition_flag == 1)) {  // :1783-1796
        d.sde = d.sdc + kST;
        d.k_old = d.T - d.N + 1;
        d.n_old = d.T + 1;
        d.T = mT;
        d.B = mB;
        d.N = mN;
        d.nw.reset(new SymDsw());
        d.dcf = 1;
        ++d.switches;
    }
    if (d.dcf == 0) {  // :1798-1822
        dest_slot(*d.main, d.n_last, cwr, wend, new_header, *d.main);
        if (int st = emit(*d.main, d.k_last, d.n_last, seq)) return st;
    } else {  // :1823-1873
        // (a single-part word: the old part starts at or past the word's end and reads as zeros,
        // still a received slot)
        dest_slot(*d.main, d.n_old, cwt, wend, new_header_trans, *d.main);
        if (int st = emit(*d.main, d.k_old, d.n_old, seq)) return st;
        dest_slot(*d.nw, n, cwr, wend, new_header, *d.main);
    }
    d.latest = seq + 1;
    return FEC_OK;
}

void SessionPlan::run(int relay_type, int max_payload, int64_t Q_, const uint8_t* e1, int64_t n1, const uint8_t* e2,
                      int64_t n2) {
    const auto t0 = std::chrono::steady_clock::now();
    R = relay_type;
    L = max_payload;
    Q = Q_;
    if ((R != 2 && R != 3) || L < 1 || L > 300 || Q < 1) throw std::invalid_argument("session arguments");
    if (n1 > 0 && e1[0]) throw std::invalid_argument("hop-1 seq 0 erased");
    hdr1.assign(static_cast<size_t>(Q) * 16, 0);
    prefix.assign(static_cast<size_t>(Q), SesPrefix{});
    rpk_off.assign(static_cast<size_t>(Q) + 1, 0);
    proc.assign(static_cast<size_t>(Q), 0);
    dflag.assign(static_cast<size_t>(Q), 0);
    // ---- source: Application_Layer_Sender (T = T_TOT, B = N = -1, :9-53) and its relay-mode
    // Variable_Rate_FEC_Encoder (T2 = T_TOT, N2 = B2 = 0: application_local_simulation.cpp:136-143)
    int sT = kST, sN = 0, sT_ack = kST, sB_ack = 0, sN_ack = 0, sN2 = 0;
    struct {
        bool live = false;
        int T = 0, B = 0, N = 0, T_old = 0, N_old = 0, T2 = kST, B2 = 0, N2 = 0, T2_old = 0, N2_old = 0;
        int counter = 0, transition = 1, dcf = 1;
    } v;
    uint8_t udp[12] = {}, udp2[6] = {};
    // ---- relay receiver (Application_Layer_Receiver.cpp:10-39) ----
    std::unique_ptr<Estimator> est(new Estimator()), bg(new Estimator());
    int64_t cycle = 1, last_received = -1;
    bool first_call = true;
    int T_s_r = 0, N_s_r = 0, stale_counter = 0;
    int n2_new = kST + 1, k2_new = kST + 1;  // application_local_simulation.cpp:316-324
    VrdState relay;
    relay.main = fresh();
    // ---- destination ----
    std::unique_ptr<Estimator> dest(new Estimator()), dbg(new Estimator());
    int64_t dcycle = 1;
    VrdState dst;
    dst.main.reset(new SymDsw());
    for (int64_t i = 0; i < Q; ++i) {
        // ---- source, Application_Layer_Sender.cpp:64-282 ----
        if (udp[0] != 0) {
            sT = udp[0];
            sN = udp[2];
            sT_ack = udp[3];
            sB_ack = udp[4];
            sN_ack = udp[5];
            sN2 = udp[8];
        }
        if (i > 0) {  // :109-198 (DOUBLE_ERAUSRE_NUM = 1, MIN_T2 = MIN_N2 = SPLIT_PROP = 0)
            sN = std::min(sN, kST);
            sN2 = std::min(sN2, kST);
            if (sN + sN2 <= kST) {
                sT = kST - sN2;
                if (sT >= 1) {
                    v.N2 = v.B2 = sN2;
                } else {
                    sT = 1;
                    sN2 = kST - sT;
                    sN = std::min(sN, sT);
                    v.N2 = v.B2 = sN2;
                }
            } else {
                sN = sN_ack;
                sT = sT_ack;
            }
        }
        int mT = sT, mB = sN, mN = sN, counter;  // set_parameters(seq, T, N, N) :200-201
        // Variable_Rate_FEC_Encoder::encode, :74-235
        if (!v.live) {
            v.live = true;
            v.T = mT;
            v.B = mB;
            v.N = mN;
            v.transition = 1;
            v.dcf = 0;
            enc.push_back(VrInstance{v.T, v.B, v.N, i, Q, Q});
        } else if ((mT != v.T || mB != v.B || mN != v.N) && v.transition == 0 && sT_ack == v.T && sB_ack == v.B) {
            ++src_switches;
            v.T_old = v.T;
            v.N_old = v.N;
            v.T = mT;
            v.B = mB;
            v.N = mN;
            v.T2_old = v.T2;
            v.N2_old = v.N2;
            v.T2 = kST - v.N;
            v.transition = 1;
            v.dcf = 1;
            v.counter = 0;
            VrInstance& prev = enc.back();
            prev.role_switch = i;
            prev.end = std::min(Q, i + kST + 1);  // the old encoder's T_TOT + 1 double-coded packets
            enc.push_back(VrInstance{v.T, v.B, v.N, i, Q, Q});
        } else {
            mT = v.T;
            mB = v.B;
            mN = v.N;
        }
        ++rate1_n;  // onReceivedMessage, :368-374
        rate1_curr = static_cast<float>(mT - mN + 1) / (mT + 1);
        rate1 += static_cast<float>(mT - mN + 1) / (mT + 1);
        counter = v.counter;
        if (v.counter <= kST + 1) {
            if (v.counter == kST + 1) v.dcf = 0;
            ++v.counter;
        } else {
            v.transition = 0;
            ++v.counter;
        }
        uint8_t* h = &hdr1[static_cast<size_t>(i) * 16];  // :222-244
        h[15] = static_cast<uint8_t>(v.N2_old);
        h[14] = static_cast<uint8_t>(v.T2_old);
        h[13] = static_cast<uint8_t>(v.N_old);
        h[12] = static_cast<uint8_t>(v.T_old);
        h[11] = static_cast<uint8_t>(counter);
        h[10] = static_cast<uint8_t>(v.N2);
        h[9] = static_cast<uint8_t>(v.B2);
        h[8] = static_cast<uint8_t>(v.T2);
        h[7] = static_cast<uint8_t>(counter);
        h[6] = static_cast<uint8_t>(mN);
        h[5] = static_cast<uint8_t>(mB);
        h[4] = static_cast<uint8_t>(mT);
        h[3] = static_cast<uint8_t>(i % 256);
        h[2] = static_cast<uint8_t>((i / 256) % 256);
        h[1] = static_cast<uint8_t>((i / 65536) % 256);
        h[0] = static_cast<uint8_t>((i / 16777216) % 256);
        // ---- relay receiver, Application_Layer_Receiver.cpp:56-204 ----
        if (first_call) {
            T_s_r = h[4];
            N_s_r = h[6];
            first_call = false;
        }
        const int64_t poff = rpk_off[static_cast<size_t>(i)];
        int wb;
        int64_t tseq;
        const bool lost1 = i < n1 && e1[i];
        int rcount;
        if (lost1) {  // :76-85
            tseq = last_received + 1;
            wb = relay_erased(relay, tseq, poff);
            last_received = tseq;
            rcount = stale_counter;  // the erased message keeps the counter of the last received one
        } else {
            tseq = i;
            const int hT = h[4], hB = h[5], hN = h[6], hc = h[7];
            stale_counter = hc;
            rcount = hc;
            est->estimate(tseq, hT);
            bg->estimate(tseq, hT);
            if (tseq + 1 > cycle * kSCycle) {  // :104-113
                est = std::move(bg);
                bg.reset(new Estimator());
                ++cycle;
            }
            const int k = hT - hN + 1, n = hT + 1;
            if (T_s_r != hT || N_s_r != hN) {  // :142-150
                T_s_r = hT;
                N_s_r = hN;
                k2_new = h[8] - h[10] + 1;
                n2_new = h[8] + 1;
            }
            wb = relay_received(relay, tseq, hT, hB, hN, hc, n, k, n2_new, k2_new, poff);
            udp[0] = static_cast<uint8_t>(est->T);  // :176-201
            udp[1] = static_cast<uint8_t>(est->B_cur);
            udp[2] = static_cast<uint8_t>(est->N_cur);
            udp[3] = static_cast<uint8_t>(hT);
            udp[4] = static_cast<uint8_t>(hB);
            udp[5] = static_cast<uint8_t>(hN);
            for (int q = 6; q < 12; ++q) udp[q] = udp2[q - 6];
            last_received = tseq;
        }
        if (wb < 0) throw std::runtime_error("session: relay call without a restatement at seq " + std::to_string(i));
        if (tseq != i) throw std::logic_error("session: relay out of step");
        // ---- relay sender, Application_Layer_Sender.cpp:284-346 ----
        SesPrefix& pf = prefix[static_cast<size_t>(i)];
        pf.off = poff;
        pf.type = static_cast<uint8_t>(R);
        pf.hdr8[7] = static_cast<uint8_t>(rcount);
        pf.hdr8[6] = pf.hdr8[5] = static_cast<uint8_t>(n2_new - k2_new);
        pf.hdr8[4] = static_cast<uint8_t>(n2_new - 1);
        pf.hdr8[3] = static_cast<uint8_t>(tseq % 256);
        pf.hdr8[2] = static_cast<uint8_t>((tseq / 256) % 256);
        pf.hdr8[1] = static_cast<uint8_t>((tseq / 65536) % 256);
        pf.hdr8[0] = static_cast<uint8_t>((tseq / 16777216) % 256);
        const int64_t rsize = 8 + wb - 8;  // relay_* return the packet's bytes (from poff)
        rpk_off[static_cast<size_t>(i) + 1] = poff + rsize;
        // ---- destination, Application_Layer_Receiver.cpp:206-319 ----
        const bool lost2 = tseq < n2 && e2[tseq];
        if (!lost2) {
            const int hT = pf.hdr8[4], hB = pf.hdr8[5], hN = pf.hdr8[6], hc = pf.hdr8[7];
            dest->estimate(tseq, hT);
            dbg->estimate(tseq, hT);
            if (tseq + 1 > dcycle * kSCycle) {  // :251-260
                dest = std::move(dbg);
                dbg.reset(new Estimator());
                ++dcycle;
            }
            const int k = hT - hN + 1, n = hT + 1;
            if (int st = dest_received(dst, tseq, hT, hB, hN, hc, n, k, poff, rsize - 8, pf, pf.size_first))
                throw std::runtime_error("session: destination call without a restatement at seq " + std::to_string(i) +
                                         " (" + std::to_string(st) + ")");
            udp2[0] = static_cast<uint8_t>(dest->T);  // :302-309
            udp2[1] = static_cast<uint8_t>(dest->B_cur);
            udp2[2] = static_cast<uint8_t>(dest->N_cur);
            udp2[3] = static_cast<uint8_t>(hT);
            udp2[4] = static_cast<uint8_t>(hB);
            udp2[5] = static_cast<uint8_t>(hN);
        }
        min_rate += std::min(rate1_curr, rate2_curr);  // application_local_simulation.cpp:589-592
    }
    relay_switches = relay.switches;
    relay_flags = relay.flags;
    dest_switches = dst.switches;
    // the relay calls in lineage order
    lin.assign(1, 0);
    calls.clear();
    for (const auto& lc : lin_calls) {
        calls.insert(calls.end(), lc.begin(), lc.end());
        lin.push_back(static_cast<int64_t>(calls.size()));
    }
    control_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// ------------------------------------------------------------------------------------------
// Device side
// ------------------------------------------------------------------------------------------
namespace {

struct SesDev {
    const uint8_t* cur;       // hop-1 codewords, compact rows (fec_vr.h)
    const uint8_t* old;
    const int64_t* cur_off;   // [Q+1]
    const int64_t* old_off;
    const int32_t* len_cur;   // trimmed sizes (FEC_Encoder.cpp:55-60)
    const int32_t* len_old;   // 0 where a packet carries no old codeword
    uint8_t* rpk;             // relay packets, compact
    const int64_t* parts;     // [2 x nparts]: part start, packet end (offsets in rpk)
    const uint8_t* coef;
    const uint8_t* gf;        // exp[512] | log[256]
};

constexpr int kApplyRows = 24;  // rows of one job's window (<= n2 + n - 1 = 21)

__device__ __forceinline__ uint8_t gf_mul_t(const uint8_t* gexp, const uint8_t* glog, uint8_t a, uint8_t b) {
    return (a && b) ? gexp[glog[a] + glog[b]] : 0;
}

// Every job's outputs: a wave per job (its window rows resolved once into the wave's LDS slots, four
// jobs per workgroup, no workgroup barrier), a lane per output symbol (block j, output o).  HOP1:
// window rows are hop-1 references (seq*2 + part; the current part is followed by the old part, as
// in the received packet); else part indices into the relay buffer.
template <bool HOP1>
__global__ __launch_bounds__(256) void ses_apply_kernel(SesDev d, const SesJob* jobs, int64_t njobs, const void* refs,
                                                        uint8_t* out) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ const uint8_t* rp_a_s[4][kApplyRows];  // first segment (current part, or the relay part)
    __shared__ const uint8_t* rp_b_s[4][kApplyRows];  // second segment (the old part after the current one)
    __shared__ int32_t rl_a_s[4][kApplyRows], rl_b_s[4][kApplyRows];
    for (int i = threadIdx.x; i < 512; i += 256) gexp[i] = d.gf[i];
    glog[threadIdx.x] = d.gf[512 + threadIdx.x];
    __syncthreads();
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint8_t** rp_a = rp_a_s[wv];
    const uint8_t** rp_b = rp_b_s[wv];
    int32_t* rl_a = rl_a_s[wv];
    int32_t* rl_b = rl_b_s[wv];
    for (int64_t jb = static_cast<int64_t>(blockIdx.x) * 4 + wv; jb < njobs; jb += static_cast<int64_t>(gridDim.x) * 4) {
        const SesJob J = jobs[jb];
        const int nrows = J.rb0 + J.nin;
        __builtin_amdgcn_wave_barrier();  // (the previous job's rows are no longer read)
        if (lane < nrows) {
            const int r = lane;
            const uint8_t* pa = nullptr;
            const uint8_t* pb = nullptr;
            int la = 0, lb = 0;
            if (HOP1) {
                const int64_t ref = static_cast<const int64_t*>(refs)[J.ref0 + r];
                if (ref >= 0) {
                    const int64_t seq = ref >> 1;
                    const int lc = d.len_cur[seq], lo = d.len_old[seq];
                    if ((ref & 1) == 0) {
                        pa = d.cur + d.cur_off[seq];
                        la = lc;
                    }
                    pb = d.old + d.old_off[seq];
                    lb = lo;
                }
            } else {
                const int32_t pi = static_cast<const int32_t*>(refs)[J.ref0 + r];
                if (pi >= 0) {
                    const int64_t pp = d.parts[2 * pi], e = d.parts[2 * pi + 1];
                    pa = d.rpk + pp;
                    la = pp < e ? static_cast<int32_t>(e - pp) : 0;
                }
            }
            rp_a[r] = pa;
            rp_b[r] = pb;
            rl_a[r] = la;
            rl_b[r] = lb;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int total = J.nout * J.blocks;
        const uint8_t* cf = d.coef + J.coef;
        for (int id = lane; id < total; id += 64) {
            const int o = id / J.blocks, j = id - o * J.blocks;
            const int rbase = J.rb0 - J.rstep * o;
            const int x0 = J.base - 2 + j * J.bs;  // the part's byte of the window's position 0
            uint8_t acc = 0;
            for (int p = 0; p < J.nin; ++p) {
                const uint8_t c = cf[o * J.nin + p];
                if (!c) continue;
                const int r = rbase + p, x = x0 + p;
                uint8_t v = 0;
                if (x < rl_a[r]) v = rp_a[r][x];
                else if (x - rl_a[r] < rl_b[r]) v = rp_b[r][x - rl_a[r]];
                acc ^= gf_mul_t(gexp, glog, c, v);
            }
            out[J.out + static_cast<int64_t>(j) * J.ostride + o] = acc;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// A workgroup per lineage: codeword_new_vector's rows in LDS (logical row -> physical row map),
// per call in order: the shift of :124-129 (rows 0..n2-2 take rows 1..n2-1, row n2-1 keeps its
// bytes), the call's symbols into row n2-1 (type 2: data at 2 + j*n2 + i; type 3: every position),
// type 2's parity from rows 0..n2-2 (:601-613), then row n2-1's first `size` bytes to the packet.
__global__ __launch_bounds__(256) void ses_lineage_map_kernel(SesDev d, const SesCall* calls, const int64_t* lin,
                                                              int64_t nlin, const uint8_t* sym) {
    extern __shared__ uint8_t rows[];  // kSMaxN x kSRow
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ int map[kSMaxN];
    for (int i = threadIdx.x; i < 512; i += 256) gexp[i] = d.gf[i];
    glog[threadIdx.x] = d.gf[512 + threadIdx.x];
    for (int64_t l = blockIdx.x; l < nlin; l += gridDim.x) {
        __syncthreads();
        for (int i = threadIdx.x; i < kSMaxN * kSRow / 16; i += 256)
            reinterpret_cast<uint4*>(rows)[i] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x < kSMaxN) map[threadIdx.x] = threadIdx.x;
        __syncthreads();
        for (int64_t ci = lin[l]; ci < lin[l + 1]; ++ci) {
            const SesCall c = calls[ci];
            const int n2 = c.n2, k = c.k, blocks = c.blocks;
            __syncthreads();  // the previous call's part is stored
            if (n2 >= 2) {
                const int p0 = map[0];
                const int src = map[n2 - 1];
                __syncthreads();
                if (threadIdx.x == 0) {
                    for (int i = 0; i < n2 - 1; ++i) map[i] = map[i + 1];
                    map[n2 - 1] = p0;
                }
                // the new row n2-1 = the old row n2-1's bytes (which is now row n2-2)
                uint4* dst = reinterpret_cast<uint4*>(rows + p0 * kSRow);
                const uint4* sr = reinterpret_cast<const uint4*>(rows + src * kSRow);
                for (int i = threadIdx.x; i < kSRow / 16; i += 256) dst[i] = sr[i];
                __syncthreads();
            }
            uint8_t* top = rows + map[n2 - 1] * kSRow;
            const uint8_t* s = sym + c.d;
            if (c.type == 3) {
                for (int id = threadIdx.x; id < blocks * n2; id += 256) {
                    const int j = id / n2, i = id - j * n2;
                    top[2 + j * n2 + i] = s[j * n2 + i];
                }
            } else {
                for (int id = threadIdx.x; id < blocks * k; id += 256) {
                    const int j = id / k, i = id - j * k;
                    top[2 + j * n2 + i] = s[j * k + i];
                }
                const int np = n2 - k;
                const uint8_t* g = d.coef + c.g2;
                for (int id = threadIdx.x; id < blocks * np; id += 256) {
                    const int j = id / np, delta = id - j * np;
                    uint8_t acc = 0;
                    for (int m = 0; m < k; ++m)
                        acc ^= gf_mul_t(gexp, glog, g[delta * k + m], rows[map[m + delta] * kSRow + 2 + j * n2 + m]);
                    top[2 + j * n2 + n2 - 1 - delta] = acc;
                }
            }
            __syncthreads();
            uint8_t* o = d.rpk + c.out;
            for (int x = threadIdx.x; x < c.size; x += 256) o[x] = top[x];
        }
    }
}

// The same walk with the map in registers: logical row i at physical row (map >> 4i) & 15, the
// shift of :124-129 a rotation of the low n2 nibbles, computed by every thread alike (no map in
// LDS, no barrier for it; a lineage's n2 can change where copy_elements hands a new code's object
// to the main one); the new top row keeps the old one's bytes only where the call does not write
// them ([0, 2) and [2 + blocks*n2, hwm): every byte at or past hwm is still zero in every row); one
// barrier a call, between its writes and the store of its part; the next call's descriptor and the
// first 1 024 of its symbols are loaded while the current call computes (a lineage is a chain of up
// to ~600 calls, so the walk is bound by each call's latency).
__global__ __launch_bounds__(256) void ses_lineage_kernel(SesDev d, const SesCall* calls, const int64_t* lin,
                                                          int64_t nlin, const uint8_t* sym) {
    extern __shared__ uint8_t rows[];  // kSMaxN x kSRow
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    constexpr int NI = 4;  // prefetched symbol bytes per thread
    for (int i = threadIdx.x; i < 512; i += 256) gexp[i] = d.gf[i];
    glog[threadIdx.x] = d.gf[512 + threadIdx.x];
    const int tid = threadIdx.x;
    for (int64_t l = blockIdx.x; l < nlin; l += gridDim.x) {
        __syncthreads();
        for (int i = tid; i < kSMaxN * kSRow / 16; i += 256) reinterpret_cast<uint4*>(rows)[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        const int64_t c0 = lin[l], c1 = lin[l + 1];
        uint64_t map = 0;
        for (int i = 0; i < kSMaxN; ++i) map |= static_cast<uint64_t>(i) << (4 * i);
        int hwm = 2;
        SesCall nc{};
        uint8_t pre[NI];
        auto nsym = [](const SesCall& c) { return c.type == 3 ? c.blocks * c.n2 : c.blocks * c.k; };
        auto prefetch = [&](const SesCall& c) __attribute__((always_inline)) {
            const uint8_t* s = sym + c.d;
            const int ns = nsym(c);
#pragma unroll
            for (int q = 0; q < NI; ++q) {
                const int id = tid + 256 * q;
                pre[q] = id < ns ? s[id] : 0;
            }
        };
        if (c0 < c1) {
            nc = calls[c0];
            prefetch(nc);
        }
        for (int64_t ci = c0; ci < c1; ++ci) {
            const SesCall c = nc;
            uint8_t cur[NI];
#pragma unroll
            for (int q = 0; q < NI; ++q) cur[q] = pre[q];
            if (ci + 1 < c1) nc = calls[ci + 1];
            const int n2 = c.n2, k = c.k, blocks = c.blocks;
            const int end = 2 + blocks * n2;
            const int old_top = static_cast<int>((map >> (4 * (n2 - 1))) & 15), top_row = static_cast<int>(map & 15);
            {
                const uint64_t mask = (uint64_t(1) << (4 * n2)) - 1, lo = map & mask;
                map = (map & ~mask) | (lo >> 4) | ((lo & 15) << (4 * (n2 - 1)));
            }
            uint8_t* top = rows + top_row * kSRow;
            const uint8_t* ot = rows + old_top * kSRow;
            if (tid < 2) top[tid] = ot[tid];
            for (int x = end + tid; x < hwm; x += 256) top[x] = ot[x];
            hwm = max(hwm, end);
            const uint8_t* s = sym + c.d;
            const int ns = nsym(c);
            const int per = c.type == 3 ? n2 : k;  // symbols per block
            for (int id = tid, q = 0; id < ns; id += 256, ++q) {
                const int j = id / per, i = id - j * per;
                top[2 + j * n2 + i] = q < NI ? cur[q < NI ? q : 0] : s[id];
            }
            if (c.type != 3) {
                const int np = n2 - k;
                const uint8_t* g = d.coef + c.g2;
                for (int id = tid; id < blocks * np; id += 256) {
                    const int j = id / np, delta = id - j * np;
                    uint8_t acc = 0;
                    for (int m = 0; m < k; ++m) {
                        const int pr = static_cast<int>((map >> (4 * (m + delta))) & 15);  // logical row m + delta
                        acc ^= gf_mul_t(gexp, glog, g[delta * k + m], rows[pr * kSRow + 2 + j * n2 + m]);
                    }
                    top[2 + j * n2 + n2 - 1 - delta] = acc;
                }
            }
            if (ci + 1 < c1) prefetch(nc);
            __syncthreads();
            uint8_t* o = d.rpk + c.out;
            for (int x = tid; x < c.size; x += 256) o[x] = top[x];
            if (n2 == 1) __syncthreads();  // one row: the next call may write the row this store reads
        }
    }
}

// Per seq: the relay packet's 8-byte header, the word's size field and (type 3) header rows.
__global__ __launch_bounds__(256) void ses_prefix_kernel(SesDev d, const SesPrefix* pf, int64_t Q) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (t >= Q) return;
    const SesPrefix p = pf[t];
    uint8_t* o = d.rpk + p.off;
    for (int i = 0; i < 8; ++i) o[i] = p.hdr8[i];
    o[8] = static_cast<uint8_t>(p.size_first / 256);
    o[9] = static_cast<uint8_t>(p.size_first % 256);
    if (p.type == 3) {
        for (int i = 0; i < kSHdr; ++i) o[10 + i] = p.hdr_a[i];
        if (p.hdr2_at)
            for (int i = 0; i < kSHdr; ++i) o[p.hdr2_at + i] = p.hdr_b[i];
    }
}

// calc_missed_chars (Variable_Rate_FEC_Decoder.cpp:2698-2792): the destination's output at seq t
// (data_with_header of packet t - T_TOT) against the source payload, first 250 bytes.
__global__ __launch_bounds__(256) void ses_loss_kernel(const uint8_t* out, const uint8_t* proc, const uint8_t* payload,
                                                       int L, int64_t Q, uint8_t* lost, int64_t* count) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= Q) return;
    bool bad = false;
    if (t >= kST && proc[t]) {
        const uint8_t* o = out + t * 320 + 2;
        const uint8_t* p = payload + (t - kST) * static_cast<int64_t>(L);
        const int lim = L < 250 ? L : 250;
        for (int kk = lane; kk < lim; kk += 64) bad |= o[kk] != p[kk];
    }
    const bool any = __any(bad);
    if (lane == 0) {
        lost[t] = any ? 1 : 0;
        if (any) atomicAdd(reinterpret_cast<unsigned long long*>(count), 1ull);
    }
}

// The hop-1 wire packets (Application_Layer_Sender.cpp:222-256): [16-byte header][size_cur BE16]
// [cur][old] at `stride`, zero past the packet.
__global__ __launch_bounds__(256) void ses_hop1_kernel(SesDev d, const uint8_t* hdr, int64_t Q, uint8_t* pk,
                                                       int64_t stride, int32_t* len) {
    const int64_t t = blockIdx.x;
    if (t >= Q) return;
    const int lc = d.len_cur[t], lo = d.len_old[t];
    const int size = 18 + lc + lo;
    uint8_t* o = pk + t * stride;
    const uint8_t* c = d.cur + d.cur_off[t];
    const uint8_t* ol = d.old + d.old_off[t];
    for (int64_t x = threadIdx.x; x < stride; x += 256) {
        uint8_t v = 0;
        if (x < 16) v = hdr[t * 16 + x];
        else if (x == 16) v = static_cast<uint8_t>(lc / 256);
        else if (x == 17) v = static_cast<uint8_t>(lc % 256);
        else if (x < 18 + lc) v = c[x - 18];
        else if (x < size) v = ol[x - 18 - lc];
        o[x] = v;
    }
    if (threadIdx.x == 0) len[t] = size;
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t bytes) {
        if (bytes <= cap) return FEC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, std::max<size_t>(bytes, 256)) != hipSuccess) return FEC_ERR_NOMEM;
        cap = std::max<size_t>(bytes, 256);
        return FEC_OK;
    }
    template <class T>
    int upload(const std::vector<T>& v, hipStream_t s) {
        if (int st = reserve(v.size() * sizeof(T))) return st;
        if (v.empty()) return FEC_OK;
        return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s) == hipSuccess ? FEC_OK
                                                                                                       : FEC_ERR_HIP;
    }
};

}  // namespace
}  // namespace fec

struct fec_relay_session {
    fec::SessionPlan plan;
    fec_vr_plan* vp = nullptr;
    int64_t cur_bytes = 0, old_bytes = 0;
    fec::DevBuf cur, old, len_cur, len_old, rjobs, rrefs, calls, lin, prefix, djobs, djr, parts, coef, gf, sym, proc,
        hdr1;
    const int64_t* cur_off = nullptr;
    const int64_t* old_off = nullptr;
    bool uploaded = false;
    hipEvent_t done = nullptr;
    ~fec_relay_session() {
        if (done) {
            (void)hipEventSynchronize(done);
            (void)hipEventDestroy(done);
        }
        if (vp) fec_vr_plan_destroy(vp);
    }
};

namespace {
template <class F>
int ses_guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (const std::invalid_argument&) {
        return FEC_ERR_ARG;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}

fec::SesDev dev_view(fec_relay_session* h, uint8_t* rpk) {
    fec::SesDev d{};
    d.cur = static_cast<const uint8_t*>(h->cur.p);
    d.old = static_cast<const uint8_t*>(h->old.p);
    d.cur_off = h->cur_off;
    d.old_off = h->old_off;
    d.len_cur = static_cast<const int32_t*>(h->len_cur.p);
    d.len_old = static_cast<const int32_t*>(h->len_old.p);
    d.rpk = rpk;
    d.parts = static_cast<const int64_t*>(h->parts.p);
    d.coef = static_cast<const uint8_t*>(h->coef.p);
    d.gf = static_cast<const uint8_t*>(h->gf.p);
    return d;
}

int ses_upload(fec_relay_session* h, hipStream_t s) {
    if (h->uploaded) return FEC_OK;
    const auto& p = h->plan;
    std::vector<uint8_t> gf;
    {
        const fec::Field& F = fec::field();
        gf.assign(F.exp, F.exp + 512);
        gf.insert(gf.end(), F.log, F.log + 256);
    }
    if (int st = h->rjobs.upload(p.rjobs, s)) return st;
    if (int st = h->rrefs.upload(p.rrefs, s)) return st;
    if (int st = h->calls.upload(p.calls, s)) return st;
    if (int st = h->lin.upload(p.lin, s)) return st;
    if (int st = h->prefix.upload(p.prefix, s)) return st;
    if (int st = h->djobs.upload(p.djobs, s)) return st;
    if (int st = h->djr.upload(p.djr, s)) return st;
    if (int st = h->parts.upload(p.parts, s)) return st;
    if (int st = h->coef.upload(p.coef, s)) return st;
    if (int st = h->gf.upload(gf, s)) return st;
    if (int st = h->proc.upload(p.proc, s)) return st;
    if (int st = h->hdr1.upload(p.hdr1, s)) return st;
    if (int st = h->sym.reserve(static_cast<size_t>(p.d_bytes) + 64)) return st;
    if (int st = h->cur.reserve(static_cast<size_t>(h->cur_bytes) + 64)) return st;
    if (int st = h->old.reserve(static_cast<size_t>(h->old_bytes) + 64)) return st;
    if (int st = h->len_cur.reserve(static_cast<size_t>(p.Q) * 4)) return st;
    if (int st = h->len_old.reserve(static_cast<size_t>(p.Q) * 4)) return st;
    if (int st = fec::vr_plan_device_offsets(h->vp, s, &h->cur_off, &h->old_off)) return st;
    // the host vectors stay alive in the plan; the copies are complete before run's kernels read them
    h->uploaded = true;
    return FEC_OK;
}
}  // namespace

extern "C" {

int fec_relay_session_create(int relay_type, int max_payload, int64_t Q, const uint8_t* e1, int64_t n_e1,
                             const uint8_t* e2, int64_t n_e2, fec_relay_session** out) {
    if (!out || Q < 1 || n_e1 < 0 || n_e2 < 0 || (n_e1 && !e1) || (n_e2 && !e2)) return FEC_ERR_ARG;
    *out = nullptr;
    return ses_guarded([&] {
        std::unique_ptr<fec_relay_session> h(new fec_relay_session());
        h->plan.run(relay_type, max_payload, Q, e1, n_e1, e2, n_e2);
        if (int st = fec::vr_plan_from_instances(max_payload, h->plan.enc, Q, &h->vp)) return st;
        if (int st = fec_vr_plan_layout(h->vp, &h->cur_bytes, &h->old_bytes)) return st;
        *out = h.release();
        return static_cast<int>(FEC_OK);
    });
}

int fec_relay_session_destroy(fec_relay_session* h) {
    delete h;
    return FEC_OK;
}

int fec_relay_session_info(const fec_relay_session* h, int64_t* stats, double* rates) {
    if (!h) return FEC_ERR_ARG;
    const auto& p = h->plan;
    if (stats) {
        int64_t longest = 0;
        for (size_t i = 0; i + 1 < p.lin.size(); ++i) longest = std::max(longest, p.lin[i + 1] - p.lin[i]);
        int64_t processed = 0;
        for (uint8_t x : p.proc) processed += x;
        const int64_t v[16] = {p.Q, p.rpk_off.back(), p.src_switches, p.relay_switches, p.dest_switches,
                               p.dest_flags, static_cast<int64_t>(p.calls.size()),
                               static_cast<int64_t>(p.lin.size()) - 1, static_cast<int64_t>(p.djobs.size()),
                               processed, p.d_bytes, static_cast<int64_t>(p.enc.size()), longest, p.relay_flags,
                               p.rate1_n, p.rate2_n};
        std::memcpy(stats, v, sizeof(v));
    }
    if (rates) {
        rates[0] = p.rate1;
        rates[1] = p.rate2;
        rates[2] = p.min_rate;
        rates[3] = p.control_ms;
    }
    return FEC_OK;
}

int fec_relay_session_relay_offsets(const fec_relay_session* h, int64_t* off) {
    if (!h || !off) return FEC_ERR_ARG;
    std::memcpy(off, h->plan.rpk_off.data(), h->plan.rpk_off.size() * sizeof(int64_t));
    return FEC_OK;
}

int fec_relay_session_hop1_headers(const fec_relay_session* h, uint8_t* hdr) {
    if (!h || !hdr) return FEC_ERR_ARG;
    std::memcpy(hdr, h->plan.hdr1.data(), h->plan.hdr1.size());
    return FEC_OK;
}

int fec_relay_session_dest_meta(const fec_relay_session* h, uint8_t* proc, uint8_t* flag) {
    if (!h) return FEC_ERR_ARG;
    if (proc) std::memcpy(proc, h->plan.proc.data(), h->plan.proc.size());
    if (flag) std::memcpy(flag, h->plan.dflag.data(), h->plan.dflag.size());
    return FEC_OK;
}

int fec_relay_session_run(fec_relay_session* h, const uint8_t* d_payload, uint8_t* d_relay, uint8_t* d_dest_out,
                          uint8_t* d_dest_lost, int64_t* d_lost, void* hip_stream) {
    if (!h || !d_payload || !d_relay || !d_dest_out || !d_dest_lost || !d_lost) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const auto& p = h->plan;
    if (int st = ses_guarded([&] { return ses_upload(h, s); })) return st;
    // the source: every encoder instance of the schedule (the batched variable-rate encoder)
    FEC_HIP(hipMemsetAsync(h->len_old.p, 0, static_cast<size_t>(p.Q) * 4, s));
    if (int st = fec_vr_encode_batch(h->vp, d_payload, nullptr, static_cast<uint8_t*>(h->cur.p),
                                     static_cast<int32_t*>(h->len_cur.p), static_cast<uint8_t*>(h->old.p),
                                     static_cast<int32_t*>(h->len_old.p), s))
        return st;
    const fec::SesDev d = dev_view(h, d_relay);
    // the relay: every call's symbols, then the lineages in order, then the fixed bytes
    if (!p.rjobs.empty()) {
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>((static_cast<int64_t>(p.rjobs.size()) + 3) / 4, 65536));
        hipLaunchKernelGGL(fec::ses_apply_kernel<true>, dim3(grid), dim3(256), 0, s, d,
                           static_cast<const fec::SesJob*>(h->rjobs.p), static_cast<int64_t>(p.rjobs.size()),
                           h->rrefs.p, static_cast<uint8_t*>(h->sym.p));
        FEC_HIP(hipGetLastError());
    }
    const int64_t nlin = static_cast<int64_t>(p.lin.size()) - 1;
    if (nlin > 0) {
        const size_t lds = static_cast<size_t>(fec::kSMaxN) * fec::kSRow;
        hipLaunchKernelGGL(!std::getenv("FEC_SES_LIN_MAP") ? fec::ses_lineage_kernel : fec::ses_lineage_map_kernel,
                           dim3(static_cast<unsigned>(std::min<int64_t>(nlin, 65536))), dim3(256), lds, s, d,
                           static_cast<const fec::SesCall*>(h->calls.p), static_cast<const int64_t*>(h->lin.p), nlin,
                           static_cast<const uint8_t*>(h->sym.p));
        FEC_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(fec::ses_prefix_kernel, dim3(static_cast<unsigned>((p.Q + 255) / 256)), dim3(256), 0, s, d,
                       static_cast<const fec::SesPrefix*>(h->prefix.p), p.Q);
    FEC_HIP(hipGetLastError());
    // the destination's outputs and the loss check
    FEC_HIP(hipMemsetAsync(d_dest_out, 0, static_cast<size_t>(p.Q) * 320, s));
    FEC_HIP(hipMemsetAsync(d_lost, 0, sizeof(int64_t), s));
    if (!p.djobs.empty()) {
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>((static_cast<int64_t>(p.djobs.size()) + 3) / 4, 65536));
        hipLaunchKernelGGL(fec::ses_apply_kernel<false>, dim3(grid), dim3(256), 0, s, d,
                           static_cast<const fec::SesJob*>(h->djobs.p), static_cast<int64_t>(p.djobs.size()),
                           h->djr.p, d_dest_out);
        FEC_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(fec::ses_loss_kernel, dim3(static_cast<unsigned>((p.Q + 3) / 4)), dim3(256), 0, s, d_dest_out,
                       static_cast<const uint8_t*>(h->proc.p), d_payload, p.L, p.Q, d_dest_lost, d_lost);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int fec_relay_session_hop1(fec_relay_session* h, uint8_t* d_packets, int64_t stride, int32_t* d_len, void* hip_stream) {
    if (!h || !d_packets || !d_len || !h->uploaded || stride < 18) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const fec::SesDev d = dev_view(h, nullptr);
    hipLaunchKernelGGL(fec::ses_hop1_kernel, dim3(static_cast<unsigned>(h->plan.Q)), dim3(256), 0, s, d,
                       static_cast<const uint8_t*>(h->hdr1.p), h->plan.Q, d_packets, stride, d_len);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // extern "C"
