// fec_sdswdf.hip -- the relay's state-dependent symbol-wise decode-and-forward (SD-SWDF,
// RELAYING_TYPE 3) and the destination's state-dependent decode, batched over many packets of
// one relay stream.
//
// Reference: Decoder_Symbol_Wise::symbol_wise_encode_state_dependent (src/Decoder_Symbol_Wise.cpp
// :178-432) at the relay, symbol_wise_decode_state_dependent (:487-546) + extract_data (:653-661)
// at the destination, driven by Variable_Rate_FEC_Decoder with one relay frame per seq
// (FLAG_FOR_CONSTANT_TRANS = 1): relay received packet :1458-1493, relay erased packet :636-675,
// destination frame :1798-1815, destination missing frame :1703-1721.
//
// The relay keeps the last 3*T_TOT packets with their erasure flags and the headers it sent.  For
// every index of its outgoing frame (symInd = k-1-index, from k-1 down to -(n2-k)) it looks at
// one diagonal of the source code: a partial one (symInd >= n-k) whose received symbols it
// forwards, or a complete one it decodes (decodeBlock, T = n-1) and re-encodes for the second hop
// (encodeBlock, G2), forwarding a symbol the destination has not had yet.  The 11-byte header
// tells the destination which symbol of its diagonal each frame symbol is.
//
// Every decision depends only on the erasure flags and the headers, never on payload bytes, and
// every forwarded byte is a GF linear combination of at most n received symbols of one diagonal:
// symbol (j, p) of source packet t-(n-1)+p+symInd at the relay, symbol (j, q) of frame
// t2-k_shift-(n-1-q) at the destination.  So a host planner replays the reference's control flow
// symbolically (coefficient vectors instead of bytes, the decode rules of fec_host.cpp instead of
// the per-call RREF) and interns one record per distinct packet plan; the byte work is two
// data-parallel kernels, one thread per (packet, code block), reading the plan of their packet.
//
// Reference behaviour kept (well-defined, restated in oracle/fec_oracle.c or_sdswdf_*): the burst
// test as written (it only acts with FLAG_FOR_SDBO = 1, a run-time flag here), header rows shifted
// 10 of their 11 ints (:133, :169; entry 10 of a row is never moved), decodeBlock clearing the flags
// of what it recovers (so the "forward a received symbol" branch also forwards recovered data),
// the block count ceil(max_payload/k)+1 on ints, the relay's flag never set.  Undefined behaviour
// defined away: slots hold zero-padded packets, the erased-packet frame has its full
// size, out-of-bounds stack writes (:309-312, :325) land nowhere, and stale temp_codeword bytes
// (:248-250) are never forwarded (the oracle proves it by filling them with garbage).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <array>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "fec_amd.h"
#include "fec_host.h"
#include "fec_kernels.h"
#include "fec_device.h"
#include "fec_status.h"

namespace fec {
namespace {

constexpr int kTT = 10;             // T_TOT (FEC_Macro.h:32)
constexpr int kSlots = 3 * kTT;     // codeword_vector_state_dependent rows
constexpr int kHdr = kTT + 1;       // header entries per row (and frame header bytes)
constexpr int kSdThreads = 256;

// A symbolic symbol: its GF coefficients over the n positions of the diagonal being read.
struct Vec {
    uint8_t c[kMaxN];
};

void vec_zero(Vec& v, int n) { std::memset(v.c, 0, static_cast<size_t>(n)); }
void vec_unit(Vec& v, int n, int p) {
    vec_zero(v, n);
    v.c[p] = 1;
}
void vec_axpy(Vec& y, uint8_t a, const Vec& x, int n) {  // y ^= a * x
    if (!a) return;
    const Field& f = field();
    for (int i = 0; i < n; ++i) y.c[i] ^= f.mt[a][x.c[i]];
}

// decodeBlock(cw, G, cw, er, k, n, T = n-1, t = 0) on symbolic symbols (codingOperations.cpp
// :149-232 through the window-n decode rule): recovered data symbols become combinations of the
// symbols the rule names, and their erasure flags are cleared (:224-229).
void sym_decode(const DecodeRules& rules, int k, int n, Vec* tc, uint8_t* er) {
    uint32_t mask = 0;
    for (int c = 0; c < n; ++c) mask |= (er[c] ? 1u : 0u) << c;
    int cnt = __builtin_popcount(mask);
    if (cnt == n) return;  // all erased (:181-182)
    const uint8_t* e = rules.entry(n, mask);
    Vec rec[kMaxK];
    uint32_t done = 0;
    for (int i = 0; i < k; ++i) {
        if (!er[i] || e[i] == 0xFF) continue;
        const uint8_t* col = e + k + i * n;
        vec_zero(rec[i], n);
        for (int c = 0; c < n; ++c) vec_axpy(rec[i], col[c], tc[c], n);
        done |= 1u << i;
    }
    for (int i = 0; i < k; ++i)
        if ((done >> i) & 1u) {
            tc[i] = rec[i];
            er[i] = 0;
        }
}

// Open-addressing map from N-word keys (linear probing, power-of-two table, grown at half load):
// the planners look up one state per packet; with a string key in std::unordered_map that lookup
// was most of the planners' time.
template <int N, class V>
class FlatMap {
public:
    using Key = std::array<uint64_t, N>;
    FlatMap() { clear(); }
    void clear() {
        keys_.assign(64, Key{});
        used_.assign(64, 0);
        vals_.assign(64, V{});
        size_ = 0;
    }
    const V* find(const Key& k) const {
        const size_t mask = keys_.size() - 1;
        for (size_t i = hash(k) & mask;; i = (i + 1) & mask) {
            if (!used_[i]) return nullptr;
            if (keys_[i] == k) return &vals_[i];
        }
    }
    const V* insert(const Key& k, const V& v) {  // k is not in the map
        if (2 * (size_ + 1) > keys_.size()) grow();
        const size_t mask = keys_.size() - 1;
        size_t i = hash(k) & mask;
        while (used_[i]) i = (i + 1) & mask;
        used_[i] = 1;
        keys_[i] = k;
        vals_[i] = v;
        ++size_;
        return &vals_[i];
    }
    size_t size() const { return size_; }

private:
    static size_t hash(const Key& k) {
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (int i = 0; i < N; ++i) {
            h = (h ^ k[i]) * 0xff51afd7ed558ccdull;
            h ^= h >> 29;
        }
        return static_cast<size_t>(h ^ (h >> 32));
    }
    void grow() {
        std::vector<Key> ok;
        std::vector<uint8_t> ou;
        std::vector<V> ov;
        ok.swap(keys_);
        ou.swap(used_);
        ov.swap(vals_);
        keys_.assign(ok.size() * 2, Key{});
        used_.assign(ok.size() * 2, 0);
        vals_.assign(ok.size() * 2, V{});
        size_ = 0;
        for (size_t i = 0; i < ok.size(); ++i)
            if (ou[i]) insert(ok[i], ov[i]);
    }
    std::vector<Key> keys_;
    std::vector<uint8_t> used_;
    std::vector<V> vals_;
    size_t size_ = 0;
};

// Distinct records, each stored once (plans repeat: an erasure-free stretch is one record).
class RecordTable {
public:
    explicit RecordTable(int bytes) : bytes_(bytes) {}
    int32_t intern(const uint8_t* rec) {
        std::string key(reinterpret_cast<const char*>(rec), static_cast<size_t>(bytes_));
        auto it = ids_.find(key);
        if (it != ids_.end()) return it->second;
        const int32_t id = static_cast<int32_t>(ids_.size());
        ids_.emplace(std::move(key), id);
        data_.insert(data_.end(), rec, rec + bytes_);
        return id;
    }
    void clear() {
        ids_.clear();
        data_.clear();
    }
    const std::vector<uint8_t>& data() const { return data_; }
    int64_t count() const { return static_cast<int64_t>(ids_.size()); }

private:
    int bytes_;
    std::unordered_map<std::string, int32_t> ids_;
    std::vector<uint8_t> data_;
};

// Header rows as small ids: entries 0..T_TOT-1 of a row (the part the reference's shifts move,
// :133, :169; entry T_TOT stays with its slot) packed into two words.  The planners keep a window
// of row ids instead of shifting 30 rows of ints per packet, and key their memo on it.
class RowIds {
public:
    uint16_t intern(const int* e) {
        uint64_t a = 0, b = 0;
        for (int i = 0; i < 8; ++i) a |= static_cast<uint64_t>(static_cast<uint8_t>(e[i])) << (8 * i);
        for (int i = 8; i < kTT; ++i) b |= static_cast<uint64_t>(static_cast<uint8_t>(e[i])) << (8 * (i - 8));
        const FlatMap<2, uint16_t>::Key key{a, b};
        if (const uint16_t* f = ids_.find(key)) return *f;
        if (rows_.size() >= 0xffff) throw std::length_error("sdswdf: header rows");
        const uint16_t id = static_cast<uint16_t>(rows_.size());
        std::array<int, kTT> r{};
        for (int i = 0; i < kTT; ++i) r[i] = e[i];
        rows_.push_back(r);
        ids_.insert(key, id);
        return id;
    }
    const std::array<int, kTT>& row(uint16_t id) const { return rows_[id]; }
    void clear() {
        ids_.clear();
        rows_.clear();
    }

private:
    FlatMap<2, uint16_t> ids_;
    std::vector<std::array<int, kTT>> rows_;
};

// The relay: symbol_wise_encode_state_dependent per packet, symbolic.  Output record per packet:
// header[n2-1][0..10] as bytes, then n2 rows of n coefficients (row index: frame symbol `index`
// of every code block j = sum_p coef[p] * symbol (j, p) of source packet t-(n-1)+p+(k-1-index)).
class SdRelayPlanner {
public:
    SdRelayPlanner(int k, int n, int n2, int sdbo, std::shared_ptr<const DecodeRules> rules,
                   std::vector<uint8_t> G2)
        : k_(k), n_(n), n2_(n2), sdbo_(sdbo), rules_(std::move(rules)), G2_(std::move(G2)),
          records_(kHdr + n2 * n) {
        if (n2 - 1 > 11) throw std::invalid_argument("sdswdf: n2 > 12");  // RelayKey
        rec_.resize(static_cast<size_t>(record_bytes()));
        reset();
    }
    int record_bytes() const { return kHdr + n2_ * n_; }
    const RecordTable& records() const { return records_; }
    void reset() {
        records_.clear();
        memo_.clear();
        rows_.clear();
        restart();
    }
    // A fresh relay's state, keeping the records, the memo and the interned header rows (their
    // meaning does not depend on the state): the plans of several streams in one table.
    void restart() {
        std::memset(er_, 0, sizeof(er_));
        std::memset(valid_, 0, sizeof(valid_));
        for (int i = 0; i < kSlots; ++i)
            for (int jj = 0; jj < kHdr; ++jj) header_[i][jj] = jj + 1;  // :60-62
        er_bits_ = valid_bits_ = 0;
        last_key_ok_ = false;
        const uint16_t id0 = rows_.intern(header_[0]);
        for (auto& w : win_) w = id0;
        prev_e10_ = kHdr;
    }
    // Packet t (t = 0, 1, ... in order), erased on hop 1: the id of its record.  The plan of a
    // packet is a function of the flags of the slots its diagonals read and of the headers of
    // the last n2-1 packets (rows n2-1 and up hold constants): repeated states are looked up.
    // Between packets the state is kept compact: the flags as bit masks (slot i = bit i) and the
    // last n2-1 emitted header rows as ids (header row r < n2-1 = emission t-(n2-1)+r; entry T_TOT of
    // those rows never moves from its initial value; row n2-1 keeps its own entry T_TOT); the
    // reference-structured arrays are rebuilt from it only when a state is planned for the first
    // time.
    int32_t step(bool erased) {
        // push_current_codeword / rotate_pointers_and_insert_zero_word: slot i <- slot i+1, the top
        // slot keeps its flags; then slot 2T is the new packet
        constexpr uint32_t top = 1u << (kSlots - 1), cur = 1u << (2 * kTT);
        er_bits_ = ((er_bits_ >> 1) | (er_bits_ & top)) & ~cur;
        valid_bits_ = ((valid_bits_ >> 1) | (valid_bits_ & top)) & ~cur;
        if (erased) er_bits_ |= cur;
        else valid_bits_ |= cur;
        const int lo = 2 * kTT - n_ + 1 - (n2_ - k_);
        const uint32_t wmask = (2 * kTT - lo + 1) >= 32 ? ~0u : ((1u << (2 * kTT - lo + 1)) - 1u);
        const uint32_t ew = (er_bits_ >> lo) & wmask, vw = (valid_bits_ >> lo) & wmask;
        // key: the window's flags, the last n2-1 emitted rows' ids (words 1-3, 4 per word; the
        // unused ones stay 0) and the previous row's entry T_TOT (word 3, top 16 bits)
        RelayKey key{static_cast<uint64_t>(ew) | static_cast<uint64_t>(vw) << 32, 0, 0, 0};
        for (int r = 0; r < n2_ - 1; ++r) key[1 + (r >> 2)] |= static_cast<uint64_t>(win_[r]) << (16 * (r & 3));
        key[3] |= static_cast<uint64_t>(static_cast<uint16_t>(prev_e10_)) << 48;
        const Memo* mp = last_key_ok_ && key == last_key_ ? &last_m_ : memo_.find(key);
        if (!mp) {
            for (int i = 0; i < kSlots; ++i) {
                er_[i] = static_cast<uint8_t>(er_bits_ >> i & 1u);
                valid_[i] = static_cast<uint8_t>(valid_bits_ >> i & 1u);
                for (int jj = 0; jj < kHdr; ++jj) header_[i][jj] = jj + 1;
            }
            for (int r = 0; r < n2_ - 1; ++r) {
                const auto& row = rows_.row(win_[r]);
                for (int e = 0; e < kTT; ++e) header_[r][e] = row[e];
            }
            header_[n2_ - 1][kTT] = prev_e10_;
            encode(rec_.data());
            Memo m;
            m.id = records_.intern(rec_.data());
            for (int i = 0; i < kHdr; ++i) m.hdr[i] = static_cast<uint8_t>(header_[n2_ - 1][i]);
            m.row = rows_.intern(header_[n2_ - 1]);
            mp = memo_.insert(key, m);
        }
        if (mp != &last_m_) {
            last_key_ = key;
            last_m_ = *mp;
            last_key_ok_ = true;
        }
        const Memo& m = last_m_;
        if (n2_ > 1) {
            for (int r = 0; r + 1 < n2_ - 1; ++r) win_[r] = win_[r + 1];
            win_[n2_ - 2] = m.row;
        }
        prev_e10_ = m.hdr[kTT];
        return m.id;
    }

    // One call of the reference method on caller-held state (the drop-in Decoder_Symbol_Wise,
    // fec_sw_state_encode): the flags and header rows as the caller's arrays hold them; every slot
    // counts as holding bytes (an erased slot holds zeros, Variable_Rate_FEC_Decoder.cpp:641-642).
    // Writes the record and header[n2-1][0..n2) back.
    void plan_state(const uint8_t* er, int* const* header, uint8_t* rec) {
        for (int i = 0; i < kSlots; ++i) {
            er_[i] = er[i] ? 1 : 0;
            valid_[i] = 1;
            std::memcpy(header_[i], header[i], sizeof(int) * kHdr);
        }
        encode(rec);
        for (int i = 0; i < n2_; ++i) header[n2_ - 1][i] = header_[n2_ - 1][i];
    }

private:
    // push_current_codeword / rotate_pointers_and_insert_zero_word (:131-135, :167-171)
    void shift() {
        for (int i = 0; i < kSlots - 1; ++i) {
            std::memcpy(header_[i], header_[i + 1], sizeof(int) * kTT);
            er_[i] = er_[i + 1];
            valid_[i] = valid_[i + 1];
        }
    }
    void encode(uint8_t* rec) {
        const int k = k_, n = n_, n2 = n2_, k2 = k_, TT = kTT;
        uint8_t stam[2 * kMaxN + 2 * kHdr];
        int tempHeader[kMaxN + kHdr];
        // burst check (:198-231); the in_burst assignments make it "longest run, first end"
        int longest = 0, end = 0, run = 0;
        for (int aa = 0; aa < n; ++aa) {
            if (er_[2 * TT - n + 1 + aa] == 1) {
                ++run;
            } else {
                if (run > longest) {
                    longest = run;
                    end = aa - 1;
                }
                run = 0;
            }
        }
        if (run > longest) {
            longest = run;
            end = n - 1;
        }
        const bool burst = sdbo_ == 1 && longest > n - k && end >= k - 1;
        uint8_t* coef = rec + kHdr;
        Vec tc[kMaxN], enc[kMaxN];
        int index = -1;
        for (int symInd = k - 1; symInd >= -(n2 - k2); --symInd) {
            ++index;
            // the diagonal: position p from slot p + symInd + 2T-n+1; a zero slot (erased, or
            // before the first packet) is a zero symbol; positions past the current packet are
            // not filled (stale in the reference, never forwarded)
            const int filled = symInd >= 0 ? n - symInd : n;
            // n2 > n (the two-hop session): the selection may read temp_codeword[i] for n <= i < n2,
            // past the reference's VLA (:367): a zero symbol here, as in the oracle
            for (int p = n; p < n2; ++p) vec_zero(tc[p], n);
            for (int p = 0; p < n; ++p) {
                const int slot = p + symInd + 2 * TT - n + 1;
                if (p < filled && valid_[slot]) vec_unit(tc[p], n, p);
                else vec_zero(tc[p], n);
            }
            const int symbolIndex = n - 1 - symInd;
            const int prev = symbolIndex - (n - k);  // == index: header entries already sent
            Vec out;
            vec_zero(out, n);
            int hdr = 0;
            if (n - symInd <= k) {  // forward from a partial diagonal (:252-301)
                for (int i = 0; i < n; ++i) tempHeader[i] = 0;
                for (int s2 = 0; s2 < prev; ++s2) tempHeader[s2] = header_[n2 - (prev - s2) - 1][s2];
                bool found = false;
                if (burst && index <= k - 1) {
                    hdr = index + 1;
                    found = true;
                } else {
                    for (int kk = index; kk < n - symInd; ++kk) {
                        if (er_[kk + symInd + 2 * TT - n + 1] != 0) continue;
                        bool sent = false;
                        for (int jj = 0; jj < kk; ++jj)
                            if (tempHeader[jj] == kk + 1) sent = true;
                        if (!sent) {
                            out = tc[kk];
                            hdr = kk + 1;
                            found = true;
                            break;
                        }
                    }
                }
                if (!found) {  // zero symbol, first header value not used yet (:285-301)
                    int pot;
                    for (pot = 1; pot < n; ++pot) {
                        bool used = false;
                        for (int aa = 0; aa < prev; ++aa)
                            if (tempHeader[aa] == pot) {
                                used = true;
                                break;
                            }
                        if (!used) break;
                    }
                    hdr = pot;
                }
            } else if (burst && index <= k - 1) {  // (:303-305)
                hdr = index + 1;
            } else {  // decode the diagonal, re-encode, forward a symbol not sent yet (:306-393)
                for (int aa = 0; aa < n2; ++aa) stam[aa] = 0;
                for (int aa = 0; aa < n - symInd; ++aa) stam[aa] = er_[aa + symInd + 2 * TT - n + 1];
                for (int aa = n - symInd; aa < n; ++aa) stam[aa] = 1;
                int erasure_count = 0;
                for (int aa = 0; aa < n; ++aa) erasure_count += stam[aa] == 1;
                sym_decode(*rules_, k, n, tc, stam);
                for (int i = 0; i < k2; ++i) enc[i] = tc[i];  // memcpy + encodeBlock(t = k2-1)
                for (int i = k2; i < n2; ++i) {
                    vec_zero(enc[i], n);
                    for (int d = 0; d < k2; ++d) vec_axpy(enc[i], G2_[d * n2 + i], tc[d], n);
                }
                for (int i = 0; i < n2; ++i) tempHeader[i] = 0;
                for (int s2 = 0; s2 < prev; ++s2) tempHeader[s2] = header_[n2 - (prev - s2) - 1][s2];
                bool assigned = false;
                for (int i = 0; i < n2; ++i) {
                    bool sent = false;
                    for (int kk = 0; kk < prev; ++kk)
                        if (tempHeader[kk] == i + 1) {
                            sent = true;
                            break;
                        }
                    if (sent) continue;
                    if (burst || erasure_count <= n - k) {
                        out = enc[i];
                        hdr = i + 1;
                        assigned = true;
                        break;
                    } else if (stam[i] == 0) {  // not decodable: forward (:361-371)
                        out = tc[i];
                        hdr = i + 1;
                        assigned = true;
                        break;
                    }
                }
                if (!assigned) {  // (:375-393)
                    for (int i = 0; i < n2; ++i) {
                        bool sent = false;
                        for (int kk = 0; kk < index; ++kk)
                            if (tempHeader[kk] == i + 1) {
                                sent = true;
                                break;
                            }
                        if (!sent) {
                            hdr = i + 1;
                            break;
                        }
                    }
                    if (!hdr) hdr = header_[n2 - 1][index];  // unreachable: index < n2 values used
                }
            }
            header_[n2 - 1][index] = hdr;
            std::memcpy(coef + index * n, out.c, static_cast<size_t>(n));
        }
        for (int aa = 0; aa < kHdr; ++aa) rec[aa] = static_cast<uint8_t>(header_[n2 - 1][aa]);
    }

    struct Memo {
        int32_t id;
        uint8_t hdr[kHdr];
        uint16_t row;  // entries 0..T_TOT-1 of the emitted header row
    };
    using RelayKey = FlatMap<4, Memo>::Key;  // n2 - 1 <= 10 row ids (n2 <= n1 <= T_TOT + 1)
    int k_, n_, n2_, sdbo_;
    std::shared_ptr<const DecodeRules> rules_;
    std::vector<uint8_t> G2_;
    uint8_t er_[kSlots];
    uint8_t valid_[kSlots];  // the slot holds a received packet (not erased, not before packet 0)
    int header_[kSlots][kHdr];
    RecordTable records_;
    std::vector<uint8_t> rec_;
    FlatMap<4, Memo> memo_;
    RelayKey last_key_{};  // the last state looked up and its memo entry
    Memo last_m_{};
    bool last_key_ok_ = false;
    RowIds rows_;
    uint32_t er_bits_ = 0, valid_bits_ = 0;
    uint16_t win_[kMaxN] = {};
    int prev_e10_ = kHdr;
};

// The destination: symbol_wise_decode_state_dependent per frame, symbolic.  Output record: k
// rows of n coefficients (row s = data symbol s of every code block j = sum_q coef[q] * frame
// symbol (j, q) of frame t2-s-(n-1-q)); the flag is returned.
class SdDestPlanner {
public:
    SdDestPlanner(int k, int n, std::shared_ptr<const DecodeRules> rules)
        : k_(k), n_(n), rules_(std::move(rules)), records_(k * n) {
        if (k + n - 1 > 28) throw std::invalid_argument("sdswdf: k + n - 1 > 28");  // DestKey
        rec_.resize(static_cast<size_t>(record_bytes()));
        reset();
    }
    int record_bytes() const { return k_ * n_; }
    const RecordTable& records() const { return records_; }
    void reset() {
        records_.clear();
        memo_.clear();
        rows_.clear();
        restart();
    }
    // A fresh destination's state, keeping the records, the memo and the interned header rows.
    void restart() {
        std::memset(valid_, 0, sizeof(valid_));
        for (int i = 0; i < kSlots; ++i)
            for (int jj = 0; jj < kHdr; ++jj) header_[i][jj] = jj + 1;
        valid_bits_ = 0;
        last_ok_ = false;
        last_key_ok_ = false;
        const uint16_t id0 = rows_.intern(header_[0]);
        for (auto& w : ids_) w = id0;
        top_e10_ = kHdr;
        win_key_ = DestKey{};
        const int lo = kSlots - k_ - n_ + 1;
        for (int r = lo; r < kSlots; ++r) win_key_[1 + ((r - lo) >> 2)] |= static_cast<uint64_t>(ids_[r]) << (16 * ((r - lo) & 3));
    }
    // Frame t2 (in order): its record id; *flag = the loss flag.  The plan is a function of the
    // header rows and presence of the last k+n-1 frames: repeated states are looked up.  Between
    // frames the state is compact: presence as a bit mask, every header row as an id of its
    // entries 0..T_TOT-1, and the top row's entry T_TOT (the rows below keep the initial one: the
    // shifts never move it, :1663-1664); the arrays are rebuilt only for a state seen first.
    int32_t step(bool erased, const uint8_t* hdr, bool* flag) {
        constexpr uint32_t top = 1u << (kSlots - 1);
        valid_bits_ = (valid_bits_ >> 1) & ~top;
        if (!erased) valid_bits_ |= top;
        std::memmove(ids_, ids_ + 1, sizeof(uint16_t) * (kSlots - 1));
        // the row's id: consecutive frames mostly carry the same header (a steady stretch), and a
        // missing frame's row is zeros (:1709, :1803)
        uint8_t bytes[kHdr] = {};
        if (!erased) std::memcpy(bytes, hdr, kHdr);
        if (!last_ok_ || std::memcmp(bytes, last_hdr_, kHdr) != 0) {
            int row[kHdr];
            for (int i = 0; i < kHdr; ++i) row[i] = bytes[i];
            last_id_ = rows_.intern(row);
            std::memcpy(last_hdr_, bytes, kHdr);
            last_ok_ = true;
        }
        ids_[kSlots - 1] = last_id_;
        top_e10_ = bytes[kTT];
        const int lo = kSlots - k_ - n_ + 1;
        const uint32_t vw = valid_bits_ >> lo;
        // key: presence, the top row's entry T_TOT (word 0) and the k+n-1 rows' ids (4 per word,
        // oldest first), slid by one id per frame
        const int W = kSlots - lo, nw = (W + 3) >> 2;
        for (int i = 1; i <= nw; ++i) win_key_[i] = (win_key_[i] >> 16) | (i < 7 ? win_key_[i + 1] << 48 : 0);
        win_key_[1 + ((W - 1) >> 2)] |= static_cast<uint64_t>(last_id_) << (16 * ((W - 1) & 3));
        win_key_[0] = static_cast<uint64_t>(vw) | static_cast<uint64_t>(static_cast<uint16_t>(top_e10_)) << 32;
        const DestKey& key = win_key_;
        if (last_key_ok_ && key == last_key_) {  // a steady stretch repeats the state
            *flag = last_m_.flag;
            return last_m_.id;
        }
        if (const Memo* f = memo_.find(key)) {
            last_key_ = key;
            last_m_ = *f;
            last_key_ok_ = true;
            *flag = f->flag;
            return f->id;
        }
        for (int r = 0; r < kSlots; ++r) {
            valid_[r] = static_cast<uint8_t>(valid_bits_ >> r & 1u);
            const auto& rw = rows_.row(ids_[r]);
            for (int e = 0; e < kTT; ++e) header_[r][e] = rw[e];
            header_[r][kTT] = r == kSlots - 1 ? top_e10_ : kHdr;
        }
        Memo m;
        m.flag = decode(rec_.data());
        m.id = records_.intern(rec_.data());
        memo_.insert(key, m);
        last_key_ = key;
        last_m_ = m;
        last_key_ok_ = true;
        *flag = m.flag;
        return m.id;
    }

    // One call on caller-held header rows (fec_sw_state_decode): every slot holds bytes (a missing
    // frame's slot is zeroed by the caller, Variable_Rate_FEC_Decoder.cpp:1710-1711).
    bool plan_state(int* const* header, uint8_t* rec) {
        for (int i = 0; i < kSlots; ++i) {
            valid_[i] = 1;
            std::memcpy(header_[i], header[i], sizeof(int) * kHdr);
        }
        return decode(rec);
    }

private:
    bool decode(uint8_t* rec) {
        const int k = k_, n = n_, TT = kTT;
        bool flag = false;
        Vec tt[kMaxN];
        uint8_t stam[kMaxN];
        int th[kMaxN];
        for (int ks = 0; ks < k; ++ks) {
            for (int c = 0; c < n; ++c) vec_zero(tt[c], n);
            int cnt = 0;
            for (int q = 0; q < n; ++q) {  // :501-508 (slot 3T-1-ks-(n-1-q))
                const int row = 3 * TT - 1 - ks - (n - 1 - q);
                th[q] = header_[row][q];
                cnt += th[q] == 0;
            }
            for (int q = 0; q < n; ++q) {  // reorder by header (:510-518)
                const int h = th[q];
                if (h != 0 && h < n + 1) {
                    const int row = 3 * TT - 1 - ks - (n - 1 - q);
                    if (valid_[row]) vec_unit(tt[h - 1], n, q);
                    else vec_zero(tt[h - 1], n);
                }
            }
            if (cnt > 0 && cnt < n - k + 1) {  // :525-533
                for (int c = 0; c < n; ++c) stam[c] = 1;
                for (int q = 0; q < n; ++q)
                    if (th[q] != 0 && th[q] < n + 1) stam[th[q] - 1] = 0;
                sym_decode(*rules_, k, n, tt, stam);
            } else if (cnt >= n - k + 1) {
                flag = true;
            }
            std::memcpy(rec + ks * n, tt[ks].c, static_cast<size_t>(n));
        }
        return flag;
    }

    struct Memo {
        int32_t id;
        bool flag;
    };
    using DestKey = FlatMap<8, Memo>::Key;  // k + n - 1 <= 28 row ids (k, n <= T_TOT + 1)
    int k_, n_;
    std::shared_ptr<const DecodeRules> rules_;
    uint8_t valid_[kSlots];
    int header_[kSlots][kHdr];
    RecordTable records_;
    std::vector<uint8_t> rec_;
    FlatMap<8, Memo> memo_;
    RowIds rows_;
    uint32_t valid_bits_ = 0;
    uint16_t ids_[kSlots] = {};
    int top_e10_ = kHdr;
    uint8_t last_hdr_[kHdr] = {};  // the last frame's header bytes and their row id
    uint16_t last_id_ = 0;
    bool last_ok_ = false;
    DestKey win_key_{};            // the current state's key (ids part kept up to date per frame)
    DestKey last_key_{};           // the last state looked up and its memo entry
    Memo last_m_{};
    bool last_key_ok_ = false;
};

struct SdRelayArgs {
    const uint8_t* cw;      // source codewords, rows of cw_stride bytes
    int64_t cw_stride;
    const int32_t* plan;    // per packet: record id
    const uint8_t* table;   // records of R bytes: header[11], coef[n2][n]
    int R;
    int64_t P;
    int k, n, n2, S, blocks;
    const uint8_t* gf;      // exp[512], log[256]
    uint8_t* frames;        // rows of F bytes
    int F;
};

struct SdDestArgs {
    const uint8_t* frames;  // relay frames, rows of F bytes; frame symbol (j, q) at 15 + j*n + q
    int F;
    const int32_t* plan;    // per seq: record id
    const uint8_t* table;   // records of k*n bytes
    int64_t P;
    int k, n, S, blocks;
    const uint8_t* gf;
    uint8_t* out;           // rows of S*k bytes
};

__global__ __launch_bounds__(kSdThreads) void fec_sdswdf_relay_kernel(SdRelayArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    for (int i = threadIdx.x; i < 512; i += kSdThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kSdThreads) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int k = a.k, n = a.n, n2 = a.n2, S = a.S;
    const int64_t total = a.P * S;
    for (int64_t id = static_cast<int64_t>(blockIdx.x) * kSdThreads + threadIdx.x; id < total;
         id += static_cast<int64_t>(gridDim.x) * kSdThreads) {
        const int64_t t = id / S;
        const int j = static_cast<int>(id - t * S);
        uint8_t* f = a.frames + t * a.F;
        const uint8_t* rec = a.table + static_cast<int64_t>(a.plan[t]) * a.R;
        if (j == 0) {  // [size BE16][header 11][codeword_new_vector's two leading zero bytes]
            const int size = (S + 1) * n2;
            f[0] = static_cast<uint8_t>(size >> 8);
            f[1] = static_cast<uint8_t>(size);
            for (int i = 0; i < kHdr; ++i) f[2 + i] = rec[i];
            f[2 + kHdr] = 0;
            f[3 + kHdr] = 0;
        }
        if (j == S - 1)
            for (int o = 4 + kHdr + S * n2; o < a.F; ++o) f[o] = 0;
        uint8_t* blk = f + 4 + kHdr + j * n2;
        if (j >= a.blocks) {  // not relayed (:184-185): stays zero
            for (int i = 0; i < n2; ++i) blk[i] = 0;
            continue;
        }
        const uint8_t* coef = rec + kHdr;
        for (int index = 0; index < n2; ++index) {
            const int64_t u0 = t - (n - 1) + (k - 1 - index);  // packet of diagonal position 0
            uint8_t acc = 0;
            for (int p = 0; p < n; ++p) {
                const uint8_t c = coef[index * n + p];
                const int64_t u = u0 + p;
                if (!c || u < 0) continue;
                const uint8_t v = a.cw[u * a.cw_stride + j * n + p];
                if (v) acc ^= gexp[glog[c] + glog[v]];
            }
            blk[index] = acc;
        }
    }
}

__global__ __launch_bounds__(kSdThreads) void fec_sdswdf_dest_kernel(SdDestArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    for (int i = threadIdx.x; i < 512; i += kSdThreads) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += kSdThreads) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int k = a.k, n = a.n, S = a.S;
    const int64_t total = a.P * S;
    for (int64_t id = static_cast<int64_t>(blockIdx.x) * kSdThreads + threadIdx.x; id < total;
         id += static_cast<int64_t>(gridDim.x) * kSdThreads) {
        const int64_t t = id / S;
        const int j = static_cast<int>(id - t * S);
        uint8_t* o = a.out + t * static_cast<int64_t>(S) * k + j * k;
        if (j >= a.blocks) {
            for (int s = 0; s < k; ++s) o[s] = 0;
            continue;
        }
        const uint8_t* coef = a.table + static_cast<int64_t>(a.plan[t]) * (k * n);
        for (int s = 0; s < k; ++s) {
            uint8_t acc = 0;
            for (int q = 0; q < n; ++q) {
                const uint8_t c = coef[s * n + q];
                const int64_t u = t - s - (n - 1 - q);
                if (!c || u < 0) continue;
                const uint8_t v = a.frames[u * a.F + 4 + kHdr + j * n + q];
                if (v) acc ^= gexp[glog[c] + glog[v]];
            }
            o[s] = acc;
        }
    }
}

// ---- tile kernels (round 5) ------------------------------------------------------------------
// The same byte work by tiles: a workgroup per TP = 4 * (64 / NS4) consecutive packets, a lane per
// (packet, group of 4 code blocks).  The rows the tile's plans read (one contiguous span) are
// staged in LDS with 16-byte loads; each record's non-zero coefficients come as a compact list
// per output row (SdEntries: per row [beg, end) into entries of p | log2(c) << 8, built on the
// host from the interned records; there were 133 records for 360 000 packets of bin/erasure.bin,
// 31 of 121 coefficients non-zero per packet, 72 % of the rows a single 1); a product is four
// branch-free log/exp lookups (log[0] = 512 past the exp table's zeros), a coefficient 1 a copy.
// The lane's 4 blocks of every output row land in an LDS output tile placed at the global rows'
// 16-byte phase, which leaves as 16-byte stores (byte stores at the tile's two ends).
struct SdTileArgs {
    const uint8_t* in;        // rows of stride bytes (source codewords / relay frames)
    int64_t stride, in_bytes; // row pitch; bytes of in (reads past them return zero)
    int in_off;               // byte of symbol (j, 0) in a row (0 / 4 + kHdr)
    const int32_t* plan;      // per packet: record id
    const uint8_t* rec;       // records (relay: header bytes at rec*R)
    int R;
    const uint32_t* ent_off;  // per record: offset of its entry block in ent (uint16 units)
    const uint16_t* ent;      // entry blocks: beg[ROWS + 1], then entries p | logc << 8
    int64_t P;
    int S, blocks;
    const uint8_t* gf;        // exp[512], log[256]
    uint8_t* out;             // relay: frames of F bytes; destination: rows of S*k bytes
    int F;
};

#ifndef FEC_SD_PASS
#define FEC_SD_PASS 1
#endif
// packets per lane and tile (halo rows staged once per tile).  2 measured slower: relay 268 vs
// 246 us, destination 129 vs 121 us per 360 000 packets (profiles/r05/relay/r05zp_*).
constexpr int kSdPass = FEC_SD_PASS;
constexpr int kSdMaxTile = 64;  // packets per tile the record-id slots hold
// shift = the row offset of an output row's diagonal: relay row index reads source packet
// t - (N-1) + (K-1-index) + p; destination row s reads frame t - s - (N2-1-q).
template <int K, int N, int ROWS, bool RELAY>
__global__ __launch_bounds__(256) void fec_sd_tile_kernel(SdTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* gexp = smem;                                          // 1040: exp[0..509], zeros after
    uint16_t* glog = reinterpret_cast<uint16_t*>(smem + 1040);    // 512: log, log[0] = 512
    int32_t* srec = reinterpret_cast<int32_t*>(smem + 1552);       // TP record ids (TP <= kSdMaxTile)
    uint8_t* raw = smem + 1552 + 4 * kSdMaxTile;                  // staged rows, then the output tile
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 1040; i += 256) gexp[i] = i < 510 ? a.gf[i] : 0;
    for (int i = tid; i < 256; i += 256) glog[i] = i ? a.gf[512 + i] : 512;
    const int S = a.S, NS4 = (S + 3) >> 2, ppw = 64 / NS4, TP = kSdPass * 4 * ppw;
    if (TP > kSdMaxTile) return;  // never launched so (sd_tile_fit): the record ids would overrun their slots
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * TP;
    const int nt = static_cast<int>(min<int64_t>(TP, a.P - t0));
    // rows read: relay [t0 - (N-1) - (ROWS-1) + (K-1), t0+nt); destination [t0 - (K-1) - (N-1), t0+nt)
    constexpr int BACK = RELAY ? (N - 1) + (ROWS - 1) - (K - 1) : (ROWS - 1) + (N - 1);
    const int64_t r0 = t0 - BACK;
    const int nrows = nt + BACK;
    const int64_t g0 = r0 * a.stride;
    const int64_t A = g0 >= 0 ? (g0 & ~int64_t(15)) : -((-g0 + 15) & ~int64_t(15));
    const int dlt = static_cast<int>(g0 - A);
    const int span = dlt + nrows * static_cast<int>(a.stride);
    {
        const int64_t base = A > 0 ? A : 0, lim = a.in_bytes - base;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(a.in + base), 0, static_cast<int>(lim < fec::kRsrcMax ? lim : fec::kRsrcMax), 0x00020000);
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        for (int c = tid; 16 * c < span; c += 256) {
            const int64_t o = A + 16 * c;  // bytes before the array read as zero (rows before seq 0)
            const v4 v = o < 0 ? v4{0, 0, 0, 0}
                               : __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(o - base), 0, 0);
            *reinterpret_cast<v4*>(raw + 16 * c) = v;
        }
    }
    if (tid < nt) srec[tid] = a.plan[t0 + tid];
    __syncthreads();
    const int pl = lane / NS4, g = lane - pl * NS4;
    uint32_t A4[kSdPass][ROWS];
#pragma unroll
    for (int ps = 0; ps < kSdPass; ++ps) {
    const int tl = (ps * 4 + wv) * ppw + pl;  // the lane's packet in the tile
    const bool on = pl < ppw && tl < nt;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) A4[ps][r] = 0;
    if (on) {
        const int rid = srec[tl];
        const uint16_t* eb = a.ent + a.ent_off[rid];
        const uint8_t* rowbase = raw + dlt + a.in_off + 4 * g * N;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            // row of the diagonal's symbol p, relative to r0
            const int lr0 = RELAY ? tl + (ROWS - 1) - r : tl + (K - 1) - r;  // + p (relay) / + q (destination)
            uint32_t acc = 0;
            for (int e = eb[r]; e < eb[r + 1]; ++e) {
                const uint32_t en = eb[ROWS + 1 + e];
                const int p = static_cast<int>(en & 0xff), lc = static_cast<int>(en >> 8);
                const uint8_t* sp = rowbase + (lr0 + p) * static_cast<int>(a.stride) + p;
                uint32_t w = 0;
                if (lc == 0) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) w |= static_cast<uint32_t>(sp[q * N]) << (8 * q);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) w |= static_cast<uint32_t>(gexp[lc + glog[sp[q * N]]]) << (8 * q);
                }
                acc ^= w;
            }
            A4[ps][r] = acc;
        }
    }
    }
    __syncthreads();  // the staged rows are read: the output tile takes their place
    const int OB = RELAY ? a.F : S * K;                 // output row bytes
    const int64_t ob0 = t0 * OB;
    const int odl = static_cast<int>(ob0 & 15);
    uint8_t* ot = raw + odl;                            // output byte b of row tl at ot[tl * OB + b]
#pragma unroll
    for (int ps = 0; ps < kSdPass; ++ps) {
    const int tl = (ps * 4 + wv) * ppw + pl;
    const bool on = pl < ppw && tl < nt;
    if (on) {
        uint8_t* orow = ot + tl * OB;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = 4 * g + q;
            if (j >= S) break;
            const bool keep = j < a.blocks;  // blocks past ceil(max_payload/k)+1 stay zero (:184-185)
            uint8_t* d = orow + (RELAY ? 4 + kHdr + j * ROWS : j * K);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) d[r] = keep ? static_cast<uint8_t>(A4[ps][r] >> (8 * q)) : 0;
        }
        if (RELAY && g == 0) {  // [size BE16][header 11][2 zero bytes] ... [zero tail]
            const int size = (S + 1) * ROWS;
            orow[0] = static_cast<uint8_t>(size >> 8);
            orow[1] = static_cast<uint8_t>(size);
            const uint8_t* h = a.rec + static_cast<int64_t>(srec[tl]) * a.R;
            for (int i = 0; i < kHdr; ++i) orow[2 + i] = h[i];
            orow[2 + kHdr] = 0;
            orow[3 + kHdr] = 0;
            for (int o = 4 + kHdr + S * ROWS; o < OB; ++o) orow[o] = 0;
        }
    }
    }
    __syncthreads();
    const int obytes = nt * OB;
    uint8_t* dst = a.out + ob0 - odl;  // 16-byte aligned when out is
    for (int c = tid; 16 * c < odl + obytes; c += 256) {
        const int lo = 16 * c;
        if (lo >= odl && lo + 16 <= odl + obytes && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            *reinterpret_cast<uint4*>(dst + lo) = *reinterpret_cast<const uint4*>(raw + lo);
        } else {
            for (int b = max(lo, odl); b < min(lo + 16, odl + obytes); ++b) dst[b] = raw[b];
        }
    }
}

#define FEC_SD_TILE_LIST(X) \
    X(11, 11, 11) X(10, 11, 11) X(9, 11, 11) X(8, 11, 11) X(7, 11, 11) X(6, 11, 11) X(5, 11, 11) X(4, 11, 11) \
    X(6, 11, 9) X(8, 11, 9)
#define FEC_SD_TILE_INST(K, N, N2) \
    template __global__ void fec_sd_tile_kernel<K, N, N2, true>(SdTileArgs); \
    template __global__ void fec_sd_tile_kernel<K, N2, K, false>(SdTileArgs);
FEC_SD_TILE_LIST(FEC_SD_TILE_INST)

// The tile kernel for the relay (k, n1, n2) / the destination (k, n2), or nullptr.
const void* sd_tile_kernel_for(bool relay, int k, int n1, int n2) {
#define FEC_SD_TILE_CASE(K, N, N2)                                                                        \
    if (k == K && n2 == N2 && (!relay || n1 == N))                                                     \
        return relay ? reinterpret_cast<const void*>(&fec_sd_tile_kernel<K, N, N2, true>)               \
                     : reinterpret_cast<const void*>(&fec_sd_tile_kernel<K, N2, K, false>);
    FEC_SD_TILE_LIST(FEC_SD_TILE_CASE)
#undef FEC_SD_TILE_CASE
    return nullptr;
}

// Entry blocks of a record table: per record, for each of its `rows` output rows of `cols`
// coefficients (starting at byte `first` of the record), the non-zero ones as p | log2(c) << 8.
void build_entries(const std::vector<uint8_t>& recs, int R, int first, int rows, int cols, std::vector<uint32_t>& off,
                   std::vector<uint16_t>& ent) {
    const Field& F = field();
    const size_t nrec = R > 0 ? recs.size() / static_cast<size_t>(R) : 0;
    off.assign(std::max<size_t>(nrec, 1), 0);
    ent.clear();
    for (size_t r = 0; r < nrec; ++r) {
        off[r] = static_cast<uint32_t>(ent.size());
        const uint8_t* c = recs.data() + r * static_cast<size_t>(R) + first;
        const size_t b0 = ent.size();
        ent.resize(b0 + static_cast<size_t>(rows) + 1, 0);
        std::vector<uint16_t> list;
        for (int i = 0; i < rows; ++i) {
            ent[b0 + static_cast<size_t>(i)] = static_cast<uint16_t>(list.size());
            for (int p = 0; p < cols; ++p)
                if (uint8_t v = c[i * cols + p]) list.push_back(static_cast<uint16_t>(p | (F.log[v] << 8)));
        }
        ent[b0 + static_cast<size_t>(rows)] = static_cast<uint16_t>(list.size());
        ent.insert(ent.end(), list.begin(), list.end());
    }
    if (ent.empty()) ent.push_back(0);
}

int grid_for(int64_t items) {
    return static_cast<int>(std::min<int64_t>((items + kSdThreads - 1) / kSdThreads, 16384));
}

// A device buffer that only grows.
// The frames' 11-byte headers gathered into contiguous rows [P][11] (one thread per header byte),
// so that the destination planner's read-back is one linear copy.
__global__ __launch_bounds__(256) void fec_sdswdf_hdr_gather_kernel(const uint8_t* frames, int64_t F, int64_t P,
                                                                     uint8_t* hdrs) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= P * kHdr) return;
    const int64_t r = i / kHdr;
    hdrs[i] = frames[r * F + 2 + (i - r * kHdr)];
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t want) {
        if (want <= bytes) return FEC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, want) != hipSuccess) return FEC_ERR_NOMEM;
        bytes = want;
        return FEC_OK;
    }
};

}  // namespace

// Per-call planning on explicit state for the two-hop session (fec_session.hip): one planner per
// geometry, kept for the process (the drop-in methods keep theirs in SwCtx).
int sd_relay_plan_state(int k, int n, int n2, int sdbo, const uint8_t* er, int* const* header, uint8_t* rec) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, int>, std::unique_ptr<SdRelayPlanner>> pls;
    if (k < 1 || n < k || n > kHdr || n2 < k || n2 > kHdr || (sdbo != 0 && sdbo != 1)) return FEC_ERR_ARG;
    std::lock_guard<std::mutex> lk(mu);
    auto& pl = pls[std::make_tuple(k, n, n2, sdbo)];
    if (!pl)
        pl.reset(new SdRelayPlanner(k, n, n2, sdbo, shared_decode_rules(n - 1, n - k, n - k),
                                    make_generator(n2 - 1, n2 - k, n2 - k)));
    pl->plan_state(er, header, rec);
    return FEC_OK;
}
int sd_relay_record_bytes(int n, int n2) { return kHdr + n2 * n; }
int sd_dest_plan_state(int k, int n, int* const* header, uint8_t* rec, bool* flag) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::unique_ptr<SdDestPlanner>> pls;
    if (k < 1 || n < k || n > kHdr) return FEC_ERR_ARG;
    std::lock_guard<std::mutex> lk(mu);
    auto& pl = pls[std::make_pair(k, n)];
    if (!pl) pl.reset(new SdDestPlanner(k, n, shared_decode_rules(n - 1, n - k, n - k)));
    *flag = pl->plan_state(header, rec);
    return FEC_OK;
}
}  // namespace fec

struct fec_sdswdf {
    // hop 1: Decoder(n1-1, n1-k, n1-k), the relay's decoder_current; hop 2: Encoder(n2-1, n2-k,
    // n2-k) / the destination's decoder_current.  The device constants (the GF tables the kernels
    // stage) come with the hop codecs, created on the first batch call: the planners are host only.
    fec::Geometry g1, g2;
    int T1 = 0, N1 = 0, T2 = 0, N2 = 0;
    fec_codec* hop1 = nullptr;
    fec_codec* hop2 = nullptr;
    fec::CodecView v1, v2;
    int sdbo = 0, blocks = 0, F = 0;
    std::unique_ptr<fec::SdRelayPlanner> relay;
    std::unique_ptr<fec::SdDestPlanner> dest;
    std::vector<int32_t> plan;
    std::vector<uint8_t> hdrs;
    fec::DevBuf d_plan, d_table, d_hdrs, d_eoff, d_ent;
    std::vector<uint32_t> eoff;
    std::vector<uint16_t> ent;
    ~fec_sdswdf() {
        if (hop1) fec_codec_destroy(hop1);
        if (hop2) fec_codec_destroy(hop2);
    }
};

namespace {

int ensure_device(fec_sdswdf* w) {
    if (w->hop1) return FEC_OK;
    if (int st = fec_codec_create(w->g1.L, w->T1, w->N1, w->N1, &w->hop1)) return st;
    if (int st = fec_codec_create(w->g2.L, w->T2, w->N2, w->N2, &w->hop2)) return st;
    fec::codec_view(w->hop1, &w->v1);
    fec::codec_view(w->hop2, &w->v2);
    return FEC_OK;
}

// The relay's host plan for seqs 0..P-1 of a fresh relay: record ids in w->plan, records in
// w->relay->records().  starts (sorted, may be null): rows at which a fresh relay takes over (the
// rows of several independent streams laid end to end, fec_relay_vr).
void plan_relay(fec_sdswdf* w, const uint8_t* h_erasure, int64_t P, const int64_t* starts = nullptr, int nstarts = 0) {
    w->relay->reset();
    w->plan.resize(static_cast<size_t>(P));
    int si = 0;
    for (int64_t t = 0; t < P; ++t) {
        while (si < nstarts && starts[si] <= t) {
            if (starts[si++] == t) w->relay->restart();
        }
        w->plan[static_cast<size_t>(t)] = w->relay->step(h_erasure[t] != 0);
    }
}

// The destination's host plan for seqs 0..P-1 given the frames' header bytes (11 per seq).
void plan_dest(fec_sdswdf* w, const uint8_t* h_erasure, const uint8_t* hdrs, int64_t P, uint8_t* h_flag,
               const int64_t* starts = nullptr, int nstarts = 0) {
    w->dest->reset();
    w->plan.resize(static_cast<size_t>(P));
    int si = 0;
    for (int64_t t = 0; t < P; ++t) {
        while (si < nstarts && starts[si] <= t) {
            if (starts[si++] == t) w->dest->restart();
        }
        bool fl = false;
        w->plan[static_cast<size_t>(t)] = w->dest->step(h_erasure[t] != 0, hdrs + t * fec::kHdr, &fl);
        if (h_flag) h_flag[t] = fl ? 1 : 0;
    }
}

int upload_plan(fec_sdswdf* w, const fec::RecordTable& tab, int64_t P, hipStream_t s) {
    const size_t pb = static_cast<size_t>(P) * sizeof(int32_t);
    const size_t tb = std::max<size_t>(tab.data().size(), 1);
    if (int st = w->d_plan.reserve(pb)) return st;
    if (int st = w->d_table.reserve(tb)) return st;
    FEC_HIP(hipMemcpyAsync(w->d_plan.p, w->plan.data(), pb, hipMemcpyHostToDevice, s));
    if (!tab.data().empty())
        FEC_HIP(hipMemcpyAsync(w->d_table.p, tab.data().data(), tab.data().size(), hipMemcpyHostToDevice, s));
    return FEC_OK;
}

}  // namespace

namespace fec {
// Whether the tile kernel (fec_sd_tile_kernel) takes a batch of this geometry, its tile (TP
// packets) and its dynamic LDS: it needs an instantiation for (k, n1, n2), at most 64 lanes of 4
// code blocks per packet, at most 64 packets per tile (the kernel's record-id slots: 256 bytes of
// LDS in front of the staged rows -- a larger tile wrote its ids over the rows and read garbage
// record ids back, the memory fault behind r05zp's HIP error) and 64 KB of LDS.
bool sd_tile_fit(bool relay, int k, int n1, int n2, int S, int F, int64_t stride, int* TP_out, int64_t* lds_out) {
    const int NS4 = (S + 3) / 4;
    if (!sd_tile_kernel_for(relay, k, n1, n2) || NS4 > 64) return false;
    const int TP = kSdPass * 4 * (64 / NS4);
    if (TP > kSdMaxTile) return false;
    const int N = relay ? n1 : n2, ROWS = relay ? n2 : k;
    const int back = relay ? (N - 1) + (ROWS - 1) - (k - 1) : (ROWS - 1) + (N - 1);
    const int OB = relay ? F : S * k;
    const int64_t stage = 16 + static_cast<int64_t>(TP + back) * stride + 16, otile = 16 + static_cast<int64_t>(TP) * OB + 16;
    const int64_t lds = 1552 + 4 * kSdMaxTile + ((std::max(stage, otile) + 15) & ~int64_t(15));
    if (lds > 65536) return false;
    if (TP_out) *TP_out = TP;
    if (lds_out) *lds_out = lds;
    return true;
}
}  // namespace fec

namespace {

// The tile kernels (fec_sd_tile_kernel): the records' entry blocks up, then one launch; returns
// 1 when the tile kernel does not apply (the caller launches the per-(packet, block) kernel).
int launch_tile(fec_sdswdf* w, bool relay, const fec::RecordTable& tab, const uint8_t* d_in, int64_t stride,
                int64_t P, uint8_t* d_out, hipStream_t s) {
    const char* e = std::getenv("FEC_SD_TILE");
    if (e && e[0] == '0') return 1;
    const int k = w->g1.k, n1 = w->g1.n, n2 = w->g2.n, S = w->g1.S;
    const void* kern = fec::sd_tile_kernel_for(relay, k, n1, n2);
    int TP = 0;
    int64_t lds = 0;
    if (!fec::sd_tile_fit(relay, k, n1, n2, S, w->F, stride, &TP, &lds)) return 1;
    const int N = relay ? n1 : n2, ROWS = relay ? n2 : k;
    const int R = relay ? fec::kHdr + n2 * n1 : k * n2;
    fec::build_entries(tab.data(), R, relay ? fec::kHdr : 0, ROWS, N, w->eoff, w->ent);
    if (int st = w->d_eoff.reserve(w->eoff.size() * 4)) return st;
    if (int st = w->d_ent.reserve(w->ent.size() * 2)) return st;
    FEC_HIP(hipMemcpyAsync(w->d_eoff.p, w->eoff.data(), w->eoff.size() * 4, hipMemcpyHostToDevice, s));
    FEC_HIP(hipMemcpyAsync(w->d_ent.p, w->ent.data(), w->ent.size() * 2, hipMemcpyHostToDevice, s));
    fec::SdTileArgs a;
    a.in = d_in;
    a.stride = stride;
    a.in_bytes = P * stride;
    a.in_off = relay ? 0 : 4 + fec::kHdr;
    a.plan = static_cast<const int32_t*>(w->d_plan.p);
    a.rec = static_cast<const uint8_t*>(w->d_table.p);
    a.R = R;
    a.ent_off = static_cast<const uint32_t*>(w->d_eoff.p);
    a.ent = static_cast<const uint16_t*>(w->d_ent.p);
    a.P = P;
    a.S = S;
    a.blocks = w->blocks;
    a.gf = relay ? w->v1.gf : w->v2.gf;
    a.out = d_out;
    a.F = w->F;
    void* args[] = {&a};
    const unsigned grid = static_cast<unsigned>((P + TP - 1) / TP);
    FEC_HIP(hipLaunchKernel(kern, dim3(grid), dim3(256), args, static_cast<size_t>(lds), s));
    return FEC_OK;
}

template <class F>
int guarded_sd(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}

}  // namespace

// ---- per-call relay methods on caller-held state (the drop-in Decoder_Symbol_Wise) -----------
namespace fec {
namespace {

constexpr int kSwMaxOut = 32;

// out[o][j] = XOR_p coef[o][p] * src_o[(rbase_o + p) * row_bytes_o + j * bs_o + p] for j < blocks:
// one GF dot product per output symbol over a diagonal of a packed window (rows = the caller's
// slots, each packed from its first symbol's byte on).
struct SwApplyArgs {
    const uint8_t* win[2];   // packed windows (device view of pinned host memory)
    int row_bytes[2];
    int bs[2];               // bytes per code block in a row
    int nout, nin, blocks;
    int src[kSwMaxOut];
    int rbase[kSwMaxOut];
    const uint8_t* coef;     // [nout][nin]
    const uint8_t* gf;
    uint8_t* res;            // [nout][blocks]
};

__global__ __launch_bounds__(256) void fec_sw_apply_kernel(SwApplyArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    for (int i = threadIdx.x; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = threadIdx.x; i < 256; i += 256) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int total = a.nout * a.blocks;
    for (int id = blockIdx.x * 256 + threadIdx.x; id < total; id += gridDim.x * 256) {
        const int o = id / a.blocks, j = id - o * a.blocks;
        const int sidx = a.src[o];
        const uint8_t* w = a.win[sidx];
        const int rb = a.row_bytes[sidx], bs = a.bs[sidx];
        uint8_t acc = 0;
        for (int p = 0; p < a.nin; ++p) {
            const uint8_t c = a.coef[o * a.nin + p];
            if (!c) continue;
            const uint8_t v = w[(a.rbase[o] + p) * rb + j * bs + p];
            if (v) acc ^= gexp[glog[c] + glog[v]];
        }
        a.res[id] = acc;
    }
}

// Pinned, mapped staging for one call (windows, coefficients, results), GF tables on the device,
// a stream; calls are serialised (the reference relay is single-threaded).
struct SwCtx {
    std::mutex mu;
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
    uint8_t* d_gf = nullptr;
    hipStream_t s = nullptr;
    std::map<std::tuple<int, int, int, int, int>, std::unique_ptr<SdRelayPlanner>> relays;
    std::map<std::pair<int, int>, std::unique_ptr<SdDestPlanner>> dests;
    int ensure(size_t bytes) {
        if (!s) FEC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        if (!d_gf) {
            const Field& F = field();
            std::vector<uint8_t> gf(F.exp, F.exp + 512);
            gf.insert(gf.end(), F.log, F.log + 256);
            if (hipMalloc(&d_gf, gf.size()) != hipSuccess) return FEC_ERR_NOMEM;
            FEC_HIP(hipMemcpy(d_gf, gf.data(), gf.size(), hipMemcpyHostToDevice));
        }
        if (bytes <= cap) return FEC_OK;
        if (h) (void)hipHostFree(h);
        h = d = nullptr;
        cap = 0;
        const size_t c = std::max<size_t>(bytes, 64 * 1024);
        if (hipHostMalloc(reinterpret_cast<void**>(&h), c, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return FEC_ERR_NOMEM;
        FEC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
        cap = c;
        return FEC_OK;
    }
};
SwCtx& sw_ctx() {
    static SwCtx* c = new SwCtx();  // process lifetime (no teardown order with the HIP runtime)
    return *c;
}

// Pack rows [lo, lo+nrows) of `rows` (caller's slots), bytes [off, off + len) of each, into dst.
void sw_pack(uint8_t* dst, int row_bytes, uint8_t* const* rows, int lo, int nrows, int off, int len) {
    for (int r = 0; r < nrows; ++r) {
        std::memcpy(dst + static_cast<size_t>(r) * row_bytes, rows[lo + r] + off, static_cast<size_t>(len));
        std::memset(dst + static_cast<size_t>(r) * row_bytes + len, 0, static_cast<size_t>(row_bytes - len));
    }
}

int sw_run(SwCtx& c, SwApplyArgs& a) {
    const int total = a.nout * a.blocks;
    hipLaunchKernelGGL(fec_sw_apply_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0, c.s, a);
    FEC_HIP(hipGetLastError());
    FEC_HIP(hipStreamSynchronize(c.s));
    return FEC_OK;
}

// The decode rule of a full window (decodeBlock T = n-1, t = 0) on unit vectors, as coefficient rows:
// position q's value after the decode = row q over the n positions.
void sw_decode_rows(int k, int n, const uint8_t* er, uint8_t* rows /* n x n */) {
    std::memset(rows, 0, static_cast<size_t>(n) * n);
    for (int q = 0; q < n; ++q) rows[q * n + q] = 1;  // received (or erased: the slot holds zeros)
    uint32_t mask = 0;
    for (int c = 0; c < n; ++c) mask |= (er[c] ? 1u : 0u) << c;
    if (__builtin_popcount(mask) == n) return;
    const auto rules = shared_decode_rules(n - 1, n - k, n - k);
    const uint8_t* e = rules->entry(n, mask);
    for (int i = 0; i < k; ++i) {
        if (!((mask >> i) & 1u) || e[i] == 0xFF) continue;
        std::memcpy(rows + i * n, e + k + i * n, static_cast<size_t>(n));
    }
}

}  // namespace
}  // namespace fec

extern "C" {

int fec_sw_state_encode(int max_payload, int k, int n, int k2, int n2, int sdbo, uint8_t* const* slots,
                        const uint8_t* er, int* const* header, uint8_t* cnv, uint8_t* cnsw) {
    using namespace fec;
    if (!slots || !er || !header || !cnv || !cnsw || k < 1 || n < k || n > kHdr || k2 != k || n2 < k || n2 < 2 ||
        n2 > n || max_payload < 1 || (sdbo != 0 && sdbo != 1))
        return FEC_ERR_ARG;
    SwCtx& c = sw_ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    return guarded_sd([&] {
        auto& pl = c.relays[std::make_tuple(k, n, n2, sdbo, max_payload)];
        if (!pl)
            pl.reset(new SdRelayPlanner(k, n, n2, sdbo, shared_decode_rules(n - 1, n - k, n - k),
                                        make_generator(n2 - 1, n2 - k2, n2 - k2)));
        std::vector<uint8_t> rec(static_cast<size_t>(pl->record_bytes()));
        pl->plan_state(er, header, rec.data());
        const int blocks = max_payload / k + 1;  // :184-185
        const int lo = 2 * kTT - n + 1 - (n2 - k), nrows = 2 * kTT - lo + 1;
        const int rb = (blocks * n + 3) & ~3;
        const size_t wbytes = static_cast<size_t>(nrows) * rb, cbytes = static_cast<size_t>(n2) * n;
        if (int st = c.ensure(wbytes + cbytes + static_cast<size_t>(n2) * blocks + 64)) return st;
        sw_pack(c.h, rb, slots, lo, nrows, 2, blocks * n);
        std::memcpy(c.h + wbytes, rec.data() + kHdr, cbytes);
        SwApplyArgs a{};
        a.win[0] = a.win[1] = c.d;
        a.row_bytes[0] = a.row_bytes[1] = rb;
        a.bs[0] = a.bs[1] = n;
        a.nout = n2;
        a.nin = n;
        a.blocks = blocks;
        for (int o = 0; o < n2; ++o) {
            a.src[o] = 0;
            a.rbase[o] = (k - 1 - o) + 2 * kTT - n + 1 - lo;  // diagonal of symInd = k-1-o
        }
        a.coef = c.d + wbytes;
        a.gf = c.d_gf;
        a.res = c.d + wbytes + cbytes;
        if (int st = sw_run(c, a)) return st;
        const uint8_t* res = c.h + wbytes + cbytes;
        for (int j = 0; j < blocks; ++j)
            for (int i = 0; i < n2; ++i) {
                cnsw[2 + j * n2 + i] = res[i * blocks + j];  // :277-393
                cnv[2 + j * n2 + i] = res[i * blocks + j];   // :405-409
            }
        return static_cast<int>(FEC_OK);
    });
}

int fec_sw_state_decode(int max_payload, int k, int n, uint8_t* const* slots, int* const* header, uint8_t* buffer,
                        int* flag) {
    using namespace fec;
    if (!slots || !header || !buffer || k < 1 || n < k || n > kHdr || max_payload < 1) return FEC_ERR_ARG;
    SwCtx& c = sw_ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    return guarded_sd([&] {
        auto& pl = c.dests[std::make_pair(k, n)];
        if (!pl) pl.reset(new SdDestPlanner(k, n, shared_decode_rules(n - 1, n - k, n - k)));
        std::vector<uint8_t> rec(static_cast<size_t>(pl->record_bytes()));
        const bool fl = pl->plan_state(header, rec.data());
        if (flag) *flag = fl ? 1 : 0;
        const int blocks = max_payload / k + 1;  // :494
        const int lo = 3 * kTT - 1 - (k - 1) - (n - 1), nrows = 3 * kTT - lo;
        const int rb = (blocks * n + 3) & ~3;
        const size_t wbytes = static_cast<size_t>(nrows) * rb, cbytes = static_cast<size_t>(k) * n;
        if (int st = c.ensure(wbytes + cbytes + static_cast<size_t>(k) * blocks + 64)) return st;
        sw_pack(c.h, rb, slots, lo, nrows, 4, blocks * n);  // symbol (j, q) at slot byte 4 + j*n + q (:504)
        std::memcpy(c.h + wbytes, rec.data(), cbytes);
        SwApplyArgs a{};
        a.win[0] = a.win[1] = c.d;
        a.row_bytes[0] = a.row_bytes[1] = rb;
        a.bs[0] = a.bs[1] = n;
        a.nout = k;
        a.nin = n;
        a.blocks = blocks;
        for (int o = 0; o < k; ++o) {
            a.src[o] = 0;
            a.rbase[o] = 3 * kTT - 1 - o - (n - 1) - lo;  // frame t2-o-(n-1-q) for position q
        }
        a.coef = c.d + wbytes;
        a.gf = c.d_gf;
        a.res = c.d + wbytes + cbytes;
        if (int st = sw_run(c, a)) return st;
        const uint8_t* res = c.h + wbytes + cbytes;
        for (int j = 0; j < blocks; ++j)
            for (int ks = 0; ks < k; ++ks) buffer[j * n + n - k + ks] = res[ks * blocks + j];  // :537
        return static_cast<int>(FEC_OK);
    });
}

int fec_sw_encode_1(int max_payload, int k, int n, int k2, int n2, uint8_t* const* cv, const uint8_t* er,
                    uint8_t* const* cnv, uint8_t* cnsw, int* flag) {
    using namespace fec;
    if (!cv || !er || !cnv || !cnsw || k < 1 || n < k || n > kMaxRuleN || k2 != k || n2 < k2 || n2 > kSwMaxOut ||
        max_payload < 1)
        return FEC_ERR_ARG;
    SwCtx& c = sw_ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    return guarded_sd([&] {
        const int blocks = max_payload / k + 1;  // :553
        int cnt = 0;
        for (int i = 0; i < n; ++i) cnt += er[i] ? 1 : 0;
        if (flag) *flag = cnt >= n - k + 1 ? 1 : 0;  // :574-576
        // the decode (:570-573; the n flags of the window reach decodeBlock), then
        // the k data symbols reversed (:577-578)
        std::vector<uint8_t> rows(static_cast<size_t>(n) * n);
        if (cnt > 0 && cnt < n - k + 1) {
            sw_decode_rows(k, n, er, rows.data());
        } else {
            std::memset(rows.data(), 0, rows.size());
            for (int q = 0; q < n; ++q) rows[q * n + q] = 1;
        }
        const int npar = n2 - k2;
        const int nout = k + npar;
        const int rbA = (blocks * n + 3) & ~3, rbB = (blocks * n2 + 3) & ~3;
        const size_t wA = static_cast<size_t>(n) * rbA, wB = static_cast<size_t>(std::max(1, n2 - 1)) * rbB;
        const int nin = std::max(n, k);
        const size_t cbytes = static_cast<size_t>(nout) * nin;
        if (int st = c.ensure(wA + wB + cbytes + static_cast<size_t>(nout) * blocks + 64)) return st;
        sw_pack(c.h, rbA, cv, 0, n, 2, blocks * n);                     // diagonal d[i] = cv[i][2+j*n+i] (:567)
        if (n2 > 1) sw_pack(c.h + wA, rbB, cnv, 0, n2 - 1, 2, blocks * n2);  // the relay's earlier frames
        uint8_t* cf = c.h + wA + wB;
        std::memset(cf, 0, cbytes);
        SwApplyArgs a{};
        a.win[0] = c.d;
        a.win[1] = c.d + wA;
        a.row_bytes[0] = rbA;
        a.row_bytes[1] = rbB;
        a.bs[0] = n;
        a.bs[1] = n2;
        a.nout = nout;
        a.nin = nin;
        a.blocks = blocks;
        for (int i = 0; i < k; ++i) {  // output i: decoded position k-1-i
            a.src[i] = 0;
            a.rbase[i] = 0;
            std::memcpy(cf + i * nin, rows.data() + (k - 1 - i) * n, static_cast<size_t>(n));
        }
        // parity position n2-1-delta (:601-613): XOR_m G2[m][n2-1-delta] * cnv[m+delta][2+j*n2+m]
        const std::vector<uint8_t> G2 = make_generator(n2 - 1, n2 - k2, n2 - k2);
        for (int delta = 0; delta < npar; ++delta) {
            const int o = k + delta;
            a.src[o] = 1;
            a.rbase[o] = delta;
            for (int m = 0; m < k; ++m) cf[o * nin + m] = G2[m * n2 + n2 - 1 - delta];
        }
        a.coef = c.d + wA + wB;
        a.gf = c.d_gf;
        a.res = c.d + wA + wB + cbytes;
        if (int st = sw_run(c, a)) return st;
        const uint8_t* res = c.h + wA + wB + cbytes;
        for (int j = 0; j < blocks; ++j) {
            for (int i = 0; i < k; ++i) {
                cnsw[2 + j * n + i] = res[i * blocks + j];
                cnv[n2 - 1][2 + j * n2 + i] = res[i * blocks + j];  // :593-597 (k_min = k, delta_k = 0)
            }
            for (int delta = 0; delta < npar; ++delta) cnv[n2 - 1][2 + j * n2 + n2 - 1 - delta] = res[(k + delta) * blocks + j];
        }
        return static_cast<int>(FEC_OK);
    });
}

int fec_sw_decode_1(int max_payload, int k, int n, uint8_t* const* cv, const uint8_t* er, uint8_t* buffer, int* flag) {
    using namespace fec;
    if (!cv || !er || !buffer || k < 1 || n < k || n > kMaxRuleN || max_payload < 1) return FEC_ERR_ARG;
    SwCtx& c = sw_ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    return guarded_sd([&] {
        const int blocks = max_payload / k + 1;  // :632
        int cnt = 0;
        for (int i = 0; i < n; ++i) cnt += er[i] ? 1 : 0;
        if (flag) *flag = cnt >= n - k + 1 ? 1 : 0;  // :644-646
        std::vector<uint8_t> rows(static_cast<size_t>(n) * n);
        if (cnt > 0 && cnt < n - k + 1) {
            sw_decode_rows(k, n, er, rows.data());
        } else {
            std::memset(rows.data(), 0, rows.size());
            for (int q = 0; q < n; ++q) rows[q * n + q] = 1;
        }
        const int rb = (blocks * n + 3) & ~3;
        const size_t wbytes = static_cast<size_t>(n) * rb, cbytes = static_cast<size_t>(n) * n;
        if (int st = c.ensure(wbytes + cbytes + static_cast<size_t>(n) * blocks + 64)) return st;
        sw_pack(c.h, rb, cv, 0, n, 4, blocks * n);  // position q = cv[q][4 + j*n + q] (:636-639)
        std::memcpy(c.h + wbytes, rows.data(), cbytes);
        SwApplyArgs a{};
        a.win[0] = a.win[1] = c.d;
        a.row_bytes[0] = a.row_bytes[1] = rb;
        a.bs[0] = a.bs[1] = n;
        a.nout = n;
        a.nin = n;
        a.blocks = blocks;
        for (int o = 0; o < n; ++o) {
            a.src[o] = 0;
            a.rbase[o] = 0;
        }
        a.coef = c.d + wbytes;
        a.gf = c.d_gf;
        a.res = c.d + wbytes + cbytes;
        if (int st = sw_run(c, a)) return st;
        const uint8_t* res = c.h + wbytes + cbytes;
        for (int j = 0; j < blocks; ++j)
            for (int i = 0; i < n; ++i) buffer[j * n + i] = res[(n - 1 - i) * blocks + j];  // :647-649
        return static_cast<int>(FEC_OK);
    });
}

int fec_sdswdf_create(int max_payload, int T1, int N1, int T2, int N2, int sdbo, fec_sdswdf** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    // k2 == k (the only case Decoder_Symbol_Wise handles, :185), n2 <= n1 (the selection reads
    // temp_codeword[i] for i < n2, :367), T <= T_TOT (header rows hold T_TOT+1 entries), n2 >= 2
    // (a frame's (S+1)*n2 code bytes hold the 2 offset bytes and S blocks only when n2 >= 2)
    if (T1 < 0 || N1 < 0 || T2 < 1 || N2 < 0 || T1 - N1 != T2 - N2 || T1 - N1 + 1 < 1 || T1 > fec::kTT ||
        T2 > T1 || (sdbo != 0 && sdbo != 1))
        return FEC_ERR_ARG;
    return guarded_sd([&] {
        std::unique_ptr<fec_sdswdf> w(new fec_sdswdf());
        w->g1 = fec::Geometry::make(max_payload, T1, N1, N1);
        w->g2 = fec::Geometry::make(max_payload, T2, N2, N2);
        w->T1 = T1;
        w->N1 = N1;
        w->T2 = T2;
        w->N2 = N2;
        const int k = w->g1.k, n1 = w->g1.n, n2 = w->g2.n;
        w->sdbo = sdbo;
        w->blocks = max_payload / k + 1;  // ceil(max_payload / k) + 1 on ints (:184-185)
        w->F = 2 + fec::kHdr + (w->g1.S + 1) * n2;
        w->relay.reset(new fec::SdRelayPlanner(k, n1, n2, sdbo, fec::shared_decode_rules(T1, N1, N1),
                                               fec::make_generator(T2, N2, N2)));
        w->dest.reset(new fec::SdDestPlanner(k, n2, fec::shared_decode_rules(T2, N2, N2)));
        *out = w.release();
        return static_cast<int>(FEC_OK);
    });
}

int fec_sdswdf_destroy(fec_sdswdf* w) {
    delete w;
    return FEC_OK;
}

int fec_sdswdf_tile_geometry(int relay, int max_payload, int T1, int N1, int T2, int N2, int64_t stride,
                             int* tile_packets, int* lds_bytes) {
    if (max_payload < 0 || T1 < 0 || N1 < 0 || N1 > T1 || T2 < 1 || N2 < 0 || T1 - N1 != T2 - N2) return FEC_ERR_ARG;
    const int k = T1 - N1 + 1, n1 = T1 + 1, n2 = T2 + 1, S = (max_payload + 2 + k - 1) / k;
    const int F = 2 + fec::kHdr + (S + 1) * n2;
    if (stride <= 0) stride = relay ? static_cast<int64_t>(S) * n1 : F;
    int TP = 0;
    int64_t lds = 0;
    const bool fit = fec::sd_tile_fit(relay != 0, k, n1, n2, S, F, stride, &TP, &lds);
    if (tile_packets) *tile_packets = fit ? TP : 0;
    if (lds_bytes) *lds_bytes = fit ? static_cast<int>(lds) : 0;
    return fit ? 1 : 0;
}

int fec_sdswdf_geometry(const fec_sdswdf* w, int* k, int* n1, int* n2, int* S, int* blocks, int* frame_bytes,
                        int* delay) {
    if (!w) return FEC_ERR_ARG;
    if (k) *k = w->g1.k;
    if (n1) *n1 = w->g1.n;
    if (n2) *n2 = w->g2.n;
    if (S) *S = w->g1.S;
    if (blocks) *blocks = w->blocks;
    if (frame_bytes) *frame_bytes = w->F;
    if (delay) *delay = w->g1.n + w->g2.n - w->g1.k - 1;
    return FEC_OK;
}

int fec_sdswdf_relay_plan(fec_sdswdf* w, const uint8_t* h_erasure, int64_t P, int32_t* h_plan,
                          uint8_t* h_records, int64_t records_cap, int64_t* n_records, int* record_bytes) {
    if (!w || P < 0 || (P > 0 && !h_erasure)) return FEC_ERR_ARG;
    return guarded_sd([&] {
        plan_relay(w, h_erasure, P);
        const auto& d = w->relay->records().data();
        if (n_records) *n_records = w->relay->records().count();
        if (record_bytes) *record_bytes = w->relay->record_bytes();
        if (h_plan) std::memcpy(h_plan, w->plan.data(), static_cast<size_t>(P) * sizeof(int32_t));
        if (h_records) {
            if (records_cap < static_cast<int64_t>(d.size())) return static_cast<int>(FEC_ERR_WORKSPACE);
            std::memcpy(h_records, d.data(), d.size());
        }
        return static_cast<int>(FEC_OK);
    });
}

int fec_sdswdf_dest_plan(fec_sdswdf* w, const uint8_t* h_erasure, const uint8_t* h_headers, int64_t P,
                         int32_t* h_plan, uint8_t* h_flag, uint8_t* h_records, int64_t records_cap,
                         int64_t* n_records, int* record_bytes) {
    if (!w || P < 0 || (P > 0 && (!h_erasure || !h_headers))) return FEC_ERR_ARG;
    return guarded_sd([&] {
        plan_dest(w, h_erasure, h_headers, P, h_flag);
        const auto& d = w->dest->records().data();
        if (n_records) *n_records = w->dest->records().count();
        if (record_bytes) *record_bytes = w->dest->record_bytes();
        if (h_plan) std::memcpy(h_plan, w->plan.data(), static_cast<size_t>(P) * sizeof(int32_t));
        if (h_records) {
            if (records_cap < static_cast<int64_t>(d.size())) return static_cast<int>(FEC_ERR_WORKSPACE);
            std::memcpy(h_records, d.data(), d.size());
        }
        return static_cast<int>(FEC_OK);
    });
}

int fec_sdswdf_relay_batch(fec_sdswdf* w, const uint8_t* d_cw, int64_t cw_stride, const uint8_t* h_erasure,
                           int64_t P, uint8_t* d_frames, void* stream) {
    return fec_sdswdf_relay_batch_starts(w, d_cw, cw_stride, h_erasure, P, nullptr, 0, d_frames, stream);
}

int fec_sdswdf_relay_batch_starts(fec_sdswdf* w, const uint8_t* d_cw, int64_t cw_stride, const uint8_t* h_erasure,
                                  int64_t P, const int64_t* h_starts, int nstarts, uint8_t* d_frames, void* stream) {
    if (!w || P < 0 || nstarts < 0 || (nstarts > 0 && !h_starts)) return FEC_ERR_ARG;
    if (P == 0) return FEC_OK;
    if (!d_cw || !h_erasure || !d_frames || cw_stride < static_cast<int64_t>(w->g1.S) * w->g1.n) return FEC_ERR_ARG;
    for (int i = 1; i < nstarts; ++i)
        if (h_starts[i] < h_starts[i - 1]) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    return guarded_sd([&] {
        if (int st = ensure_device(w)) return st;
        plan_relay(w, h_erasure, P, h_starts, nstarts);
        if (int st = upload_plan(w, w->relay->records(), P, s)) return st;
        const int tl = launch_tile(w, true, w->relay->records(), d_cw, cw_stride, P, d_frames, s);
        if (tl < 0) return tl;
        if (tl == 0) {
            FEC_HIP(hipStreamSynchronize(s));
            return static_cast<int>(FEC_OK);
        }
        fec::SdRelayArgs a;
        a.cw = d_cw;
        a.cw_stride = cw_stride;
        a.plan = static_cast<const int32_t*>(w->d_plan.p);
        a.table = static_cast<const uint8_t*>(w->d_table.p);
        a.R = w->relay->record_bytes();
        a.P = P;
        a.k = w->v1.k;
        a.n = w->v1.n;
        a.n2 = w->v2.n;
        a.S = w->v1.S;
        a.blocks = w->blocks;
        a.gf = w->v1.gf;
        a.frames = d_frames;
        a.F = w->F;
        hipLaunchKernelGGL(fec::fec_sdswdf_relay_kernel, dim3(fec::grid_for(P * a.S)), dim3(fec::kSdThreads), 0, s, a);
        FEC_HIP(hipGetLastError());
        // the host plan arrays are reused by the next call
        FEC_HIP(hipStreamSynchronize(s));
        return static_cast<int>(FEC_OK);
    });
}

int fec_sdswdf_destination_batch(fec_sdswdf* w, const uint8_t* d_frames, const uint8_t* h_erasure, int64_t P,
                                 uint8_t* d_out, uint8_t* h_flag, void* stream) {
    return fec_sdswdf_destination_batch_starts(w, d_frames, h_erasure, P, nullptr, 0, d_out, h_flag, stream);
}

int fec_sdswdf_destination_batch_starts(fec_sdswdf* w, const uint8_t* d_frames, const uint8_t* h_erasure, int64_t P,
                                        const int64_t* h_starts, int nstarts, uint8_t* d_out, uint8_t* h_flag,
                                        void* stream) {
    if (!w || P < 0 || nstarts < 0 || (nstarts > 0 && !h_starts)) return FEC_ERR_ARG;
    if (P == 0) return FEC_OK;
    if (!d_frames || !h_erasure || !d_out) return FEC_ERR_ARG;
    for (int i = 1; i < nstarts; ++i)
        if (h_starts[i] < h_starts[i - 1]) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    return guarded_sd([&] {
        if (int st = ensure_device(w)) return st;
        // the frames' 11-byte headers drive the destination's control flow (:1663-1664): fetch them
        const size_t hb = static_cast<size_t>(P) * fec::kHdr;
        w->hdrs.resize(hb);
        if (int st = w->d_hdrs.reserve(hb)) return st;
        hipLaunchKernelGGL(fec::fec_sdswdf_hdr_gather_kernel, dim3(static_cast<unsigned>((hb + 255) / 256)), dim3(256),
                           0, s, d_frames, static_cast<int64_t>(w->F), P, static_cast<uint8_t*>(w->d_hdrs.p));
        FEC_HIP(hipGetLastError());
        FEC_HIP(hipMemcpyAsync(w->hdrs.data(), w->d_hdrs.p, hb, hipMemcpyDeviceToHost, s));
        FEC_HIP(hipStreamSynchronize(s));
        plan_dest(w, h_erasure, w->hdrs.data(), P, h_flag, h_starts, nstarts);
        if (int st = upload_plan(w, w->dest->records(), P, s)) return st;
        const int tl = launch_tile(w, false, w->dest->records(), d_frames, w->F, P, d_out, s);
        if (tl < 0) return tl;
        if (tl == 0) {
            FEC_HIP(hipStreamSynchronize(s));
            return static_cast<int>(FEC_OK);
        }
        fec::SdDestArgs a;
        a.frames = d_frames;
        a.F = w->F;
        a.plan = static_cast<const int32_t*>(w->d_plan.p);
        a.table = static_cast<const uint8_t*>(w->d_table.p);
        a.P = P;
        a.k = w->v2.k;
        a.n = w->v2.n;
        a.S = w->v2.S;
        a.blocks = w->blocks;
        a.gf = w->v2.gf;
        a.out = d_out;
        hipLaunchKernelGGL(fec::fec_sdswdf_dest_kernel, dim3(fec::grid_for(P * a.S)), dim3(fec::kSdThreads), 0, s, a);
        FEC_HIP(hipGetLastError());
        FEC_HIP(hipStreamSynchronize(s));
        return static_cast<int>(FEC_OK);
    });
}

}  // extern "C"
