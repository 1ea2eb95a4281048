// fec_host.cpp -- see fec_host.h.
#include "fec_host.h"

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>

namespace fec {

const Field& field() {
    static const Field f;
    return f;
}

// gen_G_cauchy (src/codingOperations.cpp:48-95).  The ISA-L matrices it starts from
// (gf_gen_cauchy1_matrix / gf_gen_rs_matrix, n x k, identity on top) are written directly in
// transposed form: parity column j >= k of G holds row j of the ISA-L matrix.
std::vector<uint8_t> make_generator(int T, int B, int N) {
    const Field& F = field();
    const int k = T - N + 1, n = k + B;
    std::vector<uint8_t> G(static_cast<size_t>(k) * n, 0);
    auto at = [&](int i, int j) -> uint8_t& { return G[static_cast<size_t>(i) * n + j]; };
    for (int i = 0; i < k; ++i) at(i, i) = 1;
    const bool rs = (T == 10 && B == 8 && N == 4) || (T == 11 && B == 5 && N == 4);
    uint8_t gen = 1;  // RS: row j uses powers of 2^(j-k)
    for (int j = k; j < n; ++j) {
        uint8_t p = 1;
        for (int i = 0; i < k; ++i) {
            if (rs) {
                at(i, j) = p;
                p = F.mul(p, gen);
            } else {
                at(i, j) = F.inv(static_cast<uint8_t>(j ^ i));
            }
        }
        gen = F.mul(gen, 2);
    }
    if (B == 0) return G;
    const int d = B - N;  // width of the burst-only parity block
    if (2 * k >= n) {      // high-rate regime
        for (int i = 0; i < d; ++i) {
            for (int j = k + N + i; j < n; ++j) at(i, j) = 0;
            for (int j = k; j < k + i; ++j) at(i, j) = 0;
        }
        for (int i = d; i < B; ++i)
            for (int j = k; j < k + d; ++j) at(i, j) = 0;
    } else {  // low-rate regime
        for (int i = 0; i < d; ++i) {
            for (int j = k + N + i; j < n; ++j) at(i, j) = 0;
            for (int j = B; j < B + i; ++j) at(i, j) = 0;
        }
        for (int i = d; i < k; ++i)
            for (int j = B; j < B + d; ++j) at(i, j) = 0;
    }
    return G;
}

std::vector<uint32_t> parity_mul_tables(const std::vector<uint8_t>& G, int k, int n) {
    const Field& F = field();
    const int np = n - k;
    std::vector<uint32_t> tab(static_cast<size_t>(std::max(1, k * np)) * 8, 0);
    for (int i = 0; i < k; ++i)
        for (int jj = 0; jj < np; ++jj) {
            const uint8_t c = G[static_cast<size_t>(i) * n + k + jj];
            uint32_t* t = &tab[static_cast<size_t>(i * np + jj) * 8];
            auto pack = [&](int shift, int base) {
                uint32_t v = 0;
                for (int e = 0; e < 4; ++e) v |= uint32_t(F.mul(c, uint8_t((base + e) << shift))) << (8 * e);
                return v;
            };
            t[0] = pack(0, 0);
            t[1] = pack(0, 4);
            t[2] = pack(3, 0);
            t[3] = pack(3, 4);
            t[4] = pack(6, 0);
            t[5] = c ? 1u : 0u;
        }
    return tab;
}

// One column of the k x w decoding matrix together with its column of the action matrix.
struct Column {
    uint8_t v[kMaxK];
    uint8_t a[kMaxN];
};

// Column reduction with a sliding pivot row, exactly the semantics of gf256_rref_matrix
// (src/basicOperations.cpp:43-122): for column position i the pivot sits in row i+offset; a zero
// pivot is replaced by the first later column with a non-zero entry in that row (swap), and a row
// without any such column bumps the offset.  The pivot column is normalised and eliminated from
// every other column whose entry in the pivot row is non-zero.  Columns carry their action
// column along, so decoded = codeword * action.
static void column_reduce(const Field& F, int m, int w, Column* c) {
    int row = 0;
    for (int i = 0; i < w && row < m;) {
        if (c[i].v[row] == 0) {
            int j = i + 1;
            while (j < w && c[j].v[row] == 0) ++j;
            if (j == w) {  // no pivot available in this row
                ++row;
                continue;
            }
            std::swap(c[i], c[j]);
        }
        const uint8_t s = F.inv(c[i].v[row]);
        for (int r = 0; r < m; ++r) c[i].v[r] = F.mul(c[i].v[r], s);
        for (int r = 0; r < w; ++r) c[i].a[r] = F.mul(c[i].a[r], s);
        for (int j = 0; j < w; ++j) {
            if (j == i) continue;
            const uint8_t f = c[j].v[row];
            if (!f) continue;
            for (int r = 0; r < m; ++r) c[j].v[r] ^= F.mul(f, c[i].v[r]);
            for (int r = 0; r < w; ++r) c[j].a[r] ^= F.mul(f, c[i].a[r]);
        }
        ++i;
        ++row;
    }
}

void decode_rule(const uint8_t* G, int k, int n, int w, uint32_t mask, uint8_t* sel,
                 uint8_t* col) {
    const Field& F = field();
    Column c[kMaxN];
    for (int j = 0; j < w; ++j) {
        const bool erased = (mask >> j) & 1u;
        for (int r = 0; r < k; ++r) c[j].v[r] = erased ? 0 : G[r * n + j];
        std::memset(c[j].a, 0, sizeof(c[j].a));
        c[j].a[j] = 1;
    }
    column_reduce(F, k, w, c);
    // A data symbol i is declared recovered when the first unit entry of row i among columns
    // i..k-1 sits in a column that is zero below row i (codingOperations.cpp:204-230).
    for (int i = 0; i < k; ++i) {
        sel[i] = 0xFF;
        std::memset(col + i * w, 0, w);
        int j = i;
        while (j < k && c[j].v[i] != 1) ++j;
        if (j == k) continue;
        bool unit = true;
        for (int r = i + 1; r < k; ++r) unit = unit && c[j].v[r] == 0;
        if (!unit) continue;
        sel[i] = static_cast<uint8_t>(j);
        for (int r = 0; r < w; ++r) col[i * w + r] = c[j].a[r];
    }
}

void DecodeRules::build(const std::vector<uint8_t>& G, int k_, int n_, int T_) {
    k = k_;
    n = n_;
    T = T_;
    w_lo = std::min(T + 1, n);
    entry_bytes = (k * (1 + n) + 3) & ~3;  // padded: the GPU loads an entry as dwords
    w_base.assign(n + 1, -1);
    this->G = G;
    if (n > kMaxRuleN) {  // 2^n masks: no table, rules on demand (host) / in the wave (device)
        lazy = true;
        return;
    }
    int64_t total = 0;
    for (int w = w_lo; w <= n; ++w) {
        w_base[w] = total;
        total += (int64_t(1) << w) * entry_bytes;
    }
    table.assign(static_cast<size_t>(total), 0);
    struct Job { int w; uint32_t lo, hi; };
    std::vector<Job> jobs;
    for (int w = w_lo; w <= n; ++w) {
        const uint32_t count = 1u << w, chunk = 512;
        for (uint32_t m = 0; m < count; m += chunk) jobs.push_back({w, m, std::min(count, m + chunk)});
    }
    const unsigned nth = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    std::atomic<size_t> next{0};
    auto worker = [&]() {
        uint8_t col[kMaxK * kMaxN];
        for (size_t q; (q = next.fetch_add(1)) < jobs.size();) {
            const Job& jb = jobs[q];
            for (uint32_t m = jb.lo; m < jb.hi; ++m) {
                uint8_t* e = table.data() + w_base[jb.w] + int64_t(m) * entry_bytes;
                decode_rule(G.data(), k, n, jb.w, m, e, col);
                for (int i = 0; i < k; ++i) std::memcpy(e + k + i * n, col + i * jb.w, jb.w);
            }
        }
    };
    if (jobs.size() < 8) {
        worker();
    } else {
        for (unsigned i = 0; i < nth; ++i) pool.emplace_back(worker);
        for (auto& th : pool) th.join();
    }
}

const uint8_t* DecodeRules::lazy_entry(int w, uint32_t mask) const {
    const uint64_t key = (uint64_t(w) << 32) | mask;
    std::lock_guard<std::mutex> lock(mu_);
    auto it = cache_.find(key);
    if (it != cache_.end()) return it->second.get();
    std::unique_ptr<uint8_t[]> e(new uint8_t[entry_bytes]());
    uint8_t col[kMaxK * kMaxN];
    decode_rule(G.data(), k, n, w, mask, e.get(), col);
    for (int i = 0; i < k; ++i) std::memcpy(e.get() + k + i * n, col + i * w, w);
    const uint8_t* p = e.get();
    cache_.emplace(key, std::move(e));
    return p;
}

// One table per (T,B,N) for the life of the process (codecs, planners and variable-rate plans of one
// configuration share it).  The global lock only guards the map: each table is built outside it,
// once, by the first caller (std::call_once; a build that throws leaves the slot for the next
// caller), so a configuration being built does not hold up callers of the others.
std::shared_ptr<const DecodeRules> shared_decode_rules(int T, int B, int N) {
    struct Slot {
        std::once_flag once;
        DecodeRules rules;
    };
    static std::mutex mu;
    static std::map<int64_t, std::shared_ptr<Slot>> cache;
    const int64_t key = (int64_t(T) << 32) | (int64_t(B) << 16) | int64_t(N);
    std::shared_ptr<Slot> slot;
    {
        std::lock_guard<std::mutex> lock(mu);
        std::shared_ptr<Slot>& e = cache[key];
        if (!e) e = std::make_shared<Slot>();
        slot = e;
    }
    const int k = T - N + 1, n = k + B;
    std::call_once(slot->once, [&] {
        slot->rules.build(make_generator(T, B, N), k, n, T);
        slot->rules.build_resync();
    });
    return std::shared_ptr<const DecodeRules>(slot, &slot->rules);
}

// ------------------------------------------------------------------------------------------
// StreamPlanner
// ------------------------------------------------------------------------------------------
StreamPlanner::StreamPlanner(const Geometry& g, const DecodeRules* rules)
    : k_(g.k), n_(g.n), T_(g.T), rules_(rules),
      er_(g.n, 0u),
      cwc_(static_cast<size_t>(g.n) * g.n * g.n, 0),
      datc_(static_cast<size_t>(g.n) * g.k * g.n, 0),
      hist_(g.T + 1, 0) {
    if (g.B < g.N) throw std::invalid_argument("the streaming planner needs B >= N");
}

// decode_block(b, t) for t in [t0, t1): decode of data symbol t of block b with window
// min(t+T+1, n) (decodeBlock semantics).  The cheap part (the received symbol's own row, the
// masks) stays in the loop; the recovery runs out of line.
void StreamPlanner::decode_blocks(int b, int t0, int t1) {
    const uint32_t kmask = (1u << k_) - 1u;
    for (int t = t0; t < t1; ++t) {
        if (t < k_ && !((er_[b] >> t) & 1u)) std::memcpy(dat(b, t), cw(b, t), n_);
        const int w = std::min(t + T_ + 1, n_);
        const uint32_t full = (w >= 32) ? 0xffffffffu : ((1u << w) - 1u);
        const uint32_t m = er_[b] & full;
        if (m == full) continue;
        if (!(m & kmask)) continue;  // no erased data symbol: nothing to recover
        // (w, m) alone decides whether anything is recovered: a repeat of a fruitless call is one too
        if (w == memo_w_ && m == memo_m_) continue;
        recover(b, w, m);
    }
}

void StreamPlanner::recover(int b, int w, uint32_t m) {
    const Field& F = field();
    const uint8_t* e = rules_->entry(w, m);
    uint8_t fresh[kMaxK][kMaxN];
    uint32_t got = 0;
    for (int i = 0; i < k_; ++i) {
        if (!((m >> i) & 1u) || e[i] == 0xFF) continue;
        const uint8_t* colv = e + k_ + i * n_;
        std::memset(fresh[i], 0, n_);
        for (int c = 0; c < w; ++c) {
            const uint8_t f = colv[c];
            if (!f || ((m >> c) & 1u)) continue;
            const uint8_t* src = cw(b, c);
            const uint8_t* row = F.mt[f];
            for (int q = 0; q < n_; ++q) fresh[i][q] ^= row[src[q]];
        }
        got |= 1u << i;
    }
    if (!got) {
        memo_w_ = w;
        memo_m_ = m;
    }
    for (int i = 0; i < k_; ++i) {
        if (!((got >> i) & 1u)) continue;
        er_[b] &= ~(1u << i);
        std::memcpy(dat(b, i), fresh[i], n_);
        std::memcpy(cw(b, i), fresh[i], n_);
    }
}

// Decoder_Block_Code::decodeSymbol.
void StreamPlanner::decode_symbol(int b, int p, bool erased) {
    if (erased) {
        er_[b] |= 1u << p;
    } else {
        er_[b] &= ~(1u << p);
        uint8_t* v = cw(b, p);
        std::memset(v, 0, n_);
        v[p] = 1;
    }
    if (p < T_) return;
    decode_blocks(b, p - T_, p == n_ - 1 ? std::max(k_, p - T_ + 1) : p - T_ + 1);
}

// Decoder_Basic::decodeStream input half: symbol p of a packet fed at `time` goes to block
// (time - p) mod n.
void StreamPlanner::feed(int64_t time, bool erased) {
    const int r = static_cast<int>(((time % n_) + n_) % n_);
    for (int p = 0; p < n_; ++p) decode_symbol((r - p + n_) % n_, p, erased);
}

void StreamPlanner::save_state(uint8_t* dst) const {
    std::memcpy(dst, er_.data(), er_.size() * 4);
    std::memcpy(dst + er_.size() * 4, cwc_.data(), cwc_.size());
    std::memcpy(dst + er_.size() * 4 + cwc_.size(), datc_.data(), datc_.size());
}

void StreamPlanner::load_state(const uint8_t* src) {
    std::memcpy(er_.data(), src, er_.size() * 4);
    std::memcpy(cwc_.data(), src + er_.size() * 4, cwc_.size());
    std::memcpy(datc_.data(), src + er_.size() * 4 + cwc_.size(), datc_.size());
}

void DecodeRules::build_resync() {
    Geometry g;
    g.k = k;
    g.n = n;
    g.T = T;
    g.B = n - k;
    g.N = T - k + 1;
    if (g.B < g.N) return;  // no streaming planner for this configuration
    StreamPlanner pl(g, this);
    const size_t sb = pl.state_bytes();
    std::vector<uint8_t> img(static_cast<size_t>(n) * sb);
    const int64_t base = static_cast<int64_t>(n) * (T + 1);  // >= T and a multiple of n
    for (int phi = 0; phi < n; ++phi) {
        pl.resync_at(base + phi);
        pl.save_state(img.data() + static_cast<size_t>(phi) * sb);
    }
    resync_full_bytes = sb;
    resync_full.swap(img);
}

void StreamPlanner::resync_at(int64_t t) {
    if (t >= T_ && rules_ && !rules_->resync_full.empty()) {  // the per-phase image (DecodeRules::build_resync)
        load_state(rules_->resync_full.data() + static_cast<size_t>(t % n_) * rules_->resync_full_bytes);
        return;
    }
    for (int i = 0; i < n_ - T_; ++i) feed(t + i, true);
    for (int i = 0; i < T_; ++i)
        if (t - T_ + i >= 0) feed(t - T_ + i, false);
}

void StreamPlanner::block_state(int b, uint32_t* er, uint8_t* cwc, uint8_t* datc) const {
    *er = er_[b];
    std::memcpy(cwc, &cwc_[static_cast<size_t>(b) * n_ * n_], static_cast<size_t>(n_) * n_);
    std::memcpy(datc, &datc_[static_cast<size_t>(b) * k_ * n_], static_cast<size_t>(k_) * n_);
}

int resync_state_bytes(const Geometry& g) { return (4 + g.n * g.n + g.k * g.n + 3) & ~3; }

std::vector<uint8_t> build_resync_states(const Geometry& g, const DecodeRules& rules) {
    const int sb = resync_state_bytes(g);
    std::vector<uint8_t> out(static_cast<size_t>(g.n) * sb, 0);
    StreamPlanner pl(g, &rules);
    const int64_t tr = static_cast<int64_t>(g.n) * (g.T + 1);  // >= T and a multiple of n
    pl.resync_at(tr);
    for (int phi = 0; phi < g.n; ++phi) {
        const int b = static_cast<int>(((tr - phi) % g.n + g.n) % g.n);
        uint8_t* d = out.data() + static_cast<size_t>(phi) * sb;
        uint32_t er;
        pl.block_state(b, &er, d + 4, d + 4 + g.n * g.n);
        std::memcpy(d, &er, 4);
    }
    return out;
}

StepResult StreamPlanner::step(int64_t t, bool erased) {
    StepResult out;
    out.x = t - T_;
    hist_[t % (T_ + 1)] = erased ? 1 : 0;
    if (!erased) {
        if (t - latest_ > T_) latest_ = -1;
        if (latest_ == -1) {  // fast path: the stored codeword t-T is output as is
            out.fate = out.x >= 0 ? kCopy : kNone;
            out.slow = false;
            return out;
        }
    } else {
        if (latest_ == -1) resync_at(t);  // Decoder.cpp:111-133
        latest_ = t;
    }
    feed(t, erased);
    out.slow = true;
    if (out.x < 0) {
        out.fate = kNone;
        return out;
    }
    const bool x_erased = hist_[out.x % (T_ + 1)] != 0;
    if (!x_erased) {
        out.fate = kCopy;
        return out;
    }
    for (int i = 0; i < k_; ++i) {
        const int b = static_cast<int>(((out.x - i) % n_ + n_) % n_);
        if ((er_[b] >> i) & 1u) {
            out.fate = kLost;
            return out;
        }
        std::memcpy(out.coef + i * n_, dat(b, i), n_);
    }
    out.fate = kRecovered;
    return out;
}

}  // namespace fec
