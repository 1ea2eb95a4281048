// fec_vr.cpp -- variable-rate (adaptive) coding, BASELINE config 4: the symbolic P2P loop
// (VrPlan, see fec_vr.h) and the batched device execution of its schedule.
#include "fec_vr.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstring>
#include <new>
#include <stdexcept>
#include <thread>

#include "fec_amd.h"

namespace fec {

// ---- Parameter_Estimator::estimate (Parameter_Estimator.cpp:58-190) -------------------------
void ParameterEstimator::estimate(int64_t seq, int msg_T) {
    if (T == 0) return;
    if (previous_win_end == -2) {  // first packet seen: reset the window (:66-73)
        T = msg_T;
        previous_win_end = seq - 1;
    }
    const int64_t current_win_end = seq;
    if (current_win_end - previous_win_end < 1) return;  // out of order (:84-86)
    const uint32_t wmask = (T + 1 >= 32) ? 0xffffffffu : ((1u << (T + 1)) - 1u);
    for (int64_t s = previous_win_end + 1; s <= current_win_end; ++s) {
        // shift the window by one (erasure[i] = erasure[i-1]) and insert the new flag at 0
        erasure = ((erasure << 1) | (s < current_win_end ? 1u : 0u)) & wmask;  // in between: lost
        const int sum = __builtin_popcount(erasure);
        if (sum == T + 1 || sum == 0) continue;  // (:104-105)
        if (B == 0) B = 1;
        if (N == 0) N = 1;
        if (sum > N_max) N_max = sum;
        const int first = __builtin_ctz(erasure);        // first erased index
        const int last = 31 - __builtin_clz(erasure);    // last erased index
        const int span = last - first + 1;
        if (span == T + 1) {  // (:131-136)
            if (sum > N) {
                N = sum;
                B = N;
            }
        } else {  // (:137-166)
            const int max_B_and_sum = sum > B ? sum : B;
            const int max_B_and_span = span > B ? span : B;
            if ((T - N + 1) * (T - sum + 1 + max_B_and_sum) >= (T - sum + 1) * (T - N + 1 + max_B_and_span)) {
                if (span > B) {
                    B = span;
                    N = span;
                }
            } else {
                if (sum > N) {
                    N = sum;
                    B = sum;
                }
                if (N > B) B = N;
            }
        }
        if ((T - N_max + 1) * (T - N + 1 + B) > (T - N + 1) * (T + 1)) {  // (:169-173)
            B = N_max;
            N = N_max;
        }
    }
    previous_win_end = current_win_end;
    if ((T - N_current + 1) * (T - N + 1 + B) >= (T - N + 1) * (T - N_current + 1 + B_current)) {  // (:177-181)
        B_current = B;
        N_current = N;
    }
    if (adaptive_mode_MDS) make_MDS_estimates();
}

// Parameter_Estimator::make_MDS_estimates (:209-221)
void ParameterEstimator::make_MDS_estimates() {
    if (B_current > N_current) {
        while ((T - N_current) * (T - N_current + 1 + B_current) > (T + 1) * (T - N_current + 1)) ++N_current;
        B_current = N_current;
    }
}

const DecodeRules& VrPlan::rules_for(int T, int B, int N) {
    const int key = T * 1024 + B * 32 + N;
    auto it = rules_.find(key);
    if (it != rules_.end()) return *it->second;
    return *rules_.emplace(key, shared_decode_rules(T, B, N)).first->second;
}

namespace {

constexpr int kTTot = 10;                 // T_TOT (FEC_Macro.h:32)
constexpr int kEstimationCycle = 1000 / 10;  // ESTIMATION_WINDOW_SIZE / ..._REDUCTION_FACTOR (:54-55)

struct Report {        // decoder instance `id` reports packet x at its call for seq
    int64_t seq, x;
};

}  // namespace

// Two phases.  (1) The control loop -- sender, estimators, encoder switches, the receiver's
// decoder swaps -- never looks at a decoder's output (FEC_Decoder::onReceive results only feed
// onDecodedMessage), so it runs first and records, per decoder instance, its calls (consecutive
// seqs from `first`, erased = the packet was dropped) and which of them report which packet.
// (2) The symbolic decoders are independent of each other: they replay their calls in parallel
// (one StreamPlanner per instance) and fill in the reported fates and coefficient rows.
void VrPlan::run(int max_payload, int T, int B, int N, bool mds, const uint8_t* pattern, int64_t n_pattern,
                 int64_t P_value) {
    L = max_payload;
    T_init = T;
    B_init = B;
    N_init = N;
    adaptive_mode_MDS = mds;
    P = P_value;
    frames.clear();
    enc.clear();
    dec.clear();
    erased.clear();
    fate.assign(static_cast<size_t>(P), kNone);
    fate_dec.assign(static_cast<size_t>(P), -1);
    slow.assign(static_cast<size_t>(P), 0);
    rec_x.clear();
    rec_dec.clear();
    rec_coef.clear();
    lost = switches = 0;
    steady_packets = 0;
    sum_coding_rate = 0;

    // ---- sender (Application_Layer_Sender.cpp:9-31, 64-93, 221-224) ----
    const bool adaptive = B == -1 || N == -1;
    int sT = T, sB = adaptive ? 0 : B, sN = adaptive ? 0 : N;
    int sT_ack = sT, sB_ack = sB, sN_ack = sN;
    // ---- Variable_Rate_FEC_Encoder (Variable_Rate_FEC_Encoder.cpp:25-58, 74-235) ----
    int eT = 0, eB = 0, eN = 0, eN_old = 0;
    int cur = -1, old = -1;
    int counter_transition = 0;
    bool transition_flag = true, double_coding_flag = true;
    // ---- receiver (Application_Layer_Receiver.cpp:10-31, 321-468) ----
    std::unique_ptr<ParameterEstimator> est(new ParameterEstimator(kTTot, mds));
    std::unique_ptr<ParameterEstimator> bg(new ParameterEstimator(kTTot, mds));
    int64_t cycle = 1;
    uint8_t udp[12] = {};
    // ---- Variable_Rate_FEC_Decoder (Variable_Rate_FEC_Decoder.cpp:25-80, 2133-2400, 2440-2514) ----
    int64_t seq_start = -1, latest_seq = -1, sdc = -1, sde = -1;
    int dT = 0, dB = 0, dN = 0;
    int dcur = -1, dold = -1;
    bool dcf = false;
    std::vector<std::vector<Report>> reports;  // per decoder instance, in call order

    auto new_decoder = [&](int T_, int B_, int N_, int64_t first) {
        VrInstance v;
        v.T = T_;
        v.B = B_;
        v.N = N_;
        v.first = v.end = first;
        v.role_switch = -1;  // set when it becomes the old decoder
        dec.push_back(v);
        reports.emplace_back();
        return static_cast<int>(dec.size()) - 1;
    };
    auto call = [&](int id, int64_t seq) {
        if (seq != dec[id].end) throw std::logic_error("vr: decoder calls out of order");
        dec[id].end = seq + 1;
    };
    // onDecodedMessage (:2403-2436): packets seq - T >= seq_start are reported once
    auto report = [&](int id, int64_t seq) {
        const int64_t x = seq - dT;
        if (x < seq_start || x >= P) return;
        reports[id].push_back(Report{seq, x});
        fate_dec[x] = id;
    };
    auto update_decoder = [&](int T_, int B_, int N_, int64_t first) {  // (:2520-2536)
        dold = dcur;
        dT = T_;
        dB = B_;
        dN = N_;
        dcur = new_decoder(T_, B_, N_, first);
        dec[dold].role_switch = first;
    };

    const auto t_start = std::chrono::steady_clock::now();
    frames.reserve(static_cast<size_t>(P + T + 1));
    erased.reserve(static_cast<size_t>(P + T + 1));
    const int64_t n_drop = std::min<int64_t>(P + T, n_pattern);  // packets the pattern can drop
    int64_t next_drop = -1;                                        // cache of the next dropped seq
    for (int64_t seq = 0;; ++seq) {
        // ---- steady stretch: the same frame, every packet received, nothing switching ----
        // Every branch below is then fixed: the feedback repeats (both estimators at their fixed
        // point, no estimator swap before the next cycle boundary), the encoder has no switch to
        // make and no transition running, the decoder has no gap, no parameter change and no
        // double decoding.  Such packets are appended directly, in the same order and with the
        // same float accumulation of the coding rate as the loop below; the stretch ends before
        // the next drop, the next cycle boundary and the last packet.
        if (cur >= 0 && !transition_flag && !double_coding_flag && counter_transition > eT && seq_start >= 0 &&
            latest_seq == seq && !dcf && sdc < seq && dT == eT && dB == eB && dN == eN && seq < P + T - 1) {
            const int fT = adaptive && udp[0] != 0 ? udp[0] : sT, fB = adaptive && udp[0] != 0 ? udp[1] : sB,
                      fN = adaptive && udp[0] != 0 ? udp[2] : sN;
            const int aT = adaptive && udp[0] != 0 ? udp[3] : sT_ack, aB = adaptive && udp[0] != 0 ? udp[4] : sB_ack;
            const bool would_switch = (fT != eT || fB != eB || fN != eN) && aT == eT && aB == eB;
            if (!would_switch && est->steady(seq, eT) && bg->steady(seq, eT) && udp[3] == eT && udp[4] == eB &&
                udp[5] == eN && udp[0] == est->T && udp[1] == est->B_current && udp[2] == est->N_current) {
                if (next_drop < seq) {
                    next_drop = n_drop;
                    if (seq < n_drop) {
                        const void* hit = std::memchr(pattern + seq, 1, static_cast<size_t>(n_drop - seq));
                        if (hit) next_drop = static_cast<const uint8_t*>(hit) - pattern;
                    }
                }
                const int64_t end = std::min({next_drop, cycle * kEstimationCycle, P + T - 1});
                if (end > seq) {
                    if (adaptive && udp[0] != 0) {
                        sT = udp[0];
                        sB = udp[1];
                        sN = udp[2];
                        sT_ack = udp[3];
                        sB_ack = udp[4];
                        sN_ack = udp[5];
                    }
                    VrFrame fr;
                    fr.T = eT;
                    fr.B = eB;
                    fr.N = eN;
                    fr.enc_cur = cur;
                    fr.counter = counter_transition;
                    const float rate = static_cast<float>(eT - eN + 1) / (eT - eN + 1 + eB);
                    frames.insert(frames.end(), static_cast<size_t>(end - seq), fr);
                    erased.insert(erased.end(), static_cast<size_t>(end - seq), uint8_t(0));
                    std::vector<Report>& rp = reports[dcur];
                    for (int64_t s = seq; s < end; ++s) {
                        sum_coding_rate += rate;
                        const int64_t x = s - dT;  // report(dcur, s)
                        if (x >= seq_start && x < P) {
                            rp.push_back(Report{s, x});
                            fate_dec[x] = dcur;
                        }
                    }
                    enc[cur].end = end;
                    dec[dcur].end = end;  // call(dcur, s) for every s
                    est->previous_win_end = end - 1;
                    bg->previous_win_end = end - 1;
                    latest_seq = end;
                    sent = end;
                    steady_packets += end - seq;
                    seq = end;
                }
            }
        }
        // ---- Application_Layer_Sender::generate_message_and_encode ----
        if (adaptive && udp[0] != 0) {
            sT = udp[0];
            sB = udp[1];
            sN = udp[2];
            sT_ack = udp[3];
            sB_ack = udp[4];
            sN_ack = udp[5];
        }
        (void)sN_ack;
        int mT = sT, mB = sB, mN = sN;
        // ---- Variable_Rate_FEC_Encoder::encode ----
        if (cur < 0) {
            eT = mT;
            eB = mB;
            eN = mN;
            enc.push_back(VrInstance{eT, eB, eN, seq, seq, -1});
            cur = 0;
            transition_flag = true;
            double_coding_flag = false;
        } else if ((mT != eT || mB != eB || mN != eN) && !transition_flag && sT_ack == eT && sB_ack == eB) {
            ++switches;  // "Start double coding at the source"
            eN_old = eN;
            eT = mT;
            eB = mB;
            eN = mN;
            transition_flag = true;
            double_coding_flag = true;
            counter_transition = 0;
            old = cur;
            enc[old].role_switch = seq;
            enc.push_back(VrInstance{eT, eB, eN, seq, seq, -1});
            cur = static_cast<int>(enc.size()) - 1;
        } else {
            mT = eT;
            mB = eB;
            mN = eN;
        }
        VrFrame fr;
        fr.T = mT;
        fr.B = mB;
        fr.N = mN;
        fr.enc_cur = cur;
        enc[cur].end = seq + 1;
        fr.counter = counter_transition;
        if (counter_transition <= eT) {
            if (counter_transition == eT) double_coding_flag = false;
            ++counter_transition;
            if (old >= 0 && double_coding_flag) {
                fr.enc_old = old;
                enc[old].end = seq + 1;
            }
        } else {
            transition_flag = false;
        }
        if (!double_coding_flag)
            sum_coding_rate += static_cast<float>(eT - eN + 1) / (eT - eN + 1 + eB);
        else
            sum_coding_rate += static_cast<float>(eT - eN + 1) / ((eT - eN + 1 + eB) + (eT - eN_old + 1) + (eT - eN_old + 1 + eB));
        frames.push_back(fr);
        const bool drop = seq < P + T && seq < n_pattern && pattern[seq] == 1;
        erased.push_back(drop ? 1 : 0);
        sent = seq + 1;

        // ---- Application_Layer_Receiver::receive_message_and_decode ----
        if (drop) continue;  // artificial erasure: returns -1, feedback unchanged
        est->estimate(seq, fr.T);
        bg->estimate(seq, fr.T);
        if (seq + 1 > cycle * kEstimationCycle) {
            est = std::move(bg);
            bg.reset(new ParameterEstimator(kTTot, false));
            ++cycle;
        }
        // ---- Variable_Rate_FEC_Decoder::decode ----
        if (seq_start == -1) {  // initialize_decoder (:2478-2494)
            seq_start = 0;
            latest_seq = 0;
            dT = fr.T;
            dB = fr.B;
            dN = fr.N;
            dcur = new_decoder(dT, dB, dN, 0);
        }
        if (seq >= latest_seq) {
            if (dT != fr.T || dB != fr.B || dN != fr.N) sdc = seq - fr.counter;
            for (int64_t s = latest_seq; s < seq; ++s) {  // the missing packets (:2200-2330)
                if (s > sde && dcf) dcf = false;
                if (s == sdc) {
                    update_decoder(fr.T, fr.B, fr.N, s);
                    sde = sdc + dT - 1;
                    dcf = true;
                }
                if (!dcf) {
                    call(dcur, s);
                    report(dcur, s);
                } else {
                    if (dold >= 0) {
                        call(dold, s);
                        report(dold, s);
                    }
                    call(dcur, s);
                }
            }
            if (seq > sde && dcf) dcf = false;
            if (seq == sdc) {
                update_decoder(fr.T, fr.B, fr.N, seq);
                sde = sdc + dT - 1;
                dcf = true;
            }
            if (!dcf) {
                call(dcur, seq);
                report(dcur, seq);
            } else {
                if (dold >= 0) {
                    call(dold, seq);
                    report(dold, seq);
                }
                call(dcur, seq);
            }
            latest_seq = seq + 1;
        }
        udp[0] = static_cast<uint8_t>(est->T);
        udp[1] = static_cast<uint8_t>(est->B_current);
        udp[2] = static_cast<uint8_t>(est->N_current);
        udp[3] = static_cast<uint8_t>(fr.T);
        udp[4] = static_cast<uint8_t>(fr.B);
        udp[5] = static_cast<uint8_t>(fr.N);
        if (seq >= P + T - 1) break;  // application_local_simulation.cpp:813
    }
    for (auto* list : {&enc, &dec})
        for (auto& e : *list)
            if (e.role_switch < 0) e.role_switch = e.end;  // never became the old instance

    const auto t_control = std::chrono::steady_clock::now();
    // ---- phase 2: the decoder instances, symbolically and in parallel ----
    for (const auto& d : dec) rules_for(d.T, d.B, d.N);  // built before the workers share the map
    struct Rec {
        int64_t x;
        uint8_t coef[kMaxK * kMaxRuleN];
    };
    std::vector<std::vector<Rec>> recs(dec.size());
    std::atomic<size_t> next{0};
    auto worker = [&]() {
        for (size_t id; (id = next.fetch_add(1)) < dec.size();) {
            const VrInstance& d = dec[id];
            const Geometry g = Geometry::make(L, d.T, d.B, d.N);
            StreamPlanner pl(g, rules_.at(d.T * 1024 + d.B * 32 + d.N).get());
            const std::vector<Report>& rp = reports[id];
            size_t ri = 0;
            for (int64_t s = d.first; s < d.end; ++s) {
                const StepResult r = pl.step(s - d.first, erased[static_cast<size_t>(s)] != 0);
                if (ri == rp.size() || rp[ri].seq != s) continue;
                const int64_t x = rp[ri++].x;
                const PacketFate f = r.fate == kNone ? kLost : r.fate;
                fate[x] = f;
                slow[x] = r.slow ? 1 : 0;
                if (f == kRecovered) {
                    Rec rc;
                    rc.x = x;
                    std::memset(rc.coef, 0, sizeof(rc.coef));
                    std::memcpy(rc.coef, r.coef, static_cast<size_t>(g.k) * g.n);
                    recs[id].push_back(rc);
                }
            }
        }
    };
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t nth = std::min<size_t>({dec.size(), hw ? hw : 1u, 16u});
    if (nth <= 1) {
        worker();
    } else {
        std::vector<std::thread> pool;
        for (size_t i = 0; i < nth; ++i) pool.emplace_back(worker);
        for (auto& th : pool) th.join();
    }
    const auto t_decoders = std::chrono::steady_clock::now();
    control_ms = std::chrono::duration<double, std::milli>(t_control - t_start).count();
    decoders_ms = std::chrono::duration<double, std::milli>(t_decoders - t_control).count();
    for (int64_t x = 0; x < P; ++x)
        if (fate[x] == kLost) ++lost;
    std::vector<std::pair<int64_t, const Rec*>> order;
    for (size_t id = 0; id < recs.size(); ++id)
        for (const Rec& rc : recs[id]) order.emplace_back(rc.x, &rc);
    std::sort(order.begin(), order.end(),
              [](const std::pair<int64_t, const Rec*>& a, const std::pair<int64_t, const Rec*>& b) {
                  return a.first < b.first;
              });
    rec_coef.resize(order.size() * kVrCoefStride);
    for (size_t i = 0; i < order.size(); ++i) {
        rec_x.push_back(order[i].first);
        rec_dec.push_back(fate_dec[order[i].first]);
        std::memcpy(&rec_coef[i * kVrCoefStride], order[i].second->coef, kVrCoefStride);
    }
}

}  // namespace fec

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
struct fec_vr_plan {
    fec::VrPlan plan;
    int cw_max = 0;
    // ---- device tables (uploaded on first use, one allocation each for encode / decode) ----
    void* d_enc_arena = nullptr;
    void* d_dec_arena = nullptr;
    const int32_t* d_enc_inst = nullptr;   // [nenc][4]: k, n, CW, glog offset
    const int64_t* d_enc_span = nullptr;   // [nenc][2]: first, role_switch
    const int64_t* d_enc_cum = nullptr;    // [nenc+1]
    const uint32_t* d_gtab = nullptr;
    const int32_t* d_pk_dec = nullptr;
    const int32_t* d_inst = nullptr;
    const int64_t* d_inst_switch = nullptr;
    const uint8_t* d_fate = nullptr;
    const uint8_t* d_slow = nullptr;
    const int64_t* d_rec_x = nullptr;
    const int32_t* d_rec_dec = nullptr;
    const uint8_t* d_rec_coef = nullptr;
    const uint8_t* d_gf = nullptr;
    const int32_t* d_hdr = nullptr;    // [sent][4]: frame header T, B, N, counter
    void* d_hdr_arena = nullptr;
    int64_t enc_total = 0;             // codewords of all encoder instances
    int enc_tab = 0, enc_out = 0, enc_slot = 0, enc_wave = 0;  // fec_vr_encode_kernel's LDS layout
    bool enc_ready = false, dec_ready = false;

    ~fec_vr_plan() {
        for (void* p : {d_enc_arena, d_dec_arena, d_hdr_arena})
            if (p) (void)hipFree(p);
    }
};

namespace {
// Host tables packed into one buffer (256-byte aligned pieces) and uploaded with one allocation
// and one copy.
struct Arena {
    std::vector<uint8_t> host;
    std::vector<std::pair<const void**, size_t>> fix;
    template <typename T>
    void add(const T** d, const T* h, size_t count) {
        const size_t off = (host.size() + 255) & ~size_t(255);
        host.resize(off + std::max<size_t>(1, count) * sizeof(T));
        if (count) std::memcpy(host.data() + off, h, count * sizeof(T));
        fix.emplace_back(reinterpret_cast<const void**>(d), off);
    }
    template <typename T>
    void add(const T** d, const std::vector<T>& h) { add(d, h.data(), h.size()); }
    int commit(void** base) {
        if (hipMalloc(base, std::max<size_t>(16, host.size())) != hipSuccess) return FEC_ERR_NOMEM;
        if (hipMemcpy(*base, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) return FEC_ERR_HIP;
        for (auto& f : fix) *f.first = static_cast<const uint8_t*>(*base) + f.second;
        return FEC_OK;
    }
};

std::vector<uint8_t> gf_tables() {
    const fec::Field& F = fec::field();
    std::vector<uint8_t> gf(F.exp, F.exp + 512);
    gf.insert(gf.end(), F.log, F.log + 256);
    return gf;
}

// Encode tables: per encoder instance its geometry, first call, role switch and the running
// count of codewords; per (T,B,N) tuple the gf_mul4 register tables of G's parity columns.
int prepare_encode(fec_vr_plan* v) {
    if (v->enc_ready) return FEC_OK;
    const auto& p = v->plan;
    std::map<int, int> toff;  // tuple -> dword offset in gtab
    std::vector<uint32_t> gtab;
    std::vector<int32_t> inst;
    std::vector<int64_t> span, cum{0};
    int tab = 32, out = 16, slot = 16, nmax = 1;
    for (const auto& e : p.enc) {
        const fec::Geometry g = fec::Geometry::make(p.L, e.T, e.B, e.N);
        const int key = e.T * 1024 + e.B * 32 + e.N;
        auto it = toff.find(key);
        if (it == toff.end()) {
            const std::vector<uint32_t> t = fec::parity_mul_tables(fec::make_generator(e.T, e.B, e.N), g.k, g.n);
            it = toff.emplace(key, static_cast<int>(gtab.size())).first;
            gtab.insert(gtab.end(), t.begin(), t.end());
        }
        tab = std::max(tab, g.k * (g.n - g.k) * 32);
        out = std::max(out, (g.CW + 8 + 15) / 16 * 16);
        slot = std::max(slot, g.k * 4 * ((g.S + 3) / 4));
        nmax = std::max(nmax, g.n);
        inst.insert(inst.end(), {g.k, g.n, g.CW, it->second});
        span.insert(span.end(), {e.first, e.role_switch});
        cum.push_back(cum.back() + (e.end - e.first));
    }
    Arena ar;
    ar.add(&v->d_enc_inst, inst);
    ar.add(&v->d_enc_span, span);
    ar.add(&v->d_enc_cum, cum);
    ar.add(&v->d_gtab, gtab);
    if (int st = ar.commit(&v->d_enc_arena)) return st;
    v->enc_total = cum.back();
    v->enc_tab = tab;
    v->enc_out = out;
    v->enc_slot = slot;
    v->enc_wave = tab + out + nmax * slot;
    v->enc_ready = true;
    return FEC_OK;
}

int prepare_decode(fec_vr_plan* v) {
    if (v->dec_ready) return FEC_OK;
    const auto& p = v->plan;
    std::vector<int32_t> inst;
    std::vector<int64_t> sw;
    for (const auto& d : p.dec) {
        const fec::Geometry g = fec::Geometry::make(p.L, d.T, d.B, d.N);
        inst.insert(inst.end(), {g.k, g.n, g.CW, 0});
        sw.push_back(d.role_switch);
    }
    Arena ar;
    ar.add(&v->d_pk_dec, p.fate_dec);
    ar.add(&v->d_inst, inst);
    ar.add(&v->d_inst_switch, sw);
    ar.add(&v->d_fate, p.fate);
    ar.add(&v->d_slow, p.slow);
    ar.add(&v->d_rec_x, p.rec_x);
    ar.add(&v->d_rec_dec, p.rec_dec);
    ar.add(&v->d_rec_coef, p.rec_coef);
    const std::vector<uint8_t> gf = gf_tables();
    ar.add(&v->d_gf, gf);
    if (int st = ar.commit(&v->d_dec_arena)) return st;
    v->dec_ready = true;
    return FEC_OK;
}
}  // namespace

namespace {
template <typename F>
int vr_guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}
int cw_of(const fec::VrPlan& p, const fec::VrInstance& v) { return fec::Geometry::make(p.L, v.T, v.B, v.N).CW; }
}  // namespace

extern "C" {

int fec_vr_plan_create(int max_payload, int T, int B, int N, int adaptive_mode_MDS, const uint8_t* erasure,
                       int64_t n_erasure, int64_t P, fec_vr_plan** out) {
    if (!out || P < 1 || n_erasure < 0 || (n_erasure > 0 && !erasure) || T < 1 || T > 11) return FEC_ERR_ARG;
    *out = nullptr;
    return vr_guarded([&] {
        std::unique_ptr<fec_vr_plan> v(new fec_vr_plan());
        v->plan.run(max_payload, T, B, N, adaptive_mode_MDS != 0, erasure, n_erasure, P);
        for (const auto& e : v->plan.enc) v->cw_max = std::max(v->cw_max, cw_of(v->plan, e));
        for (const auto& d : v->plan.dec) v->cw_max = std::max(v->cw_max, cw_of(v->plan, d));
        *out = v.release();
        return FEC_OK;
    });
}

int fec_vr_plan_destroy(fec_vr_plan* v) {
    delete v;
    return FEC_OK;
}

int fec_vr_plan_stats(const fec_vr_plan* v, int64_t* lost, int64_t* switches, double* coding_rate,
                      int64_t* sent, int* n_encoders, int* n_decoders, int* cw_max) {
    if (!v) return FEC_ERR_ARG;
    if (lost) *lost = v->plan.lost;
    if (switches) *switches = v->plan.switches;
    if (coding_rate) *coding_rate = v->plan.coding_rate();
    if (sent) *sent = v->plan.sent;
    if (n_encoders) *n_encoders = static_cast<int>(v->plan.enc.size());
    if (n_decoders) *n_decoders = static_cast<int>(v->plan.dec.size());
    if (cw_max) *cw_max = v->cw_max;
    return FEC_OK;
}

int fec_vr_plan_timing(const fec_vr_plan* v, double* control_ms, double* decoders_ms) {
    if (!v) return FEC_ERR_ARG;
    if (control_ms) *control_ms = v->plan.control_ms;
    if (decoders_ms) *decoders_ms = v->plan.decoders_ms;
    return FEC_OK;
}

static void put_instances(const std::vector<fec::VrInstance>& in, int64_t* out) {
    for (size_t i = 0; i < in.size(); ++i) {
        int64_t* o = out + 6 * i;
        o[0] = in[i].T;
        o[1] = in[i].B;
        o[2] = in[i].N;
        o[3] = in[i].first;
        o[4] = in[i].role_switch;
        o[5] = in[i].end;
    }
}

int fec_vr_plan_instances(const fec_vr_plan* v, int64_t* encoders, int64_t* decoders) {
    if (!v) return FEC_ERR_ARG;
    if (encoders) put_instances(v->plan.enc, encoders);
    if (decoders) put_instances(v->plan.dec, decoders);
    return FEC_OK;
}

int fec_vr_plan_packets(const fec_vr_plan* v, int32_t* frames, uint8_t* erased, uint8_t* fate,
                        int32_t* fate_decoder) {
    if (!v) return FEC_ERR_ARG;
    const auto& p = v->plan;
    for (int64_t s = 0; s < p.sent; ++s) {
        if (frames) {
            int32_t* o = frames + 6 * s;
            o[0] = p.frames[s].T;
            o[1] = p.frames[s].B;
            o[2] = p.frames[s].N;
            o[3] = p.frames[s].counter;
            o[4] = p.frames[s].enc_cur;
            o[5] = p.frames[s].enc_old;
        }
        if (erased) erased[s] = p.erased[s];
    }
    if (fate) std::memcpy(fate, p.fate.data(), p.fate.size());
    if (fate_decoder) std::memcpy(fate_decoder, p.fate_dec.data(), p.fate_dec.size() * 4);
    return FEC_OK;
}

// Encode every packet the sender produced: row s of d_cw_cur (stride cw_max) = the codeword of
// frame s's current encoder, row s of d_cw_old = its old encoder's (double coding; rows of frames
// without one are left alone), trimmed sizes in d_len_*.  One launch for every instance of every
// (T,B,N) tuple (fec_vr_encode_kernel), straight from the payload rows.
int fec_vr_encode_batch(fec_vr_plan* v, const uint8_t* d_payload, const int32_t* d_payload_len, uint8_t* d_cw_cur,
                        int32_t* d_len_cur, uint8_t* d_cw_old, int32_t* d_len_old, void* hip_stream) {
    if (!v || !d_payload || !d_cw_cur || !d_len_cur || !d_cw_old || !d_len_old) return FEC_ERR_ARG;
    if (int st = vr_guarded([&] { return prepare_encode(v); })) return st;
    fec::VrEncodeArgs a{d_payload, d_payload_len, v->plan.L, v->d_enc_inst, v->d_enc_span, v->d_enc_cum,
                        static_cast<int>(v->plan.enc.size()), v->enc_total, v->enc_tab, v->enc_out, v->enc_slot,
                        v->enc_wave, v->d_gtab, v->cw_max, d_cw_cur, d_cw_old, d_len_cur, d_len_old};
    return fec::vr_launch_encode(a, hip_stream);
}

// The P2P wire packets of every frame: row s of d_packets (stride >= 10 + 2*cw_max bytes) =
// [seq BE32][T][B][N][counter_for_start_and_end] (Application_Layer_Sender.cpp:259-269) +
// [len_cur BE16][cur][old] (Variable_Rate_FEC_Encoder.cpp:194-217), sizes in d_packet_len.
int fec_vr_frames_batch(fec_vr_plan* v, const uint8_t* d_cw_cur, const int32_t* d_len_cur, const uint8_t* d_cw_old,
                        const int32_t* d_len_old, uint8_t* d_packets, int64_t stride, int32_t* d_packet_len,
                        void* hip_stream) {
    if (!v || !d_cw_cur || !d_len_cur || !d_cw_old || !d_len_old || !d_packets || !d_packet_len) return FEC_ERR_ARG;
    if (stride < 10 + 2 * static_cast<int64_t>(v->cw_max)) return FEC_ERR_ARG;
    const auto& p = v->plan;
    if (!v->d_hdr) {
        std::vector<int32_t> h(static_cast<size_t>(p.sent) * 4);
        for (int64_t s = 0; s < p.sent; ++s) {
            h[4 * s] = p.frames[s].T;
            h[4 * s + 1] = p.frames[s].B;
            h[4 * s + 2] = p.frames[s].N;
            h[4 * s + 3] = p.frames[s].counter;
        }
        Arena ar;
        ar.add(&v->d_hdr, h);
        if (int st = ar.commit(&v->d_hdr_arena)) return st;
    }
    fec::VrFrameArgs a{d_cw_cur, d_len_cur, d_cw_old, d_len_old, v->cw_max, v->d_hdr, p.sent, d_packets, stride,
                       d_packet_len};
    return fec::vr_launch_frames(a, hip_stream);
}

// Decode the schedule from the frames' arrays: every packet x < P was reported by one decoder
// instance j (fate_decoder); a received one is the systematic part of cur[x] in j's geometry, a
// recovered one the host plan's coefficient rows over j's inputs (cur rows before j became the
// old decoder, old rows after).  Two launches.  d_erased is not read (the plan holds the pattern).
int fec_vr_decode_batch(fec_vr_plan* v, const uint8_t* d_cw_cur, const uint8_t* d_cw_old, const uint8_t* d_erased,
                        uint8_t* d_out, int32_t* d_out_len, void* hip_stream) {
    (void)d_erased;
    if (!v || !d_cw_cur || !d_cw_old || !d_out || !d_out_len) return FEC_ERR_ARG;
    if (int st = vr_guarded([&] { return prepare_decode(v); })) return st;
    const auto& p = v->plan;
    fec::VrCopyArgs ca{d_cw_cur, v->cw_max, v->d_pk_dec, v->d_inst, v->d_fate, v->d_slow, p.P, p.L, d_out, d_out_len};
    if (int st = fec::vr_launch_copy(ca, hip_stream)) return st;
    fec::VrRecArgs ra{d_cw_cur, d_cw_old, v->cw_max, p.sent, v->d_rec_x, v->d_rec_dec, v->d_rec_coef,
                      static_cast<int>(p.rec_x.size()), v->d_inst, v->d_inst_switch, v->d_gf, p.L, d_out, d_out_len};
    return fec::vr_launch_recover(ra, hip_stream);
}

int fec_vr_parse_batch(const uint8_t* d_packets, int64_t stride, const int32_t* d_packet_len, int64_t rows,
                       int cw_max, uint8_t* d_cw_cur, uint8_t* d_cw_old, int32_t* d_header, void* hip_stream) {
    if (rows < 0 || cw_max < 1 || (rows > 0 && (!d_packets || !d_packet_len || !d_cw_cur || !d_cw_old)))
        return FEC_ERR_ARG;
    fec::VrParseArgs a{d_packets, stride, d_packet_len, rows, cw_max, d_cw_cur, d_cw_old, d_header};
    return fec::vr_launch_parse(a, hip_stream);
}

}  // extern "C"
