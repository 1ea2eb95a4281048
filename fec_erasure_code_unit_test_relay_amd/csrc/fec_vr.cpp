// fec_vr.cpp -- variable-rate (adaptive) coding, BASELINE config 4: the symbolic P2P loop
// (VrPlan, see fec_vr.h) and the batched device execution of its schedule.
#include "fec_vr.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <pthread.h>
#include <sched.h>
#include <sys/resource.h>
#include <new>
#include <mutex>
#include <set>
#include <stdexcept>
#include <thread>

#include "fec_amd.h"
#include "fec_kernels.h"
#include "fec_status.h"

// FEC_VR_PROFILE (diagnostic builds only): cycle counts of the control loop's parts --
// 0 steady stretch check, 1 transition stretch, 2 sender + encoder, 3 feedback, 4 decoder, 5 loop top.
#ifdef FEC_VR_PROFILE
#include <x86intrin.h>
#include <map>
#define FEC_VR_PROF_DECL uint64_t prof_c[8] = {}, prof_t = __rdtsc(); int64_t prof_cls[64] = {}; std::map<int, int64_t> prof_why_h;
#define FEC_VR_SUB(k, stmt)                            \
    {                                                  \
        const uint64_t s_ = __rdtsc();                 \
        stmt;                                          \
        prof_c[k] += __rdtsc() - s_;                   \
    }
#define FEC_VR_PROF(k)                 \
    {                                  \
        const uint64_t t_ = __rdtsc(); \
        prof_c[k] += t_ - prof_t;      \
        prof_t = t_;                   \
    }
#define FEC_VR_PROF_PRINT                                                                                  \
    std::fprintf(stderr, "vr control Mcycles: steady %.3f transition %.3f sender %.3f feedback %.3f "      \
                         "decoder %.3f top %.3f\n",                                                        \
                 prof_c[0] * 1e-6, prof_c[1] * 1e-6, prof_c[2] * 1e-6, prof_c[3] * 1e-6, prof_c[4] * 1e-6, \
                 prof_c[5] * 1e-6);                                                                    \
    std::fprintf(stderr, "vr control Mcycles inside decoder: done_with %.3f new_decoder %.3f\n", prof_c[6] * 1e-6, prof_c[7] * 1e-6); \
    for (int c_ = 0; c_ < 64; ++c_)                                                                        \
        if (prof_cls[c_]) std::fprintf(stderr, "vr iteration class %2d: %lld\n", c_, (long long)prof_cls[c_]); \
    for (auto& w_ : prof_why_h) std::fprintf(stderr, "vr class-0 why %#x: %lld\n", w_.first, (long long)w_.second);
#else
#define FEC_VR_PROF_DECL
#define FEC_VR_SUB(k, stmt) stmt;
#define FEC_VR_PROF(k)
#define FEC_VR_PROF_PRINT
#endif

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
    if (key >= 0 && static_cast<size_t>(key) < rules_fast_.size() && rules_fast_[static_cast<size_t>(key)])
        return *rules_fast_[static_cast<size_t>(key)];
    auto it = rules_.find(key);
    if (it == rules_.end()) it = rules_.emplace(key, shared_decode_rules(T, B, N)).first;
    if (key >= 0 && key < kRulesKeys) {  // a direct table beside the map (one lookup per switch)
        if (rules_fast_.empty()) rules_fast_.assign(kRulesKeys, nullptr);
        rules_fast_[static_cast<size_t>(key)] = it->second.get();
    }
    return *it->second;
}

namespace {

constexpr int kTTot = 10;                 // T_TOT (FEC_Macro.h:32)

// The plan's own threads (feedback producer, decoder workers), and the calling thread for the
// control loop, run on the 8 CPUs of the calling thread's aligned group (within the process's
// allowed set), so that what the producer writes and the control loop reads stays near: on a
// two-socket box the scheduler otherwise spreads them over both sockets (plan 2.5 - 2.7 ms
// unplaced, 1.8 - 2.1 ms with the plan's threads placed, 1.6 - 1.9 ms with the caller held too,
// profiles/r03/r03v_vr_affinity.txt).  The caller's own placement is restored when the control
// loop ends.  FEC_VR_PIN=0: nothing placed; 1: the plan's threads only; 2 (default): both.
thread_local int t_pin_home = -1;  // set by the control thread for the threads it starts
int vr_pin_mode() {
    static const int mode = [] {
        const char* v = std::getenv("FEC_VR_PIN");
        return v ? std::atoi(v) : 2;
    }();
    return mode;
}
int vr_pin_home() { return vr_pin_mode() > 0 ? sched_getcpu() : -1; }
// The allowed CPUs of home's aligned group of 8 (empty when home < 0).
cpu_set_t vr_group(int home) {
    cpu_set_t allowed, set;
    CPU_ZERO(&set);
    if (home < 0 || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return set;
    const int base = home & ~7;
    for (int c = base; c < base + 8 && c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &allowed)) CPU_SET(c, &set);
    return set;
}
void vr_pin_near(int home) {
    cpu_set_t set = vr_group(home);
    // a sparse group (fewer than 4 allowed CPUs: taskset, cgroup) is left alone: the plan's
    // spin-polling threads crowded on one or two CPUs would stall each other
    if (CPU_COUNT(&set) >= 4) (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}
// CPUs this process may run on (its affinity mask), at least 1.
int vr_allowed_cpus() {
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return static_cast<int>(std::thread::hardware_concurrency());
    return std::max(1, CPU_COUNT(&allowed));
}
constexpr int kEstimationCycle = 1000 / 10;  // ESTIMATION_WINDOW_SIZE / ..._REDUCTION_FACTOR (:54-55)

struct Report {        // decoder instance `id` reports packet x at its call for seq
    int64_t seq, x;
};

}  // namespace

// Host memory for the plan's per-packet arrays: page-locked when the HIP runtime can provide it
// (a 64-byte header records which allocator the block came from).
void* vr_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes + 64, hipHostMallocDefault) == hipSuccess && p) {
        static_cast<uint8_t*>(p)[0] = 1;
    } else {
        (void)hipGetLastError();
        p = std::malloc(bytes + 64);
        if (!p) throw std::bad_alloc();
        static_cast<uint8_t*>(p)[0] = 0;
    }
    return static_cast<uint8_t*>(p) + 64;
}

void vr_host_free(void* q) {
    if (!q) return;
    uint8_t* p = static_cast<uint8_t*>(q) - 64;
    if (p[0] == 1)
        (void)hipHostFree(p);
    else
        std::free(p);
}

VrFrame VrPlan::frame(int64_t s) const {
    auto it = std::upper_bound(frame_runs.begin(), frame_runs.end(), s,
                               [](int64_t v, const FrameRun& r) { return v < r.first; });
    const FrameRun& r = *std::prev(it);
    VrFrame f = r.f;
    f.counter += r.cstep * static_cast<int>(s - r.first);
    return f;
}

// Two parts that overlap.  (1) The control loop -- sender, estimator feedback, encoder switches,
// the receiver's decoder swaps -- never looks at a decoder's output (FEC_Decoder::onReceive
// results only feed onDecodedMessage): it records, per decoder instance, its calls (consecutive
// seqs from `first`, erased = the packet was dropped) and which of them report which packet.
// (2) The symbolic decoders are independent of each other: as soon as the control loop is done
// with an instance (it is no longer the current or the old decoder), a worker thread replays its
// calls (one StreamPlanner per instance, erasure-free stretches on the fast path skipped in one
// step) and fills in the reported fates and coefficient rows; at the end one worker adds up the
// coding rate in the reference's order.
void VrPlan::run(int max_payload, int T, int B, int N, bool mds, const uint8_t* pattern, int64_t n_pattern,
                 int64_t P_value, bool async) {
    finish();
    L = max_payload;
    T_init = T;
    B_init = B;
    N_init = N;
    adaptive_mode_MDS = mds;
    P = P_value;
    const auto t_start = std::chrono::steady_clock::now();
    try {
        control(pattern, n_pattern, T, B, N, mds);
    } catch (...) {
        close_jobs();
        finish();
        throw;
    }
    t_dec_ = std::chrono::steady_clock::now();
    control_ms = std::chrono::duration<double, std::milli>(t_dec_ - t_start).count();
    if (!async) finish();
}

// s += r, `count` times, in float (round to nearest even), with the result of the sequential loop
// (Variable_Rate_FEC_Encoder.cpp:176-190 adds one rate per packet): 360 000 dependent adds were
// the last ~0.3 ms of the plan.  While s stays in one binade [2^(e-1), 2^e) its ulp u is fixed, so
// each add gives s + d with d = r rounded to a multiple of u -- the same d every time unless r / u
// is an odd multiple of 1/2 (a tie, whose rounding depends on s's last bit: stepped one by one).
// The adds are taken in one multiplication up to the first one whose exact sum reaches 2^e (there
// the ulp doubles), which is then stepped on its own.  Every intermediate value is a multiple of u
// below 2^e, exact in double and in float.
float float_add_repeated(float s, float r, int64_t count) {
    while (count > 0) {
        if (!(s > 0.0f) || !(r > 0.0f) || !std::isfinite(s) || !std::isfinite(r)) {
            s += r;
            --count;
            continue;
        }
        int e = 0;
        (void)std::frexp(s, &e);                  // s in [2^(e-1), 2^e)
        const double hi = std::ldexp(1.0, e);
        const double u = std::ldexp(1.0, e - 24);  // 24-bit significand
        const double q = static_cast<double>(r) / u;
        const float t = s + r;
        if (q - std::floor(q) == 0.5 || static_cast<double>(s) + r >= hi) {  // a tie, or the binade's last add
            s = t;
            --count;
            continue;
        }
        const double d = static_cast<double>(t) - static_cast<double>(s);
        if (d == 0.0) return s;  // r below half an ulp: s stays
        // m = the number of adds j = 0, 1, ... with s + j*d + r < hi (each of them adds exactly d)
        int64_t m = static_cast<int64_t>(std::ceil((hi - r - static_cast<double>(s)) / d));
        while (m > 0 && static_cast<double>(s) + static_cast<double>(m - 1) * d + r >= hi) --m;
        while (static_cast<double>(s) + static_cast<double>(m) * d + r < hi) ++m;
        m = std::min(m, count);
        s = static_cast<float>(static_cast<double>(s) + static_cast<double>(m) * d);
        count -= m;
    }
    return s;
}

void VrPlan::start_workers() {
    const int hw = vr_allowed_cpus();  // not hardware_concurrency: the process's cpuset may be smaller
    size_t nth = static_cast<size_t>(std::max(1, std::min(hw > 1 ? hw - 1 : 1, 8)));
    // placed on a group: one CPU per thread -- the control loop and the feedback producer keep two
    // of them (8 workers on top of those made the control loop 15 % slower: 1.30 vs 1.23 ms plan,
    // profiles/r04/vr/r04zj_plan_threads_ab.txt)
    const cpu_set_t grp = vr_group(t_pin_home);
    if (const int g = CPU_COUNT(&grp); g >= 4)
        nth = static_cast<size_t>(std::max(1, std::min<int>(static_cast<int>(nth), g - 2)));
    if (const char* e = std::getenv("FEC_VR_THREADS")) nth = std::max(1, std::atoi(e));
    {
        std::lock_guard<std::mutex> lk(qmu_);
        q_.clear();
        qclosed_ = false;
        qclosed_flag_.store(false, std::memory_order_relaxed);
        qsize_.store(0, std::memory_order_relaxed);
        sleepers_.store(0, std::memory_order_relaxed);
    }
    batch_.clear();
    // decoder-job slots for every instance this run can make (one per switch at most), allocated
    // by the control loop as it fills them; the chunk pointers never move while workers read them
    const size_t nchunks = static_cast<size_t>((P + 64 + kJobChunk) / kJobChunk) + 1;
    if (djobs_.size() < nchunks) djobs_.resize(nchunks);
    dpub_.store(0, std::memory_order_relaxed);
    dtake_.store(0, std::memory_order_relaxed);
    dfill_ = 0;
    if (workers_.size() != nth) stop_pool();  // (first run, or another thread count)
    recs_.resize(nth);
    for (auto& r : recs_) r.clear();
    pending_ = true;
    {
        std::lock_guard<std::mutex> lk(pmu_);
        pool_quit_ = false;
        pool_set_ = grp;
        pool_active_ = static_cast<int>(nth);
        ++pool_epoch_;
    }
    if (workers_.empty()) {
        for (size_t w = 0; w < nth; ++w)
            workers_.emplace_back([this, w] {
                uint64_t seen = 0;
                cpu_set_t pinned;
                CPU_ZERO(&pinned);
                for (;;) {
                    cpu_set_t set;
                    {
                        std::unique_lock<std::mutex> lk(pmu_);
                        pcv_.wait(lk, [&] { return pool_quit_ || pool_epoch_ != seen; });
                        if (pool_quit_) return;
                        seen = pool_epoch_;
                        set = pool_set_;
                    }
                    // on the control loop's group (a sparse one -- fewer than 4 CPUs: taskset,
                    // cgroup -- is left alone, as vr_pin_near does)
                    if (!CPU_EQUAL(&set, &pinned) && CPU_COUNT(&set) >= 4) {
                        (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
                        pinned = set;
                    }
                    worker_run(w);
                    std::lock_guard<std::mutex> lk(pmu_);
                    if (--pool_active_ == 0) pdone_.notify_all();
                }
            });
    } else {
        pcv_.notify_all();
    }
}

void VrPlan::stop_pool() {
    {
        std::lock_guard<std::mutex> lk(pmu_);
        pool_quit_ = true;
    }
    pcv_.notify_all();
    for (auto& th : workers_) th.join();
    workers_.clear();
}

VrPlan::~VrPlan() {
    finish();
    stop_pool();
}

// One run's jobs on worker w: feedback runs and the rate sum from the mutex queue, decoder
// instances claimed lock-free, until the control loop has closed the queue and every job is taken.
void VrPlan::worker_run(size_t w) {
    // pause-loop iterations a worker polls for work before sleeping (FEC_VR_SPIN; 0: sleep at once)
    static const int spin_max = [] {
        const char* e = std::getenv("FEC_VR_SPIN");
        return e ? std::max(0, std::atoi(e)) : 4096;
    }();
    auto decoder_ready = [&] { return dtake_.load(std::memory_order_relaxed) < dpub_.load(std::memory_order_acquire); };
    for (;;) {
        // the mutex queue first: feedback runs (queued before any decoder job) and the rate sum
        if (qsize_.load(std::memory_order_acquire) > 0) {
            DecJob j;
            bool got = false;
            {
                std::lock_guard<std::mutex> lk(qmu_);
                if (!q_.empty()) {
                    j = std::move(q_.front());
                    q_.pop_front();
                    qsize_.store(static_cast<int64_t>(q_.size()), std::memory_order_release);
                    got = true;
                }
            }
            if (got) {
                if (j.id <= -2) {  // feedback jobs of run -2 - id, in order
                    const int64_t c = -2 - static_cast<int64_t>(j.id), nj = static_cast<int64_t>(fb_jobs_.size());
                    const int64_t ch = static_cast<int64_t>(fb_chunk_);
                    for (int64_t jf = c * ch; jf < std::min(nj, (c + 1) * ch); ++jf) feedback_job(jf, fb_T_, fb_mds_);
                } else {  // final_sum_coding_rate, one float add per packet in sending order
                    float sum = 0;
                    for (const RateRun& r : rate_runs) sum = float_add_repeated(sum, r.rate, r.count);
                    sum_coding_rate = sum;
                }
                continue;
            }
        }
        // a decoder instance, claimed lock-free
        int64_t t = dtake_.load(std::memory_order_relaxed);
        if (t < dpub_.load(std::memory_order_acquire)) {
            if (dtake_.compare_exchange_weak(t, t + 1, std::memory_order_acq_rel, std::memory_order_relaxed))
                decode_instance(dslot(t), recs_[w]);
            continue;
        }
        // nothing: poll for a while (a job comes every ~0.5 us while the control loop runs),
        // then sleep on the condition variable
        bool any = false;
        for (int spin = 0; spin < spin_max && !any; ++spin) {
            any = qsize_.load(std::memory_order_acquire) > 0 || decoder_ready() ||
                  qclosed_flag_.load(std::memory_order_acquire);
            if (!any) __builtin_ia32_pause();
        }
        std::unique_lock<std::mutex> lk(qmu_);
        auto ready = [&] { return !q_.empty() || qclosed_ || decoder_ready(); };
        if (!ready()) {
            sleepers_.fetch_add(1, std::memory_order_seq_cst);
            qcv_.wait(lk, ready);
            sleepers_.fetch_sub(1, std::memory_order_relaxed);
        }
        if (q_.empty() && qclosed_ && !decoder_ready()) return;  // closed: every job published is taken
    }
}

// Jobs go to the workers in batches (one lock and one wake-up per batch: a wake-up per small job
// would cost the control thread more than the job).
void VrPlan::publish(DecJob&& j, bool flush) {
    batch_.push_back(std::move(j));
    if (!flush && batch_.size() < 8) return;
    bool wake;
    {
        std::lock_guard<std::mutex> lk(qmu_);
        for (DecJob& b : batch_) q_.push_back(std::move(b));
        qsize_.store(static_cast<int64_t>(q_.size()), std::memory_order_release);
        wake = sleepers_.load(std::memory_order_relaxed) > 0;  // a sleeper registered under qmu_
    }
    batch_.clear();
    if (wake) qcv_.notify_all();
}

void VrPlan::publish_decoder(int id, const VrInstance& d, const DecodeRules* rules, std::vector<Reports>& reps,
                             bool flush) {
    if (id >= 0) {
        const int64_t n = dfill_++;
        auto& chunk = djobs_[static_cast<size_t>(n / kJobChunk)];
        if (!chunk) chunk.reset(new DecJob[kJobChunk]);
        DecJob& j = chunk[n % kJobChunk];
        j.id = id;
        j.d = d;
        j.rules = rules;
        j.reps.swap(reps);  // (the slot's old list goes back to the finished instance, unused)
    }
    // release the filled slots four at a time (each store takes the line the polling workers
    // share); a worker about to sleep either sees them or is counted in sleepers_ (both
    // sequentially consistent), and is then woken
    if (dfill_ == dpub_.load(std::memory_order_relaxed) || (!flush && dfill_ % 4 != 0)) return;
    dpub_.store(dfill_, std::memory_order_seq_cst);
    if (sleepers_.load(std::memory_order_seq_cst) > 0) {
        { std::lock_guard<std::mutex> lk(qmu_); }
        qcv_.notify_all();
    }
}

void VrPlan::close_jobs() {
    {
        std::lock_guard<std::mutex> lk(qmu_);
        qclosed_ = true;
        qclosed_flag_.store(true, std::memory_order_release);  // pollers stop polling and take the lock
    }
    qcv_.notify_all();
}

void VrPlan::finish() {
    if (!pending_) return;
    close_jobs();
    {
        std::unique_lock<std::mutex> lk(pmu_);
        pdone_.wait(lk, [&] { return pool_active_ == 0; });
    }
    pending_ = false;
    lost = std::count(fate.begin(), fate.end(), static_cast<uint8_t>(kLost));
    // recovered packets in x order (each worker's list is in its own job order)
    std::vector<const RecEntry*> all;
    for (const auto& r : recs_)
        for (const RecEntry& e : r) all.push_back(&e);
    std::sort(all.begin(), all.end(), [](const RecEntry* a, const RecEntry* b) { return a->x < b->x; });
    const size_t nrec = all.size();
    rec_x.resize(nrec);
    rec_dec.resize(nrec);
    rec_coef.resize(nrec * kVrCoefStride);
    for (size_t i = 0; i < nrec; ++i) {
        rec_x[i] = all[i]->x;
        rec_dec[i] = fate_dec[static_cast<size_t>(all[i]->x)];
        std::memcpy(&rec_coef[i * kVrCoefStride], all[i]->coef.data(), kVrCoefStride);
    }
    decoders_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_dec_).count();
}

// One decoder instance's calls (Decoder::decodeStream, Decoder.cpp:72-175) through a symbolic
// StreamPlanner.  Between erasures the planner is on the fast path: such a stretch is skipped in
// one step and its reported packets are copies (or, within the instance's first T calls, nothing
// -- reported as lost, like any kNone output).
void VrPlan::decode_instance(const DecJob& job, std::vector<RecEntry>& recs) {
    const VrInstance& d = job.d;
    const Geometry g = Geometry::make(L, d.T, d.B, d.N);
    StreamPlanner pl(g, job.rules);
    const Reports* rp = job.reps.data();
    const Reports* rp_end = rp + job.reps.size();
    for (const Reports* r = rp; r != rp_end; ++r)  // the packets this instance reports (report_range)
        std::fill(fate_dec.begin() + (r->lo - r->xoff), fate_dec.begin() + (r->hi - r->xoff), job.id);
    size_t di = static_cast<size_t>(std::lower_bound(drops.begin(), drops.end(), d.first) - drops.begin());
    int64_t s = d.first;
    while (s < d.end) {
        const int64_t t = s - d.first;
        const int64_t nxt = di < drops.size() ? drops[di] : INT64_MAX;
        while (rp != rp_end && rp->hi <= s) ++rp;
        if (nxt > s && pl.fast_at(t)) {
            const int64_t e = std::min(nxt, d.end);
            pl.skip_received(t, e - s);
            // reported packets of [s, e): copies once the instance is T calls old
            for (const Reports* r = rp; r != rp_end && r->lo < e; ++r) {
                const int64_t lo = std::max(r->lo, s), hi = std::min(r->hi, e);
                if (lo >= hi) continue;
                const int64_t c = std::min(hi, std::max(lo, d.first + g.T));  // seqs before c: kNone
                if (c > lo) std::memset(&fate[static_cast<size_t>(lo - r->xoff)], kLost, static_cast<size_t>(c - lo));
                if (hi > c) std::memset(&fate[static_cast<size_t>(c - r->xoff)], kCopy, static_cast<size_t>(hi - c));
                std::memset(&slow[static_cast<size_t>(lo - r->xoff)], 0, static_cast<size_t>(hi - lo));
            }
            s = e;
            continue;
        }
        const bool er = nxt == s;
        if (er) ++di;
        const StepResult r = pl.step(t, er);
        if (rp != rp_end && rp->lo <= s) {
            const int64_t x = s - rp->xoff;
            const PacketFate f = r.fate == kNone ? kLost : r.fate;
            fate[static_cast<size_t>(x)] = f;
            slow[static_cast<size_t>(x)] = r.slow ? 1 : 0;
            if (f == kRecovered) {
                recs.emplace_back();
                recs.back().x = x;
                recs.back().coef.fill(0);
                std::memcpy(recs.back().coef.data(), r.coef, static_cast<size_t>(g.k) * g.n);
            }
        }
        ++s;
    }
}

// The receiver's estimator feedback [T, B_est, N_est] after each received packet
// (Application_Layer_Receiver.cpp:375-393, :430-436) depends only on which packets arrive: the
// message T the estimators see is the sender's T, which never changes (the feedback's T is the
// estimators' own).  The foreground estimator after received packet s is
//   * s < r_2: the initial pair's (both fed from the start, so identical);
//   * r_c <= s < r_{c+1} (c >= 2): the background one created at swap c-1, fed (r_{c-1}, s];
// where r_c, the c-th swap, is the first received packet s >= max(100c, r_{c-1} + 1)
// (`seq + 1 > cycle * 100`, one swap per received packet).  So the feedback splits into
// independent jobs, one per swap; within a job, erasure-free stretches at the estimator's fixed
// point are skipped to the next drop (estimate() would change only previous_win_end there).  The
// jobs run in order on a producer thread while the control loop consumes their results (FbCursor):
// job j's list of (received seq, value) changes is published once complete.
void VrPlan::feedback_plan(int64_t end) {
    auto next_received = [&](int64_t s) {  // first received seq >= s
        auto it = std::lower_bound(drops.begin(), drops.end(), s);
        while (it != drops.end() && *it == s) {
            ++s;
            ++it;
        }
        return s;
    };
    fb_swaps_.assign({-1, -1});  // [c] = c-th swap (c >= 1); [0] unused
    for (int64_t c = 1;; ++c) {
        const int64_t s = next_received(std::max(c * kEstimationCycle, fb_swaps_.back() + 1));
        if (s >= end) break;
        if (c == 1) fb_swaps_[1] = s; else fb_swaps_.push_back(s);
    }
    const int64_t nswap = fb_swaps_[1] < 0 ? 0 : static_cast<int64_t>(fb_swaps_.size()) - 1;
    auto swap_at = [&](int64_t c) { return c <= nswap ? fb_swaps_[static_cast<size_t>(c)] : end; };
    // job 0: the initial estimator over [0, r_2); job j >= 1 (swap c = j + 1): a fresh one fed
    // from r_{c-1}+1, recording [r_c, r_{c+1})
    const int64_t njobs = 1 + std::max<int64_t>(0, nswap - 1);
    fb_jobs_.resize(static_cast<size_t>(njobs));
    for (int64_t j = 0; j < njobs; ++j) {
        FbJob& b = fb_jobs_[static_cast<size_t>(j)];
        const int64_t c = j + 1;
        b.from = j == 0 ? 0 : swap_at(c - 1) + 1;
        b.rec = j == 0 ? 0 : swap_at(c);
        b.to = j == 0 ? swap_at(2) : swap_at(c + 1);
        b.changes.clear();
    }
    fb_ready_.reset(new std::atomic<uint8_t>[static_cast<size_t>(njobs) + 1]);
    for (int64_t j = 0; j <= njobs; ++j) fb_ready_[static_cast<size_t>(j)].store(0, std::memory_order_relaxed);
}

void VrPlan::feedback_run(int T, bool mds) {
    const int64_t njobs = static_cast<int64_t>(fb_jobs_.size());
    for (int64_t j = 0; j < njobs; ++j) feedback_job(j, T, mds);
}

// One feedback job (one estimator's stretch), then its ready flag.  The jobs are independent: the
// workers run them in parallel, ahead of every decoder job (start_workers' queue is FIFO).
void VrPlan::feedback_job(int64_t j, int T, bool mds) {
    {
        FbJob& b = fb_jobs_[static_cast<size_t>(j)];
        ParameterEstimator e(kTTot, j == 0 ? mds : false);
        uint32_t last = 0xffffffffu;
        auto di = std::lower_bound(drops.begin(), drops.end(), b.from);
        auto put = [&](int64_t s) {
            const uint32_t v = uint32_t(e.T) | uint32_t(e.B_current) << 8 | uint32_t(e.N_current) << 16;
            if (v != last) {
                b.changes.push_back(FbChange{s, v});
                last = v;
            }
        };
        for (int64_t s = b.from; s < b.to;) {
            if (di != drops.end() && *di == s) {  // dropped: nothing reaches the receiver
                ++di;
                ++s;
                continue;
            }
            const int64_t nd = di != drops.end() ? std::min(*di, b.to) : b.to;
            if (e.steady(s, T)) {  // every received packet of [s, nd) leaves the estimator as it is
                if (nd > b.rec) put(std::max(s, b.rec));
                e.previous_win_end = nd - 1;
                s = nd;
                continue;
            }
            e.estimate(s, T);
            if (s >= b.rec) put(s);
            ++s;
        }
        fb_ready_[static_cast<size_t>(j)].store(1, std::memory_order_release);
    }
}

// The control loop's view of the feedback stream: value(s) = the feedback after received packet s
// (packets in increasing order), next() = the first change after the last value() asked for, or
// the end of what the producer has published so far.
struct VrPlan::FbCursor {
    VrPlan& p;
    size_t j = 0, e = 0;
    uint32_t cur = 0;
    size_t changes = 0;
    int64_t done = 0;  // jobs known complete: the shared counter is read only past them
    explicit FbCursor(VrPlan& plan) : p(plan) {}
    bool ready(size_t job) {  // jobs complete in any order; the cursor reads them in order
        if (static_cast<int64_t>(job) < done) return true;
        const int64_t n = static_cast<int64_t>(p.fb_jobs_.size());
        while (done < n && p.fb_ready_[static_cast<size_t>(done)].load(std::memory_order_acquire)) ++done;
        return static_cast<int64_t>(job) < done;
    }
    double waited_ms = 0;  // FEC_VR_DEBUG: time the control loop spent waiting for the producer
    void wait(size_t job) {
        if (ready(job)) return;
        const auto t0 = std::chrono::steady_clock::now();
        while (!ready(job)) std::this_thread::yield();
        waited_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    // skip to the next entry that changes the value; false at the end of the published jobs
    bool peek(int64_t* seq, bool block) {
        for (;;) {
            if (j >= p.fb_jobs_.size()) return false;
            if (!ready(j)) {
                if (!block) return false;
                wait(j);
            }
            const auto& ch = p.fb_jobs_[j].changes;
            if (e >= ch.size()) {
                ++j;
                e = 0;
                continue;
            }
            if (ch[e].v == cur) {
                ++e;
                continue;
            }
            *seq = ch[e].seq;
            return true;
        }
    }
    uint32_t value(int64_t s) {
        int64_t q;
        while (peek(&q, true) && q <= s) {
            cur = p.fb_jobs_[j].changes[e++].v;
            ++changes;
        }
        return cur;
    }
    // first seq >= s at which the value may change (a bound when the producer is behind)
    int64_t next(int64_t s) {
        int64_t q;
        if (peek(&q, false)) return q;
        if (j >= p.fb_jobs_.size()) return INT64_MAX;
        return std::max(s, p.fb_jobs_[j].rec);  // the first seq of the job not yet published
    }
};

void VrPlan::control(const uint8_t* pattern, int64_t n_pattern, int T, int B, int N, bool mds) {
    frame_runs.clear();
    rate_runs.clear();
    drops.clear();
    enc.clear();
    dec.clear();
    fate.assign(static_cast<size_t>(P), kNone);
    fate_dec.assign(static_cast<size_t>(P), -1);
    slow.assign(static_cast<size_t>(P), 0);
    lost = switches = 0;
    steady_packets = 0;
    transition_packets = 0;
    sum_coding_rate = 0;
    // per decoder instance: its report ranges (kept across runs with their capacity: a run's
    // instance i reuses the list of the previous run's, no allocation once warm) and its rules
    std::vector<std::vector<Reports>>& reps = reps_;
    std::vector<const DecodeRules*>& drules = drules_;
    drules.clear();

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
    // dropped packets (ERASURE_TYPE 5: pattern byte 1 for seq < P+T), then the feedback stream
    const auto tc0 = std::chrono::steady_clock::now();
    const int64_t n_drop = std::min<int64_t>(P + T, n_pattern);  // packets the pattern can drop
    // eight pattern bytes per test (a memchr call per drop cost ~20 ns each, 5 543 drops)
    {
        int64_t q = 0;
        for (; q + 8 <= n_drop; q += 8) {
            uint64_t w;
            std::memcpy(&w, pattern + q, 8);
            if (w == 0) continue;
            for (int b = 0; b < 8; ++b)
                if (pattern[q + b] == 1) drops.push_back(q + b);
        }
        for (; q < n_drop; ++q)
            if (pattern[q] == 1) drops.push_back(q);
    }
    feedback_plan(P + T + 1);
    // FEC_VR_FB_SYNC (diagnostic): the feedback jobs run to the end on this thread first
    const bool fb_sync = std::getenv("FEC_VR_FB_SYNC") != nullptr;
    if (fb_sync) feedback_run(T, mds);
    t_pin_home = vr_pin_home();
    // FEC_VR_PIN=2: the control loop itself on the group too, for the rest of this function
    struct CallerPlacement {
        cpu_set_t saved;
        bool held = false;
        explicit CallerPlacement(int home) {
            if (home < 0 || vr_pin_mode() < 2) return;
            if (pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) != 0) return;
            held = true;
            vr_pin_near(home);
        }
        ~CallerPlacement() {
            if (held) (void)pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
        }
    } caller_placement{t_pin_home};
    // The feedback jobs: on the worker pool, ahead of the decoder jobs (round 5 ran them in order on
    // one producer thread while the control loop waited for them; FEC_VR_FB_THREAD=1 restores that)
    const bool fb_thread_on = !fb_sync && std::getenv("FEC_VR_FB_THREAD") != nullptr;
    fb_T_ = T;
    fb_mds_ = mds;
    std::thread fb_thread;  // (only for FEC_VR_FB_THREAD=1)
    if (fb_thread_on)
        fb_thread = std::thread([this, T, mds, home = t_pin_home] {
            vr_pin_near(home);
            feedback_run(T, mds);
        });
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } fb_join{fb_thread};
    FbCursor fb(*this);
    const auto tc1 = std::chrono::steady_clock::now();
    start_workers();
    if (!fb_sync && !fb_thread_on) {
        // a few contiguous runs of jobs, one per worker (a queue entry per job -- thousands of
        // them -- kept the workers on the queue's lock while the control loop published)
        const size_t nj = fb_jobs_.size();
        size_t nchunk = std::max<size_t>(1, workers_.size());
        if (const char* e = std::getenv("FEC_VR_FB_CHUNKS")) nchunk = static_cast<size_t>(std::max(1, std::atoi(e)));
        nchunk = std::min(nchunk, std::max<size_t>(1, nj));
        fb_chunk_ = (nj + nchunk - 1) / nchunk;
        std::lock_guard<std::mutex> lk(qmu_);
        for (size_t c = 0; c * fb_chunk_ < nj; ++c) {
            DecJob fj;
            fj.id = -2 - static_cast<int>(c);
            q_.push_back(std::move(fj));
        }
        qsize_.store(static_cast<int64_t>(q_.size()), std::memory_order_release);
    }
    qcv_.notify_all();
    size_t dri = 0;       // next drop
    FEC_VR_PROF_DECL
    uint8_t udp[12] = {};
    // ---- Variable_Rate_FEC_Decoder (Variable_Rate_FEC_Decoder.cpp:25-80, 2133-2400, 2440-2514) ----
    int64_t seq_start = -1, latest_seq = -1, sdc = -1, sde = -1;
    int dT = 0, dB = 0, dN = 0;
    int dcur = -1, dold = -1;
    bool dcf = false;

    auto new_decoder = [&](int T_, int B_, int N_, int64_t first) {
        VrInstance v;
        v.T = T_;
        v.B = B_;
        v.N = N_;
        v.first = v.end = first;
        v.role_switch = -1;  // set when it becomes the old decoder
        dec.push_back(v);
        const size_t id = dec.size() - 1;
        if (id < reps.size())
            reps[id].clear();
        else
            reps.emplace_back();
        drules.push_back(&rules_for(T_, B_, N_));
        return static_cast<int>(dec.size()) - 1;
    };
    // an instance the control loop is done with (neither the current nor the old decoder)
    auto done_with = [&](int id) {
        publish_decoder(id, dec[static_cast<size_t>(id)], drules[static_cast<size_t>(id)], reps[static_cast<size_t>(id)]);
    };
    auto call = [&](int id, int64_t seq) {
        if (seq != dec[id].end) throw std::logic_error("vr: decoder calls out of order");
        dec[id].end = seq + 1;
    };
    auto call_range = [&](int id, int64_t lo, int64_t hi) {  // call(id, s) for s in [lo, hi)
        if (lo != dec[id].end) throw std::logic_error("vr: decoder calls out of order");
        dec[id].end = hi;
    };
    const bool fast_transitions = !std::getenv("FEC_VR_NO_FAST_TRANSITION");
    // Stretches run through dropped packets (FEC_VR_NO_DROP_STRETCH: they end before a drop): a drop
    // changes nothing the loop tracks but the receiver's view -- the next received packet calls and
    // reports the missing ones exactly as if they had arrived, and the feedback after it is bounded by
    // the feedback stream's next change -- so a stretch only has to end on a received packet.
    const bool drop_stretch = !std::getenv("FEC_VR_NO_DROP_STRETCH");
    // FEC_VR_FB_STOP (A/B): steady stretches end before the feedback change's packet (round 5)
    const bool fb_through = !std::getenv("FEC_VR_FB_STOP");
    // one past the last received packet in [lo, hi), or lo if every one of them drops.  The drop
    // cursor dri is at lo (drops[dri] is the first drop >= lo): the drops in [lo, hi) are scanned
    // from it (a stretch holds a few at most; a binary search over all of them per call was ~200
    // cycles of the control loop's transitions)
    auto received_end = [&](int64_t lo, int64_t hi) {
        size_t j = dri;
        while (j < drops.size() && drops[j] < hi) ++j;
        int64_t e = hi;
        while (e > lo && j > dri && drops[j - 1] == e - 1) {
            --j;
            --e;
        }
        return e;
    };
    // onDecodedMessage (:2403-2436): packets seq - T >= seq_start are reported once.  Instance id
    // reports the seqs [lo, hi) (packets x = seq - dT in [seq_start, P)), extending its newest range.
    auto report_range = [&](int id, int64_t lo, int64_t hi) {
        lo = std::max(lo, seq_start + dT);
        hi = std::min(hi, P + dT);
        if (lo >= hi) return;
        std::vector<Reports>& rv = reps[static_cast<size_t>(id)];
        if (!rv.empty() && rv.back().hi == lo && rv.back().xoff == dT)
            rv.back().hi = hi;
        else
            rv.push_back(Reports{id, lo, hi, dT});
        // fate_dec of [lo, hi) is written by the worker that replays instance id (decode_instance):
        // off the control loop, whose steady stretches would otherwise fill 4 bytes per packet
    };
    auto report = [&](int id, int64_t seq) { report_range(id, seq, seq + 1); };
    auto update_decoder = [&](int T_, int B_, int N_, int64_t first) {  // (:2520-2536)
        if (dold >= 0) FEC_VR_SUB(6, done_with(dold))
        dold = dcur;
        dT = T_;
        dB = B_;
        dN = N_;
        FEC_VR_SUB(7, dcur = new_decoder(T_, B_, N_, first))
        dec[dold].role_switch = first;
    };
    // frames as runs: equal frames, or a transition's frames whose counter grows by one per packet
    // (cstep 1; one run per transition instead of one per packet)
    // (`n` packets from seq carry f; seq is the packet after the last run's last)
    auto put_frame = [&](int64_t seq, const VrFrame& f, int64_t n = 1) {
        if (!frame_runs.empty()) {
            FrameRun& b = frame_runs.back();
            if (b.f.same_but_counter(f)) {
                const int64_t d = seq - b.first;
                if (b.cstep == 0 && f.counter == b.f.counter) return;
                if (n == 1 && b.cstep == 1 && f.counter == b.f.counter + d) return;
                if (n == 1 && b.cstep == 0 && d == 1 && f.counter == b.f.counter + 1) {
                    b.cstep = 1;
                    return;
                }
            }
        }
        frame_runs.push_back(FrameRun{seq, f, 0});
    };
    auto put_rate = [&](int64_t count, float rate) {
        if (!rate_runs.empty() && rate_runs.back().rate == rate)
            rate_runs.back().count += count;
        else
            rate_runs.push_back(RateRun{count, rate});
    };

    int64_t n_iter = 0, n_jump = 0;  // FEC_VR_DEBUG counters
    timespec cpu0{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &cpu0);
    rusage ru0{};
    getrusage(RUSAGE_THREAD, &ru0);
    for (int64_t seq = 0;; ++seq) {
        ++n_iter;
        FEC_VR_PROF(5)
#ifdef FEC_VR_PROFILE
        int prof_why = (cur < 0 ? 1 : 0) | (transition_flag ? 2 : 0) | (double_coding_flag ? 4 : 0) |
                       (counter_transition <= eT ? 8 : 0) | (latest_seq != seq ? 16 : 0) | (dcf ? 32 : 0) |
                       (sdc >= seq ? 64 : 0) | (dT != eT || dB != eB || dN != eN ? 128 : 0) |
                       (udp[3] != eT || udp[4] != eB || udp[5] != eN ? 256 : 0) | (fb.next(seq) <= seq ? 512 : 0);
#endif
        // ---- steady stretch: the same frame, every packet received, nothing switching ----
        // Every branch below is then fixed: the feedback repeats (no change in the feedback
        // stream), the encoder has no switch to make and no transition running, the decoder has
        // no gap, no parameter change and no double decoding.  Such packets are appended in one
        // step (frames, coding-rate terms and reports as runs).  The stretch runs through the next
        // feedback change's packet (its own frame, rate and decoder call are a steady packet's; only
        // the udp after it differs, set at the end) and ends before the last packet.  It may start
        // at the packet that ends a transition (counter T+1: the encoder cannot switch there and
        // clears transition_flag, which is all that differs from a steady packet).
        const bool flip = fast_transitions && transition_flag && counter_transition == eT + 1;
        if (cur >= 0 && (!transition_flag || flip) && !double_coding_flag && counter_transition > eT &&
            seq_start >= 0 && latest_seq == seq && !dcf && sdc < seq && dT == eT && dB == eB && dN == eN &&
            seq < P + T - 1) {
            const int fT = adaptive && udp[0] != 0 ? udp[0] : sT, fB = adaptive && udp[0] != 0 ? udp[1] : sB,
                      fN = adaptive && udp[0] != 0 ? udp[2] : sN;
            const int aT = adaptive && udp[0] != 0 ? udp[3] : sT_ack, aB = adaptive && udp[0] != 0 ? udp[4] : sB_ack;
            const bool would_switch = (fT != eT || fB != eB || fN != eN) && aT == eT && aB == eB;
#ifdef FEC_VR_PROFILE
            prof_why |= (would_switch ? 1024 : 0) | (seq >= P + T - 1 ? 2048 : 0);
#endif
            if (!would_switch && udp[3] == eT && udp[4] == eB && udp[5] == eN) {
                while (dri < drops.size() && drops[dri] < seq) ++dri;
                const int64_t next_drop = dri < drops.size() ? drops[dri] : INT64_MAX;
                const int64_t next_fb = fb.next(seq);
                // through the feedback change's packet (a received one) when it comes before the last
                const bool fb_step = drop_stretch && fb_through && next_fb < P + T - 1 &&
                                     !(next_fb < n_pattern && pattern[next_fb] == 1);
                const int64_t end = fb_step ? next_fb + 1
                                  : drop_stretch ? received_end(seq, std::min(next_fb, P + T - 1))
                                                 : std::min({next_drop, next_fb, P + T - 1});
#ifdef FEC_VR_PROFILE
                prof_why |= end > seq ? 0 : 4096;
#endif
                if (end > seq) {
                    if (adaptive && udp[0] != 0) {
                        sT = udp[0];
                        sB = udp[1];
                        sN = udp[2];
                        sT_ack = udp[3];
                        sB_ack = udp[4];
                        sN_ack = udp[5];
                    }
                    if (flip) transition_flag = false;
                    VrFrame fr;
                    fr.T = eT;
                    fr.B = eB;
                    fr.N = eN;
                    fr.enc_cur = cur;
                    fr.counter = counter_transition;
                    put_frame(seq, fr, end - seq);
                    put_rate(end - seq, static_cast<float>(eT - eN + 1) / (eT - eN + 1 + eB));
                    report_range(dcur, seq, end);
                    enc[cur].end = end;
                    dec[dcur].end = end;  // call(dcur, s) for every s
                    latest_seq = end;
                    sent = end;
                    steady_packets += end - seq;
                    ++n_jump;
                    if (fb_step) {  // the udp after the stretch's last packet (T, B, N: the frame's)
                        const uint32_t v = fb.value(end - 1);
                        udp[0] = static_cast<uint8_t>(v);
                        udp[1] = static_cast<uint8_t>(v >> 8);
                        udp[2] = static_cast<uint8_t>(v >> 16);
                    }
                    seq = end;
                }
            }
        }
        FEC_VR_PROF(0)
        // ---- transition stretch: double coding after a switch, every packet received ----
        // The encoder cannot switch again before its transition ends (transition_flag), so the
        // feedback only moves the sender's next parameters; the frames differ only in their
        // counter (and carry the old instance while double coding); the decoder, already on the new
        // tuple, calls the old and the new instance up to sde, then the new one alone.  Packets
        // [seq, end) are appended in one pass, up to the transition's last packet (counter == eT),
        // the next drop and the last packet -- the same state as packet-by-packet below.
        if (fast_transitions && cur >= 0 && transition_flag && counter_transition >= 1 && counter_transition <= eT &&
            seq_start >= 0 && latest_seq == seq && sdc < seq && dT == eT && dB == eB && dN == eN &&
            seq < P + T - 1) {
            while (dri < drops.size() && drops[dri] < seq) ++dri;
            const int64_t next_drop = dri < drops.size() ? drops[dri] : INT64_MAX;
            const int64_t tend = std::min(seq + (eT - counter_transition + 1), P + T - 1);
            const int64_t end = drop_stretch ? received_end(seq, tend) : std::min(next_drop, tend);
            if (end > seq) {
                if (adaptive && udp[0] != 0) {  // the start of packet seq's iteration
                    sT = udp[0];
                    sB = udp[1];
                    sN = udp[2];
                    sT_ack = udp[3];
                    sB_ack = udp[4];
                    sN_ack = udp[5];
                }
                const float rate1 = static_cast<float>(eT - eN + 1) / (eT - eN + 1 + eB);
                const float rate2 = static_cast<float>(eT - eN + 1) /
                                    ((eT - eN + 1 + eB) + (eT - eN_old + 1) + (eT - eN_old + 1 + eB));
                // per packet q (counter c = c0 + q - seq): the packet with c == eT ends double coding
                // before its rate is added, so packets c < eT carry the old codeword and rate2, the
                // rest rate1 -- in closed form: n2 double-coded packets, then n - n2
                const int64_t n = end - seq;
                const int c0 = counter_transition;
                const int64_t n2 = double_coding_flag ? std::min<int64_t>(n, eT - c0) : 0;
                auto frames = [&](int64_t q0, int64_t cnt, bool with_old) {
                    // the first packets per packet (they settle the run's counter step), the rest
                    // extend that run
                    for (int64_t q = q0; q < q0 + std::min<int64_t>(cnt, 3); ++q) {
                        VrFrame fr;
                        fr.T = eT;
                        fr.B = eB;
                        fr.N = eN;
                        fr.enc_cur = cur;
                        fr.counter = c0 + static_cast<int>(q - seq);
                        if (with_old) fr.enc_old = old;
                        put_frame(q, fr);
                    }
                };
                if (n2 > 0) {
                    put_rate(n2, rate2);
                    frames(seq, n2, old >= 0);
                    if (old >= 0) enc[old].end = seq + n2;
                }
                if (n > n2) {
                    put_rate(n - n2, rate1);
                    frames(seq + n2, n - n2, false);
                }
                if (double_coding_flag && c0 + n - 1 >= eT) double_coding_flag = false;
                counter_transition = c0 + static_cast<int>(n);
                enc[cur].end = end;
                // decoder: [seq, split) double decoding (old and new instance), [split, end) the new one
                const int64_t split = dcf ? std::min(end, sde + 1) : seq;
                if (split > seq) {
                    if (dold >= 0) {
                        call_range(dold, seq, split);
                        report_range(dold, seq, split);
                    }
                    call_range(dcur, seq, split);
                }
                if (end > split) {
                    dcf = false;
                    call_range(dcur, split, end);
                    report_range(dcur, split, end);
                }
                latest_seq = end;
                sent = end;
                transition_packets += end - seq;
                // the sender's parameters at the start of packet end-1's iteration (the udp after the
                // last packet received before it), and the udp after end-1 (received)
                if (const int64_t r = received_end(seq, end - 1); r > seq) {
                    const uint32_t v = fb.value(r - 1);
                    if (adaptive && (v & 0xff) != 0) {
                        sT = static_cast<int>(v & 0xff);
                        sB = static_cast<int>(v >> 8 & 0xff);
                        sN = static_cast<int>(v >> 16 & 0xff);
                        sT_ack = eT;
                        sB_ack = eB;
                        sN_ack = eN;
                    }
                }
                const uint32_t fbv = fb.value(end - 1);
                udp[0] = static_cast<uint8_t>(fbv);
                udp[1] = static_cast<uint8_t>(fbv >> 8);
                udp[2] = static_cast<uint8_t>(fbv >> 16);
                udp[3] = static_cast<uint8_t>(eT);
                udp[4] = static_cast<uint8_t>(eB);
                udp[5] = static_cast<uint8_t>(eN);
                // packet `end` from the top: a steady stretch may start at it (the transition's end)
                seq = end - 1;
                FEC_VR_PROF(1)
                continue;
            }
        }
        FEC_VR_PROF(1)
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
            put_rate(1, static_cast<float>(eT - eN + 1) / (eT - eN + 1 + eB));
        else
            put_rate(1, static_cast<float>(eT - eN + 1) / ((eT - eN + 1 + eB) + (eT - eN_old + 1) + (eT - eN_old + 1 + eB)));
        put_frame(seq, fr);
        const bool drop = seq < P + T && seq < n_pattern && pattern[seq] == 1;
        sent = seq + 1;

        // ---- Application_Layer_Receiver::receive_message_and_decode ----
        FEC_VR_PROF(2)
#ifdef FEC_VR_PROFILE
        if (!drop && !transition_flag && latest_seq == seq) ++prof_why_h[prof_why];
        ++prof_cls[(drop ? 1 : 0) | (transition_flag ? 2 : 0) | (double_coding_flag ? 4 : 0) |
                   (latest_seq != seq ? 8 : 0) | (fr.counter == 0 ? 16 : 0) | (seq_start < 0 ? 32 : 0)];
#endif
        if (drop) continue;  // artificial erasure: returns -1, feedback unchanged
        const uint32_t fbv = fb.value(seq);  // the estimators' feedback after seq
        FEC_VR_PROF(3)
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
        FEC_VR_PROF(4)
        udp[0] = static_cast<uint8_t>(fbv);
        udp[1] = static_cast<uint8_t>(fbv >> 8);
        udp[2] = static_cast<uint8_t>(fbv >> 16);
        udp[3] = static_cast<uint8_t>(fr.T);
        udp[4] = static_cast<uint8_t>(fr.B);
        udp[5] = static_cast<uint8_t>(fr.N);
        if (seq >= P + T - 1) break;  // application_local_simulation.cpp:813
    }
    for (auto* list : {&enc, &dec})
        for (auto& e : *list)
            if (e.role_switch < 0) e.role_switch = e.end;  // never became the old instance
    // dropped flags of every sent packet
    erased.assign(static_cast<size_t>(sent), 0);
    for (int64_t s : drops) erased[static_cast<size_t>(s)] = 1;
    if (std::getenv("FEC_VR_DEBUG")) {
        const auto tc2 = std::chrono::steady_clock::now();
        timespec cpu1{};
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &cpu1);
        rusage ru1{};
        getrusage(RUSAGE_THREAD, &ru1);
        FEC_VR_PROF_PRINT
        std::fprintf(stderr, "vr control: loop thread cpu %.3f ms (user %.3f sys %.3f), %ld minor faults\n",
                     (cpu1.tv_sec - cpu0.tv_sec) * 1e3 + (cpu1.tv_nsec - cpu0.tv_nsec) * 1e-6,
                     (ru1.ru_utime.tv_sec - ru0.ru_utime.tv_sec) * 1e3 + (ru1.ru_utime.tv_usec - ru0.ru_utime.tv_usec) * 1e-3,
                     (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) * 1e3 + (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec) * 1e-3,
                     ru1.ru_minflt - ru0.ru_minflt);
        std::fprintf(stderr, "vr control: drops %.3f ms, loop %.3f ms (%zu feedback changes, %.3f ms waiting for "
                     "them; %lld iterations, %lld steady stretches, %zu drops)\n",
                     std::chrono::duration<double, std::milli>(tc1 - tc0).count(),
                     std::chrono::duration<double, std::milli>(tc2 - tc1).count(), fb.changes, fb.waited_ms,
                     static_cast<long long>(n_iter), static_cast<long long>(n_jump), drops.size());
    }
    fb_wait_ms = fb.waited_ms;
    // the last two decoder instances, then the coding-rate sum; no more jobs
    if (dold >= 0) done_with(dold);
    if (dcur >= 0) done_with(dcur);
    std::vector<Reports> none;
    publish_decoder(-1, VrInstance{}, nullptr, none, true);  // the slots not yet released
    DecJob rate;
    rate.id = -1;
    publish(std::move(rate), true);
    close_jobs();
}

}  // namespace fec

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
struct fec_vr_plan;

namespace {
// Host tables sent to the device: one device buffer (grown on demand, kept across re-runs) and a
// page-locked staging buffer filled by add() and sent with one asynchronous copy.  The staging
// buffer is rewritten only after the copy out of it has completed, the device buffer only after
// the launches that read it (events `sent` / `used`).
struct Upload {
    std::vector<std::pair<const void**, size_t>> fix;
    uint8_t* h = nullptr;
    size_t hcap = 0, size = 0;
    void* d = nullptr;
    size_t dcap = 0;
    hipEvent_t sent = nullptr, used = nullptr;

    Upload() = default;
    Upload(const Upload&) = delete;
    Upload& operator=(const Upload&) = delete;
    ~Upload() {
        if (sent) (void)hipEventSynchronize(sent);
        if (used) (void)hipEventSynchronize(used);
        if (d) (void)hipFree(d);
        fec::vr_host_free(h);
        if (sent) (void)hipEventDestroy(sent);
        if (used) (void)hipEventDestroy(used);
    }
    int begin() {
        if (!sent) FEC_HIP(hipEventCreateWithFlags(&sent, hipEventDisableTiming));
        if (!used) FEC_HIP(hipEventCreateWithFlags(&used, hipEventDisableTiming));
        FEC_HIP(hipEventSynchronize(sent));
        size = 0;
        fix.clear();
        return FEC_OK;
    }
    template <typename T>
    void add(const T** dptr, const T* src, size_t count) {
        const size_t off = (size + 255) & ~size_t(255);
        const size_t need = off + std::max<size_t>(1, count) * sizeof(T);
        if (need > hcap) {
            const size_t cap = std::max(need, hcap + hcap / 2);
            uint8_t* nh = static_cast<uint8_t*>(fec::vr_host_alloc(cap));
            if (size) std::memcpy(nh, h, size);
            fec::vr_host_free(h);
            h = nh;
            hcap = cap;
        }
        if (count) std::memcpy(h + off, src, count * sizeof(T));
        fix.emplace_back(reinterpret_cast<const void**>(dptr), off);
        size = need;
    }
    template <typename T, typename A>
    void add(const T** dptr, const std::vector<T, A>& v) { add(dptr, v.data(), v.size()); }
    // device buffer of at least `bytes`, free of earlier readers on stream s
    static int reserve(void** dp, size_t* cap, size_t bytes, hipEvent_t used, hipStream_t s) {
        FEC_HIP(hipStreamWaitEvent(s, used, 0));
        if (bytes <= *cap) return FEC_OK;
        if (*dp) {
            FEC_HIP(hipEventSynchronize(used));
            (void)hipFree(*dp);
            *dp = nullptr;
            *cap = 0;
        }
        const size_t c = bytes + bytes / 4;
        if (hipMalloc(dp, c) != hipSuccess) return FEC_ERR_NOMEM;
        *cap = c;
        return FEC_OK;
    }
    int commit(hipStream_t s) {
        if (int st = reserve(&d, &dcap, std::max<size_t>(16, size), used, s)) return st;
        FEC_HIP(hipMemcpyAsync(d, h, size, hipMemcpyHostToDevice, s));
        FEC_HIP(hipEventRecord(sent, s));
        for (auto& f : fix) *f.first = static_cast<const uint8_t*>(d) + f.second;
        return FEC_OK;
    }
    int done_reading(hipStream_t s) { return hipEventRecord(used, s) == hipSuccess ? FEC_OK : FEC_ERR_HIP; }
};

// Side streams for the independent launches of one batch (the tuples' tile encoders, the generic
// encoder, the recovery next to the copy): each is forked from the caller's stream by an event and
// joined back into it before the call returns, so the caller sees one ordered stream.  The small
// launches are latency-bound walks (a tuple of a few thousand packets: ~21 us whatever its size,
// r03z); on one stream their times add up.
struct Fork {
    static constexpr int kSide = 3;
    hipStream_t st[kSide] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kSide] = {};
    bool forked[kSide] = {};
    bool marked = false;  // ev_fork recorded on the caller's stream for this batch
    hipStream_t caller = nullptr;

    Fork() = default;
    Fork(const Fork&) = delete;
    Fork& operator=(const Fork&) = delete;
    ~Fork() {
        for (int i = 0; i < kSide; ++i) {
            if (st[i]) {
                (void)hipStreamSynchronize(st[i]);
                (void)hipStreamDestroy(st[i]);
            }
            if (ev_join[i]) (void)hipEventDestroy(ev_join[i]);
        }
        if (ev_fork) (void)hipEventDestroy(ev_fork);
    }
    int begin(hipStream_t s) {
        if (!ev_fork) {
            FEC_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
            for (int i = 0; i < kSide; ++i)
                if (hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking) != hipSuccess ||
                    hipEventCreateWithFlags(&ev_join[i], hipEventDisableTiming) != hipSuccess)
                    return FEC_ERR_HIP;
        }
        caller = s;
        for (bool& f : forked) f = false;
        marked = false;
        return FEC_OK;
    }
    // the fork point: recorded on the caller's stream at the first side stream's use (a batch
    // without side work records nothing), or here, ahead of later caller-stream launches the side
    // work must not wait for
    int mark() {
        if (marked) return FEC_OK;
        marked = true;
        return hipEventRecord(ev_fork, caller) == hipSuccess ? FEC_OK : FEC_ERR_HIP;
    }
    // launch slot i: 0 = the caller's stream, i > 0 = side stream (i - 1) % kSide
    int stream(int i, hipStream_t* out) {
        if (i <= 0) {
            *out = caller;
            return FEC_OK;
        }
        const int j = (i - 1) % kSide;
        if (int st = mark()) return st;
        if (!forked[j]) {
            FEC_HIP(hipStreamWaitEvent(st[j], ev_fork, 0));
            forked[j] = true;
        }
        *out = st[j];
        return FEC_OK;
    }
    int join() {
        for (int j = 0; j < kSide; ++j) {
            if (!forked[j]) continue;
            if (hipEventRecord(ev_join[j], st[j]) != hipSuccess || hipStreamWaitEvent(caller, ev_join[j], 0) != hipSuccess)
                return FEC_ERR_HIP;
            forked[j] = false;
        }
        return FEC_OK;
    }
};
// Joins a begun fork on every exit path: work queued on the side streams is ordered before the
// caller's later work even when a launch fails half way (the error is still returned).
struct ForkScope {
    Fork& f;
    bool joined = false;
    explicit ForkScope(Fork& fk) : f(fk) {}
    ForkScope(const ForkScope&) = delete;
    ForkScope& operator=(const ForkScope&) = delete;
    int join() {
        joined = true;
        return f.join();
    }
    ~ForkScope() {
        if (!joined) (void)f.join();
    }
};
}  // namespace

struct fec_vr_plan {
    fec::VrPlan plan;
    int cw_max = 0;
    // ---- compact row layout (fec_vr.h), per run: per encoder instance first, cur end, end, CWp,
    // base_cur, base_old; totals; the device per-row offsets ----
    std::vector<int64_t> layout;
    int64_t cur_bytes = 0, old_bytes = 0;
    Upload off_up;
    void* d_rowoff = nullptr;              // cur_off [sent+1] | old_off [sent+1]
    size_t d_rowoff_cap = 0;
    bool rowoff_ready = false;
    // ---- device tables, rebuilt per run ----
    Upload enc_up, dec_up, hdr_up;
    void* d_pk = nullptr;                  // per-packet decoder id, fate, slow flag [P] each
    size_t d_pk_cap = 0;
    hipEvent_t pk_sent = nullptr;          // the per-packet copies out of the plan's arrays
    const int32_t* d_enc_inst = nullptr;   // [nenc][4]: k, n, CW, glog offset
    const int64_t* d_enc_span = nullptr;   // [nenc][2]: first, role_switch
    const int64_t* d_enc_cum = nullptr;    // [nenc+1]
    const uint32_t* d_gtab = nullptr;
    const int32_t* d_pk_dec = nullptr;
    const int32_t* d_inst = nullptr;
    const int64_t* d_inst_switch = nullptr;
    const uint8_t* d_fate = nullptr;
    const uint8_t* d_slow = nullptr;
    uint32_t* d_geo = nullptr;
    uint32_t* d_tdesc = nullptr;
    const int64_t* d_rec_x = nullptr;
    const int32_t* d_rec_dec = nullptr;
    const uint8_t* d_rec_coef = nullptr;
    const uint8_t* d_gf = nullptr;
    const int32_t* d_hdr = nullptr;    // [sent][4]: frame header T, B, N, counter
    int64_t enc_total = 0;             // codewords of all encoder instances
    int enc_tab = 0, enc_out = 0, enc_slot = 0, enc_wave = 0;  // fec_vr_encode_kernel's LDS layout
    int enc_nmax = 1;
    // the same instances without the ones the tile encoder takes (tuples with a tile geometry)
    const int32_t* d_lo_inst = nullptr;
    const int64_t* d_lo_span = nullptr;
    const int64_t* d_lo_cum = nullptr;
    const int64_t* d_enc_base = nullptr;   // [nenc][2]: byte offsets of the first cur / old row
    const int64_t* d_lo_base = nullptr;
    int n_lo = 0;
    int64_t lo_total = 0;
    // per tuple with a tile geometry: one launch of fec_encode_tile_kernel<k, n-k> in segment mode
    struct TileTuple {
        const void* kfn;
        fec::TileGeom tg;
        int toff;        // dword offset of its gf_mul4 tables in gtab
        size_t seg0;     // its first segment in d_seg
        int nseg;
        int k, np;
        bool multi;      // served by the one multi-tuple launch (fec_encode_tile_multi_kernel)
    };
    std::vector<TileTuple> tiles;  // the multi-tuple launch's first (heaviest first), then the others
    int n_multi = 0;               // tiles[0, n_multi): one launch, workgroup b = segment b of d_seg
    int multi_lds = 0, multi_lds_len = 0;
    const int64_t* d_seg = nullptr;
    const int64_t* d_np0 = nullptr;  // [n_np0][8]: segments of the instances of tuples with n = k
    int n_np0 = 0;
    bool enc_ready = false, dec_ready = false, hdr_ready = false;
    bool geo_ready = false;  // d_geo / d_tdesc written for this plan (they depend on the plan alone)
    hipEvent_t geo_done = nullptr;  // after that launch: every later copy's stream waits on it
    hipStream_t geo_stream = nullptr;  // the stream it ran on (its later copies need no wait)
    Fork fork;  // side streams (declared after the uploads: destroyed, and drained, first)

    ~fec_vr_plan() {
        if (geo_done) {
            (void)hipEventSynchronize(geo_done);
            (void)hipEventDestroy(geo_done);
        }
        if (pk_sent) {
            (void)hipEventSynchronize(pk_sent);
            (void)hipEventDestroy(pk_sent);
        }
        if (d_pk) {
            (void)hipEventSynchronize(dec_up.used);
            (void)hipFree(d_pk);
        }
        if (d_rowoff) {
            (void)hipEventSynchronize(off_up.used);
            (void)hipFree(d_rowoff);
        }
    }
    // (re)plans; the per-packet arrays are rewritten only once their last copy has left them
    void run(int max_payload, int T, int B, int N, bool mds, const uint8_t* erasure, int64_t n_erasure, int64_t P,
             bool async);
    void set_layout();  // the compact row layout of plan.enc (after run, or for a schedule set from outside)
};

namespace {
std::vector<uint8_t> gf_tables() {
    const fec::Field& F = fec::field();
    std::vector<uint8_t> gf(F.exp, F.exp + 512);
    gf.insert(gf.end(), F.log, F.log + 256);
    return gf;
}

int cw_of(const fec::VrPlan& p, const fec::VrInstance& v) { return fec::Geometry::make(p.L, v.T, v.B, v.N).CW; }

// Encode tables: per encoder instance its geometry, first call, role switch and the running
// count of codewords (every instance, and the ones the tile encoder does not take); per (T,B,N)
// tuple the gf_mul4 register tables of G's parity columns; per tuple with a tile geometry the
// segment list of its instances (units of at most `unit` tiles; each unit re-reads the tile in
// front of it as parity history).
int prepare_encode(fec_vr_plan* v, hipStream_t s) {
    if (v->enc_ready) return FEC_OK;
    const auto& p = v->plan;
    std::map<int, int> toff;  // tuple -> dword offset in gtab
    std::map<int, int> tix;   // tuple -> index in v->tiles (-1: no tile geometry)
    std::vector<uint32_t> gtab;
    std::vector<int32_t> inst, lo_inst;
    std::vector<int64_t> span, cum{0}, lo_span, lo_cum{0}, base, lo_base;
    std::vector<std::vector<int64_t>> segs;
    inst.reserve(p.enc.size() * 4);
    span.reserve(p.enc.size() * 2);
    cum.reserve(p.enc.size() + 1);
    v->tiles.clear();
    int unit = 4;
    if (const char* e = std::getenv("FEC_VR_TILE_UNIT")) unit = std::max(1, std::atoi(e));
    const bool tiles_on = !std::getenv("FEC_VR_NO_TILE");
    const bool multi_on = !std::getenv("FEC_VR_NO_MULTI");
    // (10,0,0)'s rows through fec_vr_encode_np0_kernel: opt-in.  Beside the multi-tuple launch
    // (FEC_VR_NP0=1) the two took longer (encode 0.144 vs 0.125 ms; the multi-tuple launch 109 vs
    // 105 us, profiles/r05/vr/r05zh_*); in front of it on the caller's stream (FEC_VR_NP0=2) the
    // multi-tuple launch shrinks to 70 us but np0 takes 27 - 37 us: encode 0.126 - 0.128 vs
    // 0.126 - 0.129 ms (r05zn), no gain.
    const char* np0e = std::getenv("FEC_VR_NP0");
    const bool np0_on = tiles_on && np0e && (np0e[0] == '1' || np0e[0] == '2');
    std::vector<int64_t> np0;
    int tab = 32, out = 16, slot = 16, nmax = 1;
    for (size_t ei = 0; ei < p.enc.size(); ++ei) {
        const auto& e = p.enc[ei];
        const fec::Geometry g = fec::Geometry::make(p.L, e.T, e.B, e.N);
        const int key = e.T * 1024 + e.B * 32 + e.N;
        const int64_t b_cur = v->layout[6 * ei + 4], b_old = v->layout[6 * ei + 5];
        const int64_t cwp = (g.CW + 15) & ~15;
        auto it = toff.find(key);
        if (it == toff.end()) {
            const std::vector<uint32_t> t = fec::parity_mul_tables(fec::make_generator(e.T, e.B, e.N), g.k, g.n);
            it = toff.emplace(key, static_cast<int>(gtab.size())).first;
            gtab.insert(gtab.end(), t.begin(), t.end());
            int ti = -1;
            const fec::TileGeom tg = fec::tile_geometry(g.k, g.n - g.k, p.L, true);
            const void* kfn = fec::fec_encode_tile_seg_kernel_for(g.k, g.n - g.k, p.L);
            if (tiles_on && tg.ok && kfn && (p.L & 3) == 0) {
                ti = static_cast<int>(v->tiles.size());
                v->tiles.push_back({kfn, tg, it->second, 0, 0, g.k, g.n - g.k, false});
                segs.emplace_back();
            }
            tix[key] = ti;
        }
        tab = std::max(tab, g.k * (g.n - g.k) * 32);
        out = std::max(out, (g.CW + 8 + 15) / 16 * 16);
        slot = std::max(slot, g.k * 4 * ((g.S + 3) / 4));
        nmax = std::max(nmax, g.n);
        inst.insert(inst.end(), {g.k, g.n, g.CW, it->second});
        span.insert(span.end(), {e.first, e.role_switch});
        base.insert(base.end(), {b_cur, b_old});
        cum.push_back(cum.back() + (e.end - e.first));
        int ti = tix[key];
        if (ti >= 0 && (e.end - e.first) * cwp >= 0x7fff0000) ti = -1;  // 32-bit buffer offsets
        if (np0_on && g.n == g.k && (p.L & 3) == 0 && cwp <= 512) {
            // no parity: fec_vr_encode_np0_kernel, segments of kVrNp0Rows rows
            const int64_t rows = e.end - e.first;
            for (int64_t t0 = 0; t0 < rows; t0 += fec::kVrNp0Rows) {
                const int64_t c = std::min<int64_t>(fec::kVrNp0Rows, rows - t0);
                np0.insert(np0.end(), {e.first, e.role_switch, rows, t0 | (c << 32), b_cur, b_old,
                                       static_cast<int64_t>(g.CW) | (cwp << 32), 0});
            }
        } else if (ti >= 0) {
            const int64_t rows = e.end - e.first, R = v->tiles[static_cast<size_t>(ti)].tg.R;
            const int64_t nt = (rows + R - 1) / R;
            for (int64_t t0 = 0; t0 < nt; t0 += unit) {
                const int64_t c = std::min<int64_t>(unit, nt - t0);
                segs[static_cast<size_t>(ti)].insert(segs[static_cast<size_t>(ti)].end(),
                                                     {e.first, e.role_switch, rows, t0 | (c << 32), b_cur, b_old});
            }
        } else {
            lo_inst.insert(lo_inst.end(), {g.k, g.n, g.CW, it->second});
            lo_span.insert(lo_span.end(), {e.first, e.role_switch});
            lo_base.insert(lo_base.end(), {b_cur, b_old});
            lo_cum.push_back(lo_cum.back() + (e.end - e.first));
        }
    }
    // order: the tuples of the multi-tuple launch first, heaviest walk (k * (n-k)) first so that its
    // workgroups start first; then the others by segment count, largest first
    for (size_t i = 0; i < v->tiles.size(); ++i) {
        auto& t = v->tiles[i];
        t.nseg = static_cast<int>(segs[i].size() / 6);
        t.multi = multi_on && fec::fec_encode_tile_multi_supports(t.k, t.np, p.L);
    }
    std::vector<size_t> order(v->tiles.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
        const auto &a = v->tiles[x], &b = v->tiles[y];
        if (a.multi != b.multi) return a.multi;
        return a.multi ? a.k * a.np > b.k * b.np : a.nseg > b.nseg;
    });
    std::vector<int64_t> seg;
    std::vector<fec_vr_plan::TileTuple> sorted;
    v->n_multi = 0;
    v->multi_lds = v->multi_lds_len = 0;
    for (size_t i : order) {
        auto t = v->tiles[i];
        t.seg0 = seg.size() / 6;
        seg.insert(seg.end(), segs[i].begin(), segs[i].end());
        if (t.multi && v->n_multi < fec::kEncMultiMax) {
            ++v->n_multi;
            v->multi_lds = std::max(v->multi_lds, t.tg.lds);
            v->multi_lds_len = std::max(v->multi_lds_len, t.tg.lds_len);
        } else {
            t.multi = false;
        }
        sorted.push_back(t);
    }
    v->tiles.swap(sorted);
    Upload& u = v->enc_up;
    if (int st = u.begin()) return st;
    u.add(&v->d_enc_inst, inst);
    u.add(&v->d_enc_span, span);
    u.add(&v->d_enc_cum, cum);
    u.add(&v->d_gtab, gtab);
    u.add(&v->d_lo_inst, lo_inst);
    u.add(&v->d_lo_span, lo_span);
    u.add(&v->d_lo_cum, lo_cum);
    u.add(&v->d_enc_base, base);
    u.add(&v->d_lo_base, lo_base);
    u.add(&v->d_seg, seg);
    u.add(&v->d_np0, np0);
    if (int st = u.commit(s)) return st;
    v->enc_total = cum.back();
    v->n_np0 = static_cast<int>(np0.size() / 8);
    v->n_lo = static_cast<int>(lo_span.size() / 2);
    v->lo_total = lo_cum.back();
    v->enc_tab = tab;
    v->enc_out = out;
    v->enc_slot = slot;
    v->enc_wave = tab + out + nmax * slot;
    v->enc_nmax = nmax;
    v->enc_ready = true;
    return FEC_OK;
}

// The instances of one tuple through the tile encoder, one workgroup per segment.
int launch_tile_tuple(const fec_vr_plan* v, const fec_vr_plan::TileTuple& tt, const uint8_t* d_payload,
                      const int32_t* d_len, uint8_t* d_cw_cur, int32_t* d_len_cur, uint8_t* d_cw_old,
                      int32_t* d_len_old, hipStream_t s) {
    if (tt.nseg <= 0) return FEC_OK;
    static std::mutex mu;
    static std::set<const void*> ready;  // kernels whose dynamic LDS limit is raised
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!ready.count(tt.kfn)) {
            if (hipFuncSetAttribute(tt.kfn, hipFuncAttributeMaxDynamicSharedMemorySize, tt.tg.lds_len) != hipSuccess)
                return FEC_ERR_HIP;
            ready.insert(tt.kfn);
        }
    }
    const fec::TileGeom& tg = tt.tg;
    fec::EncTileArgs a{};
    a.payload_base = d_payload;
    a.len_base = d_len;
    a.payload_bytes = 0;
    a.len_bytes = 0;
    a.history = 0;
    a.P = 0;
    a.cw = nullptr;
    a.cw_bytes = 0;
    a.cw_len = nullptr;
    a.ptab = v->d_gtab + tt.toff;
    a.L = v->plan.L;
    a.CW = tg.CW;
    a.NS4 = tg.NS4;
    a.PPW = tg.PPW;
    a.rem = tg.rem;
    a.nvl = tg.nvl;
    a.tiles_per_wg = 0;
    a.ntiles = 0;
    a.ngl = tg.ngl;
    a.nso = tg.nso;
    a.off_in = tg.off_in;
    a.in_bytes = tg.in_bytes;
    a.off_pw = tg.off_pw;
    a.off_q = tg.off_q;
    a.off_out = tg.off_out;
    a.off_len = tg.off_len;
    a.off_scratch = tg.off_scratch;
    a.dbg = 0;
    a.nt = 0;
    a.seg = v->d_seg + 6 * tt.seg0;
    a.cur_rows = d_cw_cur;
    a.old_rows = d_cw_old;
    a.cur_len = d_len_cur;
    a.old_len = d_len_old;
    a.W = (tg.CW + 15) & ~15;  // the compact layout's row stride of this tuple
    void* args[] = {&a};
    if (hipLaunchKernel(tt.kfn, dim3(static_cast<unsigned>(tt.nseg)), dim3(256), args, d_len ? tg.lds_len : tg.lds, s) !=
        hipSuccess)
        return FEC_ERR_HIP;
    return FEC_OK;
}

// The tuples tiles[0, n_multi) in one launch of fec_encode_tile_multi_kernel: workgroup b serves
// segment b of d_seg.
int launch_tile_multi(const fec_vr_plan* v, const uint8_t* d_payload, const int32_t* d_len, uint8_t* d_cw_cur,
                      int32_t* d_len_cur, uint8_t* d_cw_old, int32_t* d_len_old, const fec::VrEncodeArgs* cf,
                      hipStream_t s) {
    const void* kfn = fec::fec_encode_tile_multi_kernel_ptr();
    int lds = d_len ? v->multi_lds_len : v->multi_lds;
    if (cf) lds = std::max(lds, static_cast<int>(fec::vr_encode_cf_lds(*cf)));
    {
        static std::mutex mu;
        static int raised = 0;
        std::lock_guard<std::mutex> lk(mu);
        if (lds > raised) {
            if (hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
                return FEC_ERR_HIP;
            raised = lds;
        }
    }
    fec::EncMultiArgs m{};
    m.payload = d_payload;
    m.len = d_len;
    m.gtab = v->d_gtab;
    m.seg = v->d_seg;
    m.cur_rows = d_cw_cur;
    m.old_rows = d_cw_old;
    m.cur_len = d_len_cur;
    m.old_len = d_len_old;
    m.L = v->plan.L;
    m.ntuple = v->n_multi;
    m.nt = 0;  // (A/B switch FEC_VR_TILE_NT, as the one-stream encoder's FEC_TILE_NT)
    if (const char* e = std::getenv("FEC_VR_TILE_NT")) m.nt = std::atoi(e) & 2;
    // an instance's first tile without the zero history tile in front of it (FEC_VR_HIST0=1: with)
    if (const char* e = std::getenv("FEC_VR_HIST0")) m.nt |= std::atoi(e) ? 4 : 0;
    int nwg = 0;
    for (int i = 0; i < v->n_multi; ++i) {
        const auto& t = v->tiles[static_cast<size_t>(i)];
        if (static_cast<int>(t.seg0) != nwg) return FEC_ERR_ARG;  // segments in launch order
        m.tkey[i] = t.k * 32 + t.np;
        m.tfirst[i] = nwg;
        m.toff[i] = t.toff;
        nwg += t.nseg;
    }
    m.tfirst[v->n_multi] = nwg;
    fec::VrEncodeArgs cfa{};
    if (cf) {
        cfa = *cf;
        m.ncf = static_cast<int>(std::min<int64_t>(cf->cum_host_total, 16384));
        const char* e = std::getenv("FEC_VR_CF_FIRST");
        m.cf_first = e && e[0] == '1';
    }
    if (nwg + m.ncf <= 0) return FEC_OK;
    void* args[] = {&m, &cfa};
    return hipLaunchKernel(kfn, dim3(static_cast<unsigned>(nwg + m.ncf)), dim3(256), args, static_cast<size_t>(lds), s) ==
                   hipSuccess
               ? FEC_OK
               : FEC_ERR_HIP;
}

int prepare_decode(fec_vr_plan* v, hipStream_t s) {
    if (v->dec_ready) return FEC_OK;
    const auto& p = v->plan;
    std::vector<int32_t> inst;
    std::vector<int64_t> sw;
    inst.reserve(p.dec.size() * 4);
    sw.reserve(p.dec.size());
    for (const auto& d : p.dec) {
        const fec::Geometry g = fec::Geometry::make(p.L, d.T, d.B, d.N);
        inst.insert(inst.end(), {g.k, g.n, g.CW, 0});
        sw.push_back(d.role_switch);
    }
    Upload& u = v->dec_up;
    if (int st = u.begin()) return st;
    u.add(&v->d_inst, inst);
    u.add(&v->d_inst_switch, sw);
    u.add(&v->d_rec_x, p.rec_x);
    u.add(&v->d_rec_dec, p.rec_dec);
    u.add(&v->d_rec_coef, p.rec_coef);
    static const std::vector<uint8_t> gf = gf_tables();
    u.add(&v->d_gf, gf);
    if (int st = u.commit(s)) return st;
    // the per-packet arrays go straight from the plan's (page-locked) buffers
    const size_t P = static_cast<size_t>(p.P);
    const size_t o_fate = (P * 4 + 255) & ~size_t(255), o_slow = (o_fate + P + 255) & ~size_t(255);
    const size_t o_geo = (o_slow + P + 255) & ~size_t(255);  // device scratch of the copy
    const size_t o_desc = (o_geo + 4 * P + 255) & ~size_t(255);
    if (int st = Upload::reserve(&v->d_pk, &v->d_pk_cap, o_desc + 32 * ((P + 31) / 32 + 1), u.used, s)) return st;
    uint8_t* d = static_cast<uint8_t*>(v->d_pk);
    if (hipMemcpyAsync(d, p.fate_dec.data(), P * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d + o_fate, p.fate.data(), P, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d + o_slow, p.slow.data(), P, hipMemcpyHostToDevice, s) != hipSuccess)
        return FEC_ERR_HIP;
    if (!v->pk_sent) FEC_HIP(hipEventCreateWithFlags(&v->pk_sent, hipEventDisableTiming));
    FEC_HIP(hipEventRecord(v->pk_sent, s));
    v->d_pk_dec = reinterpret_cast<const int32_t*>(d);
    v->d_fate = d + o_fate;
    v->d_slow = d + o_slow;
    v->d_geo = reinterpret_cast<uint32_t*>(d + o_geo);
    v->d_tdesc = reinterpret_cast<uint32_t*>(d + o_desc);
    v->dec_ready = true;
    return FEC_OK;
}

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
}  // namespace

void fec_vr_plan::run(int max_payload, int T, int B, int N, bool mds, const uint8_t* erasure, int64_t n_erasure,
                      int64_t P, bool async) {
    if (pk_sent) (void)hipEventSynchronize(pk_sent);
    plan.run(max_payload, T, B, N, mds, erasure, n_erasure, P, async);
    set_layout();
}

void fec_vr_plan::set_layout() {
    cw_max = 0;
    for (const auto& e : plan.enc) cw_max = std::max(cw_max, cw_of(plan, e));
    for (const auto& d : plan.dec) cw_max = std::max(cw_max, cw_of(plan, d));
    cw_max = (cw_max + 15) & ~15;  // the widest row (wire packets' stride)
    // the compact layout: per encoder instance (creation order = seq order) its cur rows
    // [first, role_switch) and old rows [role_switch, end), each CW rounded to 16 bytes
    layout.assign(plan.enc.size() * 6, 0);
    cur_bytes = old_bytes = 0;
    for (size_t i = 0; i < plan.enc.size(); ++i) {
        const auto& e = plan.enc[i];
        const int64_t cwp = (cw_of(plan, e) + 15) & ~15;
        const int64_t cend = std::min(e.role_switch < 0 ? e.end : e.role_switch, e.end);
        if (i > 0 && e.first != std::min(plan.enc[i - 1].role_switch, plan.enc[i - 1].end))
            throw std::logic_error("encoder instances do not tile the frames");
        int64_t* l = &layout[6 * i];
        l[0] = e.first;
        l[1] = cend;
        l[2] = e.end;
        l[3] = cwp;
        l[4] = cur_bytes;
        l[5] = old_bytes;
        cur_bytes += (cend - e.first) * cwp;
        old_bytes += (e.end - cend) * cwp;
    }
    enc_ready = dec_ready = hdr_ready = rowoff_ready = geo_ready = false;
}

namespace {
// The device per-row offsets of the compact layout (fec_vr_offsets_kernel), once per run.
int ensure_rowoff(fec_vr_plan* v, hipStream_t s) {
    if (v->rowoff_ready) return FEC_OK;
    const int64_t rows = v->plan.sent;
    Upload& u = v->off_up;
    if (int st = u.begin()) return st;
    const int64_t* d_inst = nullptr;
    u.add(&d_inst, v->layout);
    if (int st = u.commit(s)) return st;
    if (int st = Upload::reserve(&v->d_rowoff, &v->d_rowoff_cap, 2 * sizeof(int64_t) * (rows + 1), u.used, s))
        return st;
    fec::VrOffsetsArgs a{d_inst, static_cast<int>(v->plan.enc.size()), rows, v->cur_bytes, v->old_bytes,
                         static_cast<int64_t*>(v->d_rowoff), static_cast<int64_t*>(v->d_rowoff) + rows + 1};
    if (int st = fec::vr_launch_offsets(a, s)) return st;
    if (int st = u.done_reading(s)) return st;
    v->rowoff_ready = true;
    return FEC_OK;
}
const int64_t* cur_off(const fec_vr_plan* v) { return static_cast<const int64_t*>(v->d_rowoff); }
const int64_t* old_off(const fec_vr_plan* v) { return static_cast<const int64_t*>(v->d_rowoff) + v->plan.sent + 1; }
}  // namespace

namespace fec {
// An encoder schedule built outside VrPlan's P2P loop (the two-hop session, fec_session.hip): its
// instances go through the same batched encoder and compact layout.
int vr_plan_from_instances(int max_payload, const std::vector<VrInstance>& enc, int64_t sent, fec_vr_plan** out) {
    if (!out || enc.empty() || sent < 1) return FEC_ERR_ARG;
    *out = nullptr;
    return vr_guarded([&] {
        std::unique_ptr<fec_vr_plan> v(new fec_vr_plan());
        v->plan.L = max_payload;
        v->plan.enc = enc;
        v->plan.sent = sent;
        v->plan.P = sent;
        v->set_layout();
        *out = v.release();
        return FEC_OK;
    });
}
// The device per-row offsets of the compact layout ([sent+1] each), built on first use on `s`.
int vr_plan_device_offsets(fec_vr_plan* v, void* s, const int64_t** cur_offs, const int64_t** old_offs) {
    if (!v) return FEC_ERR_ARG;
    if (int st = vr_guarded([&] { return ensure_rowoff(v, static_cast<hipStream_t>(s)); })) return st;
    *cur_offs = cur_off(v);
    *old_offs = old_off(v);
    return FEC_OK;
}
}  // namespace fec

extern "C" {

int fec_vr_plan_create(int max_payload, int T, int B, int N, int adaptive_mode_MDS, const uint8_t* erasure,
                       int64_t n_erasure, int64_t P, fec_vr_plan** out) {
    if (!out || P < 1 || n_erasure < 0 || (n_erasure > 0 && !erasure) || T < 1 || T > 11) return FEC_ERR_ARG;
    *out = nullptr;
    return vr_guarded([&] {
        std::unique_ptr<fec_vr_plan> v(new fec_vr_plan());
        v->run(max_payload, T, B, N, adaptive_mode_MDS != 0, erasure, n_erasure, P, false);
        *out = v.release();
        return FEC_OK;
    });
}

int fec_vr_plan_rerun(fec_vr_plan* v, const uint8_t* erasure, int64_t n_erasure, int64_t P, int async) {
    if (!v || P < 1 || n_erasure < 0 || (n_erasure > 0 && !erasure)) return FEC_ERR_ARG;
    return vr_guarded([&] {
        const fec::VrPlan& p = v->plan;
        v->run(p.L, p.T_init, p.B_init, p.N_init, p.adaptive_mode_MDS, erasure, n_erasure, P, async != 0);
        return FEC_OK;
    });
}

int fec_vr_plan_destroy(fec_vr_plan* v) {
    delete v;
    return FEC_OK;
}

int fec_vr_plan_stats(const fec_vr_plan* vc, int64_t* lost, int64_t* switches, double* coding_rate,
                      int64_t* sent, int* n_encoders, int* n_decoders, int* cw_max) {
    if (!vc) return FEC_ERR_ARG;
    fec_vr_plan* v = const_cast<fec_vr_plan*>(vc);
    if (lost || coding_rate) v->plan.finish();  // the rest is final after the control loop
    if (lost) *lost = v->plan.lost;
    if (switches) *switches = v->plan.switches;
    if (coding_rate) *coding_rate = v->plan.coding_rate();
    if (sent) *sent = v->plan.sent;
    if (n_encoders) *n_encoders = static_cast<int>(v->plan.enc.size());
    if (n_decoders) *n_decoders = static_cast<int>(v->plan.dec.size());
    if (cw_max) *cw_max = v->cw_max;
    return FEC_OK;
}

int fec_vr_plan_timing(const fec_vr_plan* vc, double* control_ms, double* decoders_ms) {
    if (!vc) return FEC_ERR_ARG;
    fec_vr_plan* v = const_cast<fec_vr_plan*>(vc);
    v->plan.finish();
    if (control_ms) *control_ms = v->plan.control_ms;
    if (decoders_ms) *decoders_ms = v->plan.decoders_ms;
    return FEC_OK;
}

int fec_vr_plan_feedback_wait(const fec_vr_plan* v, double* waited_ms) {
    if (!v || !waited_ms) return FEC_ERR_ARG;
    *waited_ms = v->plan.fb_wait_ms;
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

int fec_vr_plan_packets(const fec_vr_plan* vc, int32_t* frames, uint8_t* erased, uint8_t* fate,
                        int32_t* fate_decoder) {
    if (!vc) return FEC_ERR_ARG;
    fec_vr_plan* v = const_cast<fec_vr_plan*>(vc);
    v->plan.finish();
    const auto& p = v->plan;
    if (frames) {
        for (size_t r = 0; r < p.frame_runs.size(); ++r) {
            const int64_t hi = r + 1 < p.frame_runs.size() ? p.frame_runs[r + 1].first : p.sent;
            const fec::VrFrame& f = p.frame_runs[r].f;
            const int32_t cstep = p.frame_runs[r].cstep;
            for (int64_t s = p.frame_runs[r].first; s < hi; ++s) {
                int32_t* o = frames + 6 * s;
                o[0] = f.T;
                o[1] = f.B;
                o[2] = f.N;
                o[3] = f.counter + cstep * static_cast<int32_t>(s - p.frame_runs[r].first);
                o[4] = f.enc_cur;
                o[5] = f.enc_old;
            }
        }
    }
    if (erased) std::memcpy(erased, p.erased.data(), p.erased.size());
    if (fate) std::memcpy(fate, p.fate.data(), p.fate.size());
    if (fate_decoder) std::memcpy(fate_decoder, p.fate_dec.data(), p.fate_dec.size() * 4);
    return FEC_OK;
}

// Encode every packet the sender produced: row s of d_cw_cur (stride cw_max) = the codeword of
// frame s's current encoder, row s of d_cw_old = its old encoder's (double coding; rows of frames
// without one are left alone), trimmed sizes in d_len_*.  One launch for every instance of every
// (T,B,N) tuple (fec_vr_encode_kernel), straight from the payload rows.  Needs only the control
// loop's results: after an asynchronous fec_vr_plan_rerun it overlaps the symbolic decoders.
int fec_vr_encode_batch(fec_vr_plan* v, const uint8_t* d_payload, const int32_t* d_payload_len, uint8_t* d_cw_cur,
                        int32_t* d_len_cur, uint8_t* d_cw_old, int32_t* d_len_old, void* hip_stream) {
    if (!v || !d_payload || !d_cw_cur || !d_len_cur || !d_cw_old || !d_len_old) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (int st = vr_guarded([&] { return prepare_encode(v, s); })) return st;
    // the tile encoder writes 16-byte chunks of rows at stride cw_max (a multiple of 16)
    auto al = [](const void* q, uintptr_t m) { return (reinterpret_cast<uintptr_t>(q) & m) == 0; };
    const bool tiled = !v->tiles.empty() && al(d_cw_cur, 15) && al(d_cw_old, 15) &&
                       al(d_payload, 3) && al(d_len_cur, 3) && al(d_len_old, 3);
    // The tuples of the multi-tuple launch in one launch on the caller's stream; the generic encoder
    // (a latency-bound walk over the few tuples without a tile geometry) and any other tuple on side
    // streams, forked and joined with events (one stream with hipExtAnyOrderLaunch does not overlap
    // launches on gfx950).
    const int n_multi = tiled ? v->n_multi : 0;
    const int n_side_tiles = tiled ? static_cast<int>(v->tiles.size()) - n_multi : 0;
    const bool gen = !tiled || v->n_lo > 0;
    if (int st = v->fork.begin(s)) return st;
    ForkScope scope(v->fork);
    if (n_side_tiles > 0)  // (their launches follow the multi-tuple launch on the caller's stream)
        if (int st = v->fork.mark()) return st;
    int next_side = n_multi > 0 ? 1 : 0;  // stream index 0 = the caller's
    // the closed-form leftovers after the multi-tuple launch on the caller's stream (beside it on a
    // side stream they took its CUs: encode 0.128 - 0.129 vs 0.126 ms, profiles/r05/vr/r05zzc_*;
    // FEC_VR_GEN_AFTER=0 puts them beside it)
    const char* ga = std::getenv("FEC_VR_GEN_AFTER");
    const bool gen_after = gen && tiled && n_multi > 0 && !(ga && ga[0] == '0');
    if (gen && !gen_after) {
        hipStream_t sg;
        if (int st = v->fork.stream(next_side++, &sg)) return st;
        fec::VrEncodeArgs a{d_payload, d_payload_len, v->plan.L,
                            tiled ? v->d_lo_inst : v->d_enc_inst, tiled ? v->d_lo_span : v->d_enc_span,
                            tiled ? v->d_lo_cum : v->d_enc_cum,
                            tiled ? v->n_lo : static_cast<int>(v->plan.enc.size()), tiled ? v->lo_total : v->enc_total,
                            v->enc_tab, v->enc_out, v->enc_slot, v->enc_wave, v->d_gtab,
                            tiled ? v->d_lo_base : v->d_enc_base, d_cw_cur, d_cw_old, d_len_cur, d_len_old,
                            v->enc_nmax};
        // the tile encoder's leftovers in closed form (FEC_VR_LO_CF=0: the ring walk)
        const char* cf = std::getenv("FEC_VR_LO_CF");
        const bool use_cf = tiled && !(cf && cf[0] == '0');
        if (int st = use_cf ? fec::vr_launch_encode_cf(a, sg) : fec::vr_launch_encode(a, sg)) return st;
    }
    if (tiled && v->n_np0 > 0) {
        hipStream_t s0 = s;  // FEC_VR_NP0=2: in front of the multi-tuple launch on the caller's stream
        const char* np0e = std::getenv("FEC_VR_NP0");
        if (!(np0e && np0e[0] == '2'))
            if (int st = v->fork.stream(next_side++, &s0)) return st;
        fec::VrNp0Args a0{d_payload, d_payload_len, v->plan.L, v->d_np0, v->n_np0, d_cw_cur, d_cw_old, d_len_cur, d_len_old};
        if (int st = fec::vr_launch_encode_np0(a0, s0)) return st;
    }
    fec::VrEncodeArgs lo{d_payload, d_payload_len, v->plan.L, v->d_lo_inst, v->d_lo_span, v->d_lo_cum, v->n_lo,
                         v->lo_total, v->enc_tab, v->enc_out, v->enc_slot, v->enc_wave, v->d_gtab, v->d_lo_base,
                         d_cw_cur, d_cw_old, d_len_cur, d_len_old, v->enc_nmax};
    // the closed-form leftovers inside the multi-tuple launch, in the workgroups after its segments'
    // (FEC_VR_CF_FUSE=0: their own launch after it on the caller's stream)
    const char* cfu = std::getenv("FEC_VR_CF_FUSE");
    const bool cf_fuse = gen_after && !(cfu && cfu[0] == '0') && v->n_lo > 0 && v->lo_total > 0 &&
                         fec::vr_encode_cf_lds(lo) <= 65536;
    if (n_multi > 0)
        if (int st = launch_tile_multi(v, d_payload, d_payload_len, d_cw_cur, d_len_cur, d_cw_old, d_len_old,
                                       cf_fuse ? &lo : nullptr, s))
            return st;
    if (gen_after && !cf_fuse)
        if (int st = fec::vr_launch_encode_cf(lo, s)) return st;
    for (int i = 0; i < n_side_tiles; ++i) {
        hipStream_t st_i;
        if (int st = v->fork.stream(next_side++, &st_i)) return st;  // side streams round robin
        if (int st = launch_tile_tuple(v, v->tiles[static_cast<size_t>(n_multi + i)], d_payload, d_payload_len,
                                       d_cw_cur, d_len_cur, d_cw_old, d_len_old, st_i))
            return st;
    }
    if (int st = scope.join()) return st;
    return v->enc_up.done_reading(s);
}

// The P2P wire packets of every frame: row s of d_packets (stride >= 10 + 2*cw_max bytes) =
// [seq BE32][T][B][N][counter_for_start_and_end] (Application_Layer_Sender.cpp:259-269) +
// [len_cur BE16][cur][old] (Variable_Rate_FEC_Encoder.cpp:194-217), sizes in d_packet_len.
int fec_vr_frames_batch(fec_vr_plan* v, const uint8_t* d_cw_cur, const int32_t* d_len_cur, const uint8_t* d_cw_old,
                        const int32_t* d_len_old, uint8_t* d_packets, int64_t stride, int32_t* d_packet_len,
                        void* hip_stream) {
    if (!v || !d_cw_cur || !d_len_cur || !d_cw_old || !d_len_old || !d_packets || !d_packet_len) return FEC_ERR_ARG;
    if (stride < 10 + 2 * static_cast<int64_t>(v->cw_max)) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const auto& p = v->plan;
    if (!v->hdr_ready) {
        int st = vr_guarded([&] {
            std::vector<int32_t> h(static_cast<size_t>(p.sent) * 4);
            for (size_t r = 0; r < p.frame_runs.size(); ++r) {
                const int64_t hi = r + 1 < p.frame_runs.size() ? p.frame_runs[r + 1].first : p.sent;
                const fec::VrFrame& f = p.frame_runs[r].f;
                const int32_t cstep = p.frame_runs[r].cstep;
                for (int64_t q = p.frame_runs[r].first; q < hi; ++q) {
                    h[4 * q] = f.T;
                    h[4 * q + 1] = f.B;
                    h[4 * q + 2] = f.N;
                    h[4 * q + 3] = f.counter + cstep * static_cast<int32_t>(q - p.frame_runs[r].first);
                }
            }
            Upload& u = v->hdr_up;
            if (int e = u.begin()) return e;
            u.add(&v->d_hdr, h);
            return u.commit(s);
        });
        if (st) return st;
        v->hdr_ready = true;
    }
    if (int st = ensure_rowoff(v, s)) return st;
    fec::VrFrameArgs a{d_cw_cur, d_len_cur, d_cw_old, d_len_old, cur_off(v), old_off(v), v->d_hdr, p.sent,
                       d_packets, stride, d_packet_len};
    if (int st = fec::vr_launch_frames(a, hip_stream)) return st;
    return v->hdr_up.done_reading(s);
}

// Decode the schedule from the frames' arrays: every packet x < P was reported by one decoder
// instance j (fate_decoder); a received one is the systematic part of cur[x] in j's geometry, a
// recovered one the host plan's coefficient rows over j's inputs (cur rows before j became the
// old decoder, old rows after).  Two launches.  d_erased is not read (the plan holds the pattern).
int fec_vr_decode_batch(fec_vr_plan* v, const uint8_t* d_cw_cur, const uint8_t* d_cw_old, const uint8_t* d_erased,
                        uint8_t* d_out, int32_t* d_out_len, void* hip_stream) {
    (void)d_erased;
    if (!v || !d_cw_cur || !d_cw_old || !d_out || !d_out_len) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (int st = vr_guarded([&] {
            v->plan.finish();
            return prepare_decode(v, s);
        }))
        return st;
    const auto& p = v->plan;
    if (int st = ensure_rowoff(v, s)) return st;
    fec::VrCopyArgs ca{d_cw_cur, cur_off(v), v->d_pk_dec, v->d_inst, v->d_fate, v->d_slow, p.P, p.L, d_out,
                       d_out_len, v->d_geo, v->d_tdesc, v->cur_bytes};
    fec::VrRecArgs ra{d_cw_cur, d_cw_old, cur_off(v), old_off(v), p.sent, v->d_rec_x, v->d_rec_dec, v->d_rec_coef,
                      static_cast<int>(p.rec_x.size()), v->d_inst, v->d_inst_switch, v->d_gf, p.L, d_out, d_out_len};
    // the recovery writes only the rows (and lengths) the copy leaves alone: one launch holding both
    // (FEC_VR_FUSED=0: the copy on the caller's stream, the recovery beside it on a side stream)
    if (!v->geo_ready) {
        if (!v->geo_done) FEC_HIP(hipEventCreateWithFlags(&v->geo_done, hipEventDisableTiming));
        if (int st = fec::vr_launch_geo(ca, hip_stream)) return st;
        FEC_HIP(hipEventRecord(v->geo_done, s));
        v->geo_ready = true;
        v->geo_stream = s;
    } else if (s != v->geo_stream && hipStreamWaitEvent(s, v->geo_done, 0) != hipSuccess) {  // a decode on another stream
        return FEC_ERR_HIP;
    }
    const char* fu = std::getenv("FEC_VR_FUSED");
    if (!(fu && fu[0] == '0')) {
        const int st = fec::vr_launch_decode(ca, ra, hip_stream);
        if (st == FEC_OK) return v->dec_up.done_reading(s);
        if (st != 1) return st;
    }
    if (int st = v->fork.begin(s)) return st;
    ForkScope scope(v->fork);
    hipStream_t sr;
    if (int st = v->fork.stream(p.rec_x.empty() ? 0 : 1, &sr)) return st;
    if (int st = fec::vr_launch_copy(ca, hip_stream)) return st;
    if (int st = fec::vr_launch_recover(ra, sr)) return st;
    if (int st = scope.join()) return st;
    return v->dec_up.done_reading(s);
}

int fec_vr_parse_batch(fec_vr_plan* v, const uint8_t* d_packets, int64_t stride, const int32_t* d_packet_len,
                       uint8_t* d_cw_cur, uint8_t* d_cw_old, int32_t* d_header, void* hip_stream) {
    if (!v || !d_packets || !d_packet_len || !d_cw_cur || !d_cw_old) return FEC_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (int st = vr_guarded([&] { return ensure_rowoff(v, s); })) return st;
    fec::VrParseArgs a{d_packets, stride, d_packet_len, v->plan.sent, cur_off(v), old_off(v), d_cw_cur, d_cw_old,
                       d_header};
    return fec::vr_launch_parse(a, hip_stream);
}

int fec_vr_plan_layout(const fec_vr_plan* v, int64_t* cur_bytes, int64_t* old_bytes) {
    if (!v) return FEC_ERR_ARG;
    if (cur_bytes) *cur_bytes = v->cur_bytes;
    if (old_bytes) *old_bytes = v->old_bytes;
    return FEC_OK;
}

int fec_vr_plan_row_offsets(const fec_vr_plan* v, int64_t* cur_off, int64_t* old_off) {
    if (!v) return FEC_ERR_ARG;
    const auto& L = v->layout;
    const int64_t rows = v->plan.sent;
    const size_t ne = L.size() / 6;
    size_t e = 0;
    for (int64_t s = 0; s < rows; ++s) {  // as fec_vr_offsets_kernel
        while (e + 1 < ne && L[6 * (e + 1)] <= s) ++e;
        const int64_t* me = &L[6 * e];
        if (cur_off) cur_off[s] = me[4] + (s - me[0]) * me[3];
        const int64_t* pv = e > 0 ? me - 6 : nullptr;
        if (old_off) old_off[s] = (pv && s >= pv[1] && s < pv[2]) ? pv[5] + (s - pv[1]) * pv[3] : me[5];
    }
    if (cur_off) cur_off[rows] = v->cur_bytes;
    if (old_off) old_off[rows] = v->old_bytes;
    return FEC_OK;
}

}  // extern "C"
