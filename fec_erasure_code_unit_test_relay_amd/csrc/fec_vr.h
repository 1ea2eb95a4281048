// fec_vr.h -- variable-rate (adaptive) coding: the control plane of BASELINE config 4.
//
// The reference's P2P loop (application_local_simulation.cpp:328-345, RELAYING_TYPE 0) chains
//   Application_Layer_Sender::generate_message_and_encode   (src/Application_Layer_Sender.cpp:64-282)
//     -> Variable_Rate_FEC_Encoder::encode                  (src/Variable_Rate_FEC_Encoder.cpp:74-235)
//   Application_Layer_Receiver::receive_message_and_decode  (src/Application_Layer_Receiver.cpp:321-468)
//     -> Parameter_Estimator::estimate x2 (foreground / background, swapped every
//        ESTIMATION_WINDOW_SIZE / ESTIMATION_WINDOW_SIZE_REDUCTION_FACTOR packets)
//     -> Variable_Rate_FEC_Decoder::decode                  (src/Variable_Rate_FEC_Decoder.cpp:2133-2400)
// with the receiver's 6-byte feedback [T, B_est, N_est, T_ack, B_ack, N_ack] read by the sender at
// the next packet.  Which (T,B,N) encodes which packet, when double coding starts and stops, which
// decoder instance reports which packet and whether it is lost depend only on the erasure
// pattern, never on payload bytes (recovered headers always carry max_payload here).  VrPlan runs
// that loop symbolically (StreamPlanner per decoder instance) and records the schedule: encoder
// and decoder instances with their sequence ranges, per-packet frame headers and the reported
// fate of every packet.  The byte work of the schedule then runs batched on the GPU
// (fec_vr_encode_batch / fec_vr_decode_batch in fec_vr.cpp): one launch pair per instance.
#pragma once

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <sched.h>
#include <thread>
#include <utility>
#include <vector>

#include "fec_host.h"

struct fec_vr_plan;  // the C ABI's plan handle (fec_vr.cpp)

namespace fec {

// Parameter_Estimator (src/Parameter_Estimator.cpp:21-223), RELAYING_TYPE 0.
struct ParameterEstimator {
    bool adaptive_mode_MDS = false;
    int T = 0, B = 0, N = 0, N_max = 0, B_current = 0, N_current = 0;
    uint32_t erasure = 0;  // bit i = the reference's erasure[i] (window of T+1 flags, newest at 0)
    int64_t previous_win_end = -2;
    ParameterEstimator(int T_value, bool mds) : adaptive_mode_MDS(mds), T(T_value) {}
    void estimate(int64_t seq, int msg_T);
    void make_MDS_estimates();
    // estimate(seq, T) for the next in-order seq would change nothing but previous_win_end: the
    // window holds no erasure (a received packet shifts in a 0: sum == 0 skips the update,
    // Parameter_Estimator.cpp:104-105) and the closing recommendation step is at its fixed point
    // (:177-181, and make_MDS_estimates when on).
    bool steady(int64_t seq, int msg_T) const {
        if (T == 0 || previous_win_end != seq - 1 || erasure != 0 || msg_T != T) return false;
        if ((T - N_current + 1) * (T - N + 1 + B) >= (T - N + 1) * (T - N_current + 1 + B_current) &&
            (B_current != B || N_current != N))
            return false;
        return !(adaptive_mode_MDS && B_current > N_current);
    }
};

constexpr int kVrCoefStride = kMaxK * kMaxRuleN;

struct VrInstance {
    int T = 0, B = 0, N = 0;
    int64_t first = 0;   // seq of its first call
    int64_t end = 0;     // one past the seq of its last call (calls are consecutive)
    int64_t role_switch = -1;  // seq from which it is the old instance (double coding); == end if never
};

struct VrFrame {  // Application_Layer_Sender header (Application_Layer_Sender.cpp:259-269) + VR frame
    int T = 0, B = 0, N = 0, counter = 0;
    int enc_cur = -1, enc_old = -1;  // encoder instances whose codewords the frame carries
    bool operator==(const VrFrame& o) const { return same_but_counter(o) && counter == o.counter; }
    bool same_but_counter(const VrFrame& o) const {
        return T == o.T && B == o.B && N == o.N && enc_cur == o.enc_cur && enc_old == o.enc_old;
    }
};

// Page-locked host memory (hipHostMalloc) when a GPU runtime is present, plain heap memory
// otherwise: the plan's per-packet arrays go to the device with asynchronous copies straight from
// where the plan wrote them, and stay allocated across re-runs of one plan.
void* vr_host_alloc(size_t bytes);
void vr_host_free(void* p);
template <typename T>
struct VrHostAlloc {
    using value_type = T;
    VrHostAlloc() = default;
    template <typename U>
    VrHostAlloc(const VrHostAlloc<U>&) {}
    T* allocate(size_t n) { return static_cast<T*>(vr_host_alloc(n * sizeof(T))); }
    void deallocate(T* p, size_t) { vr_host_free(p); }
    template <typename U>
    bool operator==(const VrHostAlloc<U>&) const { return true; }
    template <typename U>
    bool operator!=(const VrHostAlloc<U>&) const { return false; }
};
template <typename T>
using VrHostVec = std::vector<T, VrHostAlloc<T>>;

// s += r, `count` times, in float: the sequential loop's result in O(binades) steps (fec_vr.cpp).
float float_add_repeated(float s, float r, int64_t count);

struct VrPlan {
    struct FrameRun {      // frames[first .. next run's first): `f`, the counter + cstep per packet
        int64_t first;
        VrFrame f;
        int32_t cstep = 0;  // 1: a transition's frames, whose counter grows by one per packet
    };
    struct RateRun {       // `count` packets adding `rate` to final_sum_coding_rate, in order
        int64_t count;
        float rate;
    };
    struct Reports {       // decoder instance `id` reports packet seq - xoff at its calls for seq in [lo, hi)
        int32_t id;
        int64_t lo, hi, xoff;
    };

    int L = 0, T_init = 0, B_init = 0, N_init = 0;
    bool adaptive_mode_MDS = false;
    int64_t P = 0;                    // NUMBER_OF_ITERATIONS: packets whose output is counted
    int64_t sent = 0;                 // packets the sender produced (>= P + T)
    std::vector<uint8_t> erased;      // [sent]: dropped before the receiver (Application_Layer_Receiver.cpp:352-360)
    std::vector<int64_t> drops;       // the seqs with erased == 1, increasing
    std::vector<FrameRun> frame_runs; // frames of [0, sent), run-length coded
    std::vector<RateRun> rate_runs;
    std::vector<VrInstance> enc, dec;
    VrHostVec<uint8_t> fate;          // [P]: PacketFate of the output reported for packet x
    VrHostVec<int32_t> fate_dec;      // [P]: decoder instance that reported it
    VrHostVec<uint8_t> slow;          // [P]: reported by the block decoders (length clamped)
    // recovered packets: x, reporting decoder, its k x n coefficient rows (stride kVrCoefStride)
    std::vector<int64_t> rec_x;
    std::vector<int32_t> rec_dec;
    std::vector<uint8_t> rec_coef;
    int64_t lost = 0, switches = 0;   // "Start double coding at the source" count
    float sum_coding_rate = 0;        // Variable_Rate_FEC_Encoder final_sum_coding_rate
    int64_t steady_packets = 0;       // packets the control loop appended as steady stretches
    int64_t transition_packets = 0;   // ... and as transition stretches (double coding, no drop)
    double control_ms = 0, decoders_ms = 0;  // wall time of run()'s two phases
    double fb_wait_ms = 0;            // the control loop's time waiting for feedback jobs
    double coding_rate() const { return sent ? sum_coding_rate / static_cast<float>(sent) : 0.0; }

    VrPlan() = default;
    VrPlan(const VrPlan&) = delete;
    VrPlan& operator=(const VrPlan&) = delete;
    ~VrPlan();

    // Runs the loop until the receiver has processed seq P+T-1 (application_local_simulation.cpp:813).
    // B_init = N_init = -1: adaptive (the sender starts at (T, 0, 0)).  Re-running one plan reuses
    // its buffers.  async: return after the control loop (enc, dec, frames, erased, sent, switches
    // are final); the symbolic decoders (fate, slow, rec_*, lost, coding rate) run on worker
    // threads until finish().
    void run(int max_payload, int T, int B, int N, bool mds, const uint8_t* pattern, int64_t n_pattern,
             int64_t P_value, bool async = false);
    void finish();  // waits for the decoder phase of an async run (no-op otherwise)
    VrFrame frame(int64_t s) const;  // frame of sent packet s

private:
    struct DecJob {        // a decoder instance the control loop is done with (id -1: the rate sum, <= -2: feedback job -2-id)
        int id = -1;
        VrInstance d;
        const DecodeRules* rules = nullptr;
        std::vector<Reports> reps;
    };
    struct RecEntry {      // a recovered packet and its k x n coefficient rows
        int64_t x;
        std::array<uint8_t, kVrCoefStride> coef;
    };
    void control(const uint8_t* pattern, int64_t n_pattern, int T, int B, int N, bool mds);
    struct FbChange {      // the receiver's feedback (T | B_est << 8 | N_est << 16) from received seq on
        int64_t seq;
        uint32_t v;
    };
    struct FbJob {         // one estimator's stretch: fed from `from`, its feedback for [rec, to)
        int64_t from = 0, rec = 0, to = 0;
        std::vector<FbChange> changes;
    };
    struct FbCursor;
    void feedback_plan(int64_t end);
    void feedback_run(int T, bool mds);
    void feedback_job(int64_t j, int T, bool mds);
    std::vector<int64_t> fb_swaps_;
    std::vector<FbJob> fb_jobs_;
    std::unique_ptr<std::atomic<uint8_t>[]> fb_ready_;  // per job: complete (any order)
    int fb_T_ = 0;
    bool fb_mds_ = false;
    size_t fb_chunk_ = 1;  // feedback jobs per worker-pool run
    void start_workers();
    void publish(DecJob&& j, bool flush = false);
    // Decoder-instance jobs go to the workers without a lock: the control loop fills slot dpub_ of
    // a chunked array (slots never move) and releases it; a worker claims slot dtake_ by
    // compare-and-swap.  The mutex queue keeps the few other jobs (feedback runs, the rate sum).
    static constexpr int64_t kJobChunk = 256;
    std::vector<std::unique_ptr<DecJob[]>> djobs_;
    std::atomic<int64_t> dpub_{0}, dtake_{0};
    int64_t dfill_ = 0;  // slots filled by the control loop (released up to dpub_)
    DecJob& dslot(int64_t i) { return djobs_[static_cast<size_t>(i / kJobChunk)][i % kJobChunk]; }
    void publish_decoder(int id, const VrInstance& d, const DecodeRules* rules, std::vector<Reports>& reps,
                         bool flush = false);
    void close_jobs();
    void decode_instance(const DecJob& job, std::vector<RecEntry>& recs);
    std::map<int, std::shared_ptr<const DecodeRules>> rules_;  // key T*1024 + B*32 + N
    static constexpr int kRulesKeys = 64 * 1024;
    std::vector<const DecodeRules*> rules_fast_;               // the same, by key (filled on use)
    const DecodeRules& rules_for(int T, int B, int N);
    std::vector<std::vector<Reports>> reps_;                   // the control loop's per-instance lists
    std::vector<const DecodeRules*> drules_;
    // The worker pool lives as long as the plan: a run hands it a new epoch (one wake-up per
    // worker) instead of creating and joining threads (~0.1 ms per run on the control loop and as
    // much again at finish()); pool_active_ counts the workers still inside the current run.
    std::vector<std::thread> workers_;
    std::mutex pmu_;
    std::condition_variable pcv_, pdone_;
    uint64_t pool_epoch_ = 0;      // (pmu_) bumped by each run's start_workers
    int pool_active_ = 0;          // (pmu_) workers not yet done with the current epoch
    cpu_set_t pool_set_;           // (pmu_) the CPUs the workers of this epoch run on (the control
                                   // loop's group, taken in its context: a worker's own affinity is
                                   // the previous run's group)
    bool pool_quit_ = false;       // (pmu_) the destructor's
    void worker_run(size_t w);     // one epoch's jobs (until the queue is closed and drained)
    void stop_pool();
    std::vector<std::vector<RecEntry>> recs_;  // per worker
    std::mutex qmu_;
    std::condition_variable qcv_;
    std::deque<DecJob> q_;
    std::vector<DecJob> batch_;  // jobs not yet handed to the workers
    bool qclosed_ = false;
    // Workers poll these before sleeping on qcv_, and the control loop wakes the queue only when a
    // worker sleeps: a futex wake per published batch cost the control loop ~0.7 ms of system time
    std::atomic<int64_t> qsize_{0};  // q_.size() (written under qmu_)
    std::atomic<bool> qclosed_flag_{false};  // qclosed_, for the pollers
    std::atomic<int> sleepers_{0};   // workers waiting on qcv_ (changed under qmu_)
    std::chrono::steady_clock::time_point t_dec_;
    bool pending_ = false;
};

// Device side of the schedule (fec_vr_kernels.hip).  All launches go to `s`.
//
// Row layout of the frames' codeword arrays (compact): row s of `cur` holds the codeword of frame
// s's current encoder instance, row s of `old` the old instance's during double coding (no row
// otherwise).  Every row is its instance's CW rounded up to 16 bytes; the rows of one instance are
// consecutive at that stride, and instances follow each other in seq order, so both arrays are
// dense and a run of consecutive packets is one contiguous span.  Per instance e: cur rows
// [first_e, role_switch_e) from byte base_cur_e, old rows [role_switch_e, end_e) from base_old_e;
// per row: cur_off[s] / old_off[s] (sent + 1 entries each, prefix form: row s spans
// [off[s], off[s+1]), empty for a frame without an old codeword).
// Every encoder instance of the schedule in one launch (any mix of (T,B,N)): codeword c of the
// list = instance e's call for seq = first_e + (c - cum[e]), written to cur[seq] before e's
// role switch and to old[seq] after (Variable_Rate_FEC_Encoder.cpp:140-217).
struct VrEncodeArgs {
    const uint8_t* payload;   // [sent][L]
    const int32_t* len;       // may be null (all L)
    int L;
    const int32_t* inst;      // [nenc][4]: k, n, CW, offset (dwords) of the tuple's gf_mul4 tables
    const int64_t* span;      // [nenc][2]: first, role_switch
    const int64_t* cum;       // [nenc+1]: codewords of instances < e
    int nenc;
    int64_t cum_host_total;   // cum[nenc] (host copy: sizes the grid)
    int tab_bytes;            // per wave LDS: tables of the widest tuple (k*(n-k)*32)
    int out_bytes;            //   output row (max CW + 8, rounded to 16)
    int slot_bytes;           //   one ring slot (k planes of ceil(S/4) words, max over tuples)
    int wave_bytes;           //   tab + out + n_max * slot
    const uint32_t* gtab;     // per tuple [k][n-k][8]: gf_mul4 tables of G[i][k+jj] (+ non-zero flag)
    const int64_t* base;      // [nenc][2]: byte offsets of the instance's first cur row / first old row
    uint8_t* cur;
    uint8_t* old;
    int32_t* len_cur;
    int32_t* len_old;
    int n_max;                //   widest n over the instances (fec_vr_encode_cf_kernel's LDS rows)
};
// Encoder instances of tuples with n = k (no parity: the codeword is X itself, [len BE16, payload,
// zero pad] to S*k bytes): a workgroup per segment of at most kVrNp0Rows rows of one instance.
constexpr int kVrNp0Rows = 32;
struct VrNp0Args {
    const uint8_t* payload;   // [sent][L]
    const int32_t* len;       // may be null (all L)
    int L;
    const int64_t* seg;       // [nseg][8]: first seq, role switch, rows, t0 | cnt << 32, byte offsets of
                              //   the first cur / old row, CW | W << 32 (W = CW rounded to 16, <= 512), 0
    int nseg;
    uint8_t* cur;
    uint8_t* old;
    int32_t* len_cur;
    int32_t* len_old;
};
int vr_launch_encode_np0(const VrNp0Args& a, void* s);

struct VrCopyArgs {     // received packets: systematic bytes of cur[x] in its decoder's geometry
    const uint8_t* cur;
    const int64_t* cur_off;  // [sent+1]
    const int32_t* pk_dec;   // [P] reporting decoder
    const int32_t* inst;     // [ndec][4]: k, n, CW, 0
    const uint8_t* fate;     // [P]
    const uint8_t* slow;     // [P]
    int64_t P;
    int L;
    uint8_t* out;
    int32_t* out_len;
    uint32_t* geo;           // [P] scratch: k | n << 8 | fate << 16 | slow << 24 (fec_vr_geo_kernel)
    uint32_t* tdesc;         // [ceil(P/32)] scratch: the copy's tile descriptors (fec_vr_geo_kernel,
                             //   VrTileDesc in fec_vr_kernels.hip, 32 bytes each)
    int64_t cur_bytes;       // bytes of cur (reads past them return zero)
};
struct VrRecArgs {      // recovered packets: coefficient rows over the reporting decoder's inputs
    const uint8_t* cur;
    const uint8_t* old;
    const int64_t* cur_off;  // [sent+1]
    const int64_t* old_off;  // [sent+1]
    int64_t rows;            // sent packets (valid rows of cur / old)
    const int64_t* rec_x;
    const int32_t* rec_dec;
    const uint8_t* rec_coef; // stride kVrCoefStride
    int nrec;
    const int32_t* inst;
    const int64_t* inst_switch;  // [ndec]: rows >= it come from `old`
    const uint8_t* gf;
    int L;
    uint8_t* out;
    int32_t* out_len;
};
// P2P wire packets (Application_Layer_Sender.cpp:259-269 over Variable_Rate_FEC_Encoder.cpp:194-217):
// row s (stride bytes) = [seq BE32][T][B][N][counter][len_cur BE16][cur: len_cur][old: len_old].
struct VrFrameArgs {
    const uint8_t* cur;
    const int32_t* len_cur;
    const uint8_t* old;
    const int32_t* len_old;
    const int64_t* cur_off;  // [rows+1]
    const int64_t* old_off;  // [rows+1]
    const int32_t* hdr;      // [rows][4]: T, B, N, counter
    int64_t rows;
    uint8_t* packets;
    int64_t stride;
    int32_t* packet_len;
};
// The receiver's split of a wire packet (Application_Layer_Receiver.cpp:361-366,
// Variable_Rate_FEC_Decoder.cpp:2156-2160): cur / old rows zero-padded to their row size, header
// fields out.
struct VrParseArgs {
    const uint8_t* packets;
    int64_t stride;
    const int32_t* packet_len;
    int64_t rows;
    const int64_t* cur_off;  // [rows+1]
    const int64_t* old_off;  // [rows+1]
    uint8_t* cur;
    uint8_t* old;
    int32_t* hdr;            // [rows][5]: seq, T, B, N, counter (may be null)
};
// The per-row offsets from the encoder instances (one thread per instance: its cur rows, and the
// old rows of the instance before it, which are the same seqs).
struct VrOffsetsArgs {
    const int64_t* inst;     // [nenc][6]: first, role_switch (cur end), end, CW rounded to 16, base_cur, base_old
    int nenc;
    int64_t rows;            // sent
    int64_t cur_total, old_total;
    int64_t* cur_off;        // [rows+1]
    int64_t* old_off;        // [rows+1]
};
int vr_launch_offsets(const VrOffsetsArgs& a, void* s);
int vr_launch_frames(const VrFrameArgs& a, void* s);
int vr_launch_parse(const VrParseArgs& a, void* s);
int vr_launch_encode(const VrEncodeArgs& a, void* s);
// The same in closed form, a workgroup per codeword (no LDS ring; the instance list's few codewords
// beside the tile encoder)
int vr_launch_encode_cf(const VrEncodeArgs& a, void* s);
// The per-packet geometry words and tile descriptors of a plan (fec_vr_geo_kernel): once per plan,
// in front of its first copy.
int vr_launch_geo(const VrCopyArgs& a, void* s);
int vr_launch_copy(const VrCopyArgs& a, void* s);
int vr_launch_recover(const VrRecArgs& a, void* s);
// copy and recovery in one launch (fec_vr_decode_kernel); 1 = not applicable (no fast copy tiles,
// or nothing to recover): launch the two instead
int vr_launch_decode(const VrCopyArgs& a, const VrRecArgs& ra, void* s);
// dynamic LDS of the closed-form leftovers' workgroup (fec_vr_encode_cf_kernel, fec_vr_cf.h)
size_t vr_encode_cf_lds(const VrEncodeArgs& a);

// A schedule of encoder instances from outside the P2P loop (fec_session.hip) as a plan handle of
// the C ABI (fec_vr_encode_batch, fec_vr_plan_layout, fec_vr_plan_destroy); its device row offsets.
int vr_plan_from_instances(int max_payload, const std::vector<VrInstance>& enc, int64_t sent, fec_vr_plan** out);
int vr_plan_device_offsets(fec_vr_plan* v, void* s, const int64_t** cur_off, const int64_t** old_off);

}  // namespace fec
