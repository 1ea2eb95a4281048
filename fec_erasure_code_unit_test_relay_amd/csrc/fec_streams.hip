// fec_streams.hip -- many independent streams of one (T,B,N), one packet of each per call, coded in
// one launch (north_star: "many independent (T,B,N) coding windows batched across wavefronts").
//
// The reference runs one FEC_Encoder / FEC_Decoder per stream (include/FEC_Encoder.h:26-48,
// FEC_Decoder.h:27-46), one packet per onTransmit / onReceive call, and keeps each stream's state
// inside those objects.  Here a group holds the state of N streams in HBM:
//   * encoder: the last n-1 windows X_{t-1..t-n+1} of every stream (bytes [len_hi, len_lo,
//     payload, zero pad] of S*k bytes, Encoder.cpp:73-95), a ring indexed by seq % (n-1);
//   * decoder: the last RR received codewords of every stream (zero padded like
//     FEC_Decoder.cpp:55-63), a ring indexed by seq % RR, and per stream the symbolic planner
//     (fec::StreamPlanner, the reference decoder's state machine without the bytes) on the host.
// A call names M distinct streams and hands over one packet of each; one wave per packet does
// its byte work: the encoder's closed form (Encoder.cpp:65-98 -> codingOperations.cpp:131-147)
// over the stream's window, or the decoder's output for packet seq - T (fast path copy,
// Decoder.cpp:77-108, or the planner's recovery coefficients, codingOperations.cpp:149-232).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

#include "fec_amd.h"
#include "fec_host.h"
#include "fec_kernels.h"
#include "fec_status.h"

namespace fec {
namespace {

constexpr int kRR = 64;  // decoder ring rows per stream (>= T + k, the per-packet decoder's)

struct StreamsEncArgs {
    const uint8_t* payload;  // M rows of L bytes
    const int32_t* len;      // M payload sizes (null: all L)
    const int32_t* ids;      // M stream ids
    const int64_t* seq;      // M: packets the stream sent before this one
    uint8_t* win;            // [streams][W][SK] window ring
    uint8_t* cw;             // M rows of CW bytes
    int32_t* cw_len;         // M trimmed sizes
    const uint8_t* G;        // k x n
    const uint8_t* gf;       // exp[512], log[256]
    int M, L, k, n, S, CW, SK, W;
    // single-packet calls (stream_encode_one): seq / ids / len null -> seq1, stream 0, len1; after the
    // packet's outputs the wave stores ticket into the host-visible word `done` (null: none)
    int64_t seq1;
    int len1;
    uint32_t* done;
    uint32_t ticket;
};

struct StreamItem {
    int32_t id;
    int32_t fate;    // PacketFate of the packet output by this call (x = seq - T)
    int32_t clamp;   // slow path: payload clamped to L (Decoder.cpp:148-149)
    int32_t coef;    // kRecovered: index of its k x n block in coefs
    int64_t seq;     // packets the stream received before this one
    int64_t x;       // packet output by this call
    int32_t erased;  // this call's packet is missing
    int32_t pad;
};

struct StreamsDecArgs {
    const uint8_t* cw_in;    // M rows of CW bytes (rows of erased packets are not read)
    const StreamItem* items;
    const uint8_t* coefs;    // recovered outputs' coefficient blocks
    uint8_t* ring;           // [streams][RR][CW]
    const uint8_t* gf;
    uint8_t* out;            // M rows of L bytes
    int32_t* out_len;
    int M, L, k, n, CW, RR;
    // single-packet calls (stream_decode_one): items null -> item1; after the outputs the wave stores
    // ticket into the host-visible word `done` (null: none)
    StreamItem item1;
    uint32_t* done;
    uint32_t ticket;
};

__device__ __forceinline__ uint8_t gmul(const uint8_t* gexp, const uint8_t* glog, uint8_t a, uint8_t b) {
    return (a && b) ? gexp[glog[a] + glog[b]] : 0;
}

// Single-packet calls (stream_encode_one, M == 1): the whole workgroup on the one codeword, a thread
// per codeword byte, so that no thread walks a long chain of table lookups (the per-packet
// FEC_Encoder's latency).  prow / wst / rowoff / cwl are the kernel's LDS (wave 0's slices).
__device__ __forceinline__ void single_packet_encode(const StreamsEncArgs& a, int tid, const uint8_t* gexp,
                                                     const uint8_t* glog, const uint8_t* Gs, const uint8_t* pay,
                                                     const uint32_t* wst, int* ro, uint32_t* cwl) {
    __shared__ int last_nz;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW, SK = a.SK, W = a.W;
    const int ln = min(max(a.len1, 0), L);
    const int64_t seq = a.seq1;
    if (tid < 32) ro[tid] = (tid >= 1 && seq - tid >= 0) ? static_cast<int>((seq - tid) % W) * SK : -1;
    if (tid == 0) last_nz = -1;
    __syncthreads();  // payload row, window, offsets
    auto xbyte = [&](int b) -> uint8_t {  // [len_hi, len_lo, payload, zero pad] (Encoder.cpp:75-83)
        return b == 0 ? static_cast<uint8_t>(ln >> 8)
                      : b == 1 ? static_cast<uint8_t>(ln & 0xff) : (b - 2 < ln ? pay[b - 2] : 0);
    };
    const bool lds_out = CW <= 2048 && (reinterpret_cast<uintptr_t>(a.cw) & 3) == 0;
    uint8_t* cwb = lds_out ? reinterpret_cast<uint8_t*>(cwl) : a.cw;
    int last = -1;
    for (int c = tid; c < CW; c += 256) {
        const int s = c / n, j = c - s * n;
        uint8_t v = 0;
        if (j < k) {
            v = xbyte(s * k + j);
        } else {  // parity: XOR_i G[i][j] * X_{t-(j-i)}[s][i], rows before the stream start = 0
            for (int i = 0; i < k; ++i) {
                const int r = ro[j - i];
                if (r < 0) continue;
                const int o = r + s * k + i;
                const uint8_t xb = wst ? reinterpret_cast<const uint8_t*>(wst)[o] : a.win[o];
                v ^= gmul(gexp, glog, Gs[i * n + j], xb);
            }
        }
        cwb[c] = v;
        if (v) last = c;
    }
    if (last >= 0) atomicMax(&last_nz, last);
    __syncthreads();  // codeword complete; the window slot of seq - W (= seq % W) has been read
    const int own = static_cast<int>(seq % W) * SK;
    for (int b = tid; b < SK; b += 256) a.win[own + b] = xbyte(b);
    if (lds_out)
        for (int w = tid; 4 * w < CW; w += 256) reinterpret_cast<uint32_t*>(a.cw)[w] = cwl[w];
    if (tid == 0) a.cw_len[0] = last_nz + 1;  // FEC_Encoder.cpp:55-60
    if (a.done) {  // every thread's stores complete, then the completion word
        __threadfence_system();
        __syncthreads();
        if (tid == 0) *reinterpret_cast<volatile uint32_t*>(a.done) = a.ticket;
    }
}

// One wave per packet: lane = sub-stream (and sub-stream + 64, ...).
__global__ __launch_bounds__(256) void fec_streams_encode_kernel(StreamsEncArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t Gs[16 * 32];
    __shared__ uint32_t prow[4][376];  // each wave's payload row (L <= 1500), read once with dword loads
    __shared__ uint32_t wst[4][1024];  // each wave's window ring when it fits 4 KB: all loads in flight
    __shared__ uint32_t cwst[512];     // single-packet calls: the codeword (CW <= 2048)
    __shared__ int rowoff[4][32];      // per wave: window offset of packet seq - d (-1: before the stream)
    const int tid = threadIdx.x;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    for (int i = tid; i < a.k * a.n; i += 256) Gs[i] = a.G[i];
    const int m = blockIdx.x * 4 + (tid >> 6), lane = tid & 63;
    if (m < a.M) {  // the payload may be a host-visible row: all loads in flight at once
        const uint8_t* src = a.payload + static_cast<int64_t>(m) * a.L;
        uint8_t* dst = reinterpret_cast<uint8_t*>(prow[tid >> 6]);
        if (((a.L | static_cast<int>(reinterpret_cast<uintptr_t>(src))) & 3) == 0) {
            for (int w = lane; 4 * w < a.L; w += 64) prow[tid >> 6][w] = reinterpret_cast<const uint32_t*>(src)[w];
        } else {
            for (int b = lane; b < a.L; b += 64) dst[b] = src[b];
        }
    }
    const int wbytes = a.W * a.SK;
    const bool wlds = wbytes <= 4096 && (wbytes & 3) == 0;
    if (m < a.M && wlds) {
        const uint32_t* wsrc = reinterpret_cast<const uint32_t*>(a.win + static_cast<int64_t>(a.ids ? a.ids[m] : 0) * wbytes);
        for (int w = lane; 4 * w < wbytes; w += 64) wst[tid >> 6][w] = wsrc[w];
    }
    if (!a.ids) {
        single_packet_encode(a, tid, gexp, glog, Gs, reinterpret_cast<const uint8_t*>(prow[0]), wlds ? wst[0] : nullptr,
                             rowoff[0], cwst);
        return;
    }
    __syncthreads();
    if (m >= a.M) return;
    const int L = a.L, k = a.k, n = a.n, S = a.S, CW = a.CW, SK = a.SK, W = a.W;
    const int ln = min(max(a.len ? a.len[m] : a.len1, 0), L);
    const int64_t seq = a.seq ? a.seq[m] : a.seq1;
    uint8_t* win = a.win + static_cast<int64_t>(a.ids ? a.ids[m] : 0) * W * SK;
    const uint8_t* pay = reinterpret_cast<const uint8_t*>(prow[tid >> 6]);
    uint8_t* cwo = a.cw + static_cast<int64_t>(m) * CW;
    // single-packet calls write the codeword into LDS first, then to the (host-visible) result row
    // in dwords (the row is padded to whole dwords)
    const bool lds_out = !a.ids && CW <= 2048 && (reinterpret_cast<uintptr_t>(cwo) & 3) == 0;
    uint8_t* cwl = reinterpret_cast<uint8_t*>(cwst);
    // window byte b of this packet: [len_hi, len_lo, payload, zero pad] (Encoder.cpp:75-83)
    auto xbyte = [&](int b) -> uint8_t {
        return b == 0 ? static_cast<uint8_t>(ln >> 8)
                      : b == 1 ? static_cast<uint8_t>(ln & 0xff) : (b - 2 < ln ? pay[b - 2] : 0);
    };
    int* ro = rowoff[tid >> 6];
    if (lane < 32) ro[lane] = (lane >= 1 && seq - lane >= 0) ? static_cast<int>((seq - lane) % W) * SK : -1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int own = static_cast<int>(seq % W) * SK;
    int last = -1;  // last non-zero codeword byte of this lane's sub-streams
    for (int s = lane; s < S; s += 64) {
        for (int j = 0; j < n; ++j) {
            uint8_t v;
            if (j < k) {
                v = xbyte(s * k + j);
            } else {  // parity: XOR_i G[i][j] * X_{t-(j-i)}[s][i], rows before the stream start = 0
                v = 0;
                for (int i = 0; i < k; ++i) {
                    const int r = ro[j - i];
                    if (r < 0) continue;
                    const int o = r + s * k + i;
                    const uint8_t xb = wlds ? reinterpret_cast<const uint8_t*>(wst[tid >> 6])[o] : win[o];
                    v ^= gmul(gexp, glog, Gs[i * n + j], xb);
                }
            }
            if (lds_out)
                cwl[s * n + j] = v;
            else
                cwo[s * n + j] = v;
            if (v) last = s * n + j;
        }
        // this lane's own bytes of slot seq % W: read above (d = W), now overwritten
        for (int i = 0; i < k; ++i) win[own + s * k + i] = xbyte(s * k + i);
    }
    if (lds_out) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int w = lane; 4 * w < CW; w += 64) reinterpret_cast<uint32_t*>(cwo)[w] = cwst[w];
    }
    for (int d = 32; d >= 1; d >>= 1) last = max(last, __shfl_xor(last, d, 64));
    if (lane == 0) a.cw_len[m] = last + 1;  // FEC_Encoder.cpp:55-60
    if (a.done) {  // every lane's stores complete, then the completion word (one wave: M == 1)
        __threadfence_system();
        if (lane == 0) *reinterpret_cast<volatile uint32_t*>(a.done) = a.ticket;
    }
}

template <class Sym>
__device__ __forceinline__ void stream_output(const StreamsDecArgs& a, const StreamItem& it, uint8_t* orow, int m,
                                              int lane, const uint8_t* gexp, const uint8_t* glog, Sym sym);

// One wave per packet: store the received codeword in the stream's ring, output packet x.
__global__ __launch_bounds__(256) void fec_streams_decode_kernel(StreamsDecArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    const int tid = threadIdx.x;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int m = blockIdx.x * 4 + (tid >> 6), lane = tid & 63;
    if (m >= a.M) return;
    const StreamItem it = a.items ? a.items[m] : a.item1;
    const int L = a.L, CW = a.CW, RR = a.RR;
    uint8_t* ring = a.ring + static_cast<int64_t>(it.id) * RR * CW;
    const uint8_t* cwin = a.cw_in + static_cast<int64_t>(m) * CW;
    if (!it.erased) {  // FEC_Decoder.cpp:55-59: the decoder keeps its own copy
        uint8_t* dst = ring + (it.seq % RR) * CW;
        if (!a.items && (reinterpret_cast<uintptr_t>(cwin) & 3) == 0) {
            // single packet from a host-visible row padded to whole dwords: dword loads, all in flight
            for (int w = lane; 4 * w < CW; w += 64) {
                const uint32_t v = reinterpret_cast<const uint32_t*>(cwin)[w];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (4 * w + e < CW) dst[4 * w + e] = static_cast<uint8_t>(v >> (8 * e));
            }
        } else {
            for (int b = lane; b < CW; b += 64) dst[b] = cwin[b];
        }
    }
    // symbol (s, q) of packet sp: this call's codeword straight from the input (the ring row it
    // was just written to is not read back), older ones from the ring
    auto sym = [&](int64_t sp, int o) -> uint8_t {
        return sp == it.seq ? cwin[o] : ring[(((sp % RR) + RR) % RR) * CW + o];  // sp < 0: a zero row
    };
    uint8_t* orow = a.out + static_cast<int64_t>(m) * L;
    if (it.fate == kNone || it.fate == kLost) {
        for (int b = lane; b < L; b += 64) orow[b] = 0;
        if (lane == 0) a.out_len[m] = 0;
    } else {
        stream_output(a, it, orow, m, lane, gexp, glog, sym);
    }
    if (a.done) {  // every lane's stores complete, then the completion word (one wave: M == 1)
        __threadfence_system();
        if (lane == 0) *reinterpret_cast<volatile uint32_t*>(a.done) = a.ticket;
    }
}

template <class Sym>
__device__ __forceinline__ void stream_output(const StreamsDecArgs& a, const StreamItem& it, uint8_t* orow, int m,
                                              int lane, const uint8_t* gexp, const uint8_t* glog, Sym sym) {
    const int L = a.L, k = a.k, n = a.n;
    const uint8_t* coef = a.coefs + static_cast<int64_t>(it.coef) * k * n;
    // header bytes 0, 1 (sub-stream 0, positions 0 and 1 -> (1/k)*n + 1%k) first: they bound the copy
    auto byte_at = [&](int h) -> uint8_t {
        const int s = h / k, i = h - s * k;
        if (it.fate == kCopy) return sym(it.x, s * n + i);
        uint8_t acc = 0;
        for (int q = 0; q < n; ++q) {
            const uint8_t c = coef[i * n + q];
            if (c) acc ^= gmul(gexp, glog, c, sym(it.x - i + q, s * n + q));
        }
        return acc;
    };
    const int hdr = byte_at(0) * 256 + byte_at(1);
    const int ln = it.clamp ? min(hdr, L) : hdr;
    const int cp = min(ln, L);
    for (int b = lane; b < L; b += 64) orow[b] = b < cp ? byte_at(b + 2) : 0;
    if (lane == 0) a.out_len[m] = ln;
}

}  // namespace
}  // namespace fec

namespace {
// Fork-join pool for the decoders' symbolic steps of one call: the streams are independent, so the
// call's items are cut into contiguous parts, one per thread (the calling thread takes part 0).  A
// worker polls for the next job for a while (calls come back to back) before it sleeps: a sleeping
// thread's wake-up costs tens of microseconds, as much as its share of the steps.
// The workers run on the 8 CPUs of the creating thread's aligned group (within the allowed set):
// on a two-socket box the scheduler otherwise spreads them over both sockets (FEC_STREAMS_PIN=0:
// unplaced).
// A group with fewer than 4 allowed CPUs (a sparse cpuset: taskset, cgroup) is left alone: spin-
// polling workers crowded on one or two CPUs stall each other for milliseconds.
void place_near(int home) {
    if (home < 0) return;
    cpu_set_t allowed, set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
    const int base = home & ~7;
    for (int c = base; c < base + 8 && c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &allowed)) CPU_SET(c, &set);
    if (CPU_COUNT(&set) >= 4) (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}
// CPUs this process may run on (its affinity mask), at least 1.
int allowed_cpus() {
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return static_cast<int>(std::thread::hardware_concurrency());
    return std::max(1, CPU_COUNT(&allowed));
}

class StepPool {
public:
    explicit StepPool(int threads) {
        const char* pin = std::getenv("FEC_STREAMS_PIN");
        const int home = (pin && std::atoi(pin) == 0) ? -1 : sched_getcpu();
        for (int i = 1; i < threads; ++i) th_.emplace_back([this, i, home] {
            place_near(home);
            loop(i);
        });
    }
    ~StepPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int parts() const { return static_cast<int>(th_.size()) + 1; }
    // f(part) for every part; returns after all of them
    void run(const std::function<void(int)>& f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            left_.store(static_cast<int>(th_.size()), std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        f(0);
        while (left_.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
    }

private:
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            // poll up to ~0.2 ms for the next job, then sleep
            const auto t0 = std::chrono::steady_clock::now();
            for (int spin = 0; gen_.load(std::memory_order_acquire) == seen && !stop_.load(); ++spin) {
                __builtin_ia32_pause();
                if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
            }
            const std::function<void(int)>* f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_.load() || gen_.load() != seen; });
                if (stop_.load()) return;
                seen = gen_.load();
                f = job_;
            }
            (*f)(i);
            left_.fetch_sub(1, std::memory_order_release);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    const std::function<void(int)>* job_ = nullptr;
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> stop_{false};
    std::atomic<int> left_{0};
};
}  // namespace

constexpr int kPoolMinItems = 1024;  // items per part below which a call steps on one thread

struct fec_streams {
    std::unique_ptr<StepPool> pool;          // symbolic steps of large calls (FEC_STREAMS_THREADS)
    fec_codec* codec = nullptr;
    fec::Geometry g;
    int nstreams = 0, W = 1, SK = 0;
    std::shared_ptr<const fec::DecodeRules> rules;
    std::vector<std::unique_ptr<fec::StreamPlanner>> planners;
    std::vector<int64_t> enc_seq, dec_seq;   // packets sent / received so far per stream
    std::vector<uint32_t> mark;              // duplicate-id check (call stamp per stream)
    uint32_t stamp = 0;
    uint8_t* d_win = nullptr;                // encoder windows
    uint8_t* d_ring = nullptr;               // decoder rings
    // Per-call records (ids + seqs / items + coefs) go through a ring of kStageBufs staging buffers,
    // so the host prepares a call (the decoders' symbolic steps) while the GPU still runs the ones
    // before it; a buffer is rewritten only after its upload has completed.
    static constexpr int kStageBufs = 4;
    // The kernels read the records straight from the pinned buffers (mapped: m_stage) -- an upload
    // per call put an SDMA copy and its hand-off to the kernel on the GPU's path, twice per
    // encode + decode pair (FEC_STREAMS_UPLOAD=1 keeps those uploads into d_stage).
    void* d_stage[kStageBufs] = {};
    void* h_stage[kStageBufs] = {};          // pinned records
    void* m_stage[kStageBufs] = {};          // their device addresses
    bool upload = false;
    hipEvent_t staged[kStageBufs] = {};      // the last kernel (and upload) that read h_stage[b]
    int buf = 0;                             // the next call's buffer
    size_t stage_bytes = 0;
    hipEvent_t done = nullptr;               // the last call's kernel (windows, rings, older d_stage free)
    bool poisoned = false;                   // a failed call left host and device state apart
    ~fec_streams() {
        for (hipEvent_t e : staged)
            if (e) (void)hipEventDestroy(e);
        if (done) (void)hipEventDestroy(done);
        for (void* p : {static_cast<void*>(d_win), static_cast<void*>(d_ring)})
            if (p) (void)hipFree(p);
        for (void* p : d_stage)
            if (p) (void)hipFree(p);
        for (void* p : h_stage)
            if (p) (void)hipHostFree(p);
        if (codec) fec_codec_destroy(codec);
    }
};

namespace {

#define FS_TRY(expr)                              \
    do {                                          \
        FEC_HIP((expr)); \
    } while (0)

// ids distinct and in range
int check_ids(fec_streams* h, const int32_t* ids, int M) {
    if (++h->stamp == 0) {
        std::fill(h->mark.begin(), h->mark.end(), 0u);
        h->stamp = 1;
    }
    for (int m = 0; m < M; ++m) {
        const int id = ids[m];
        if (id < 0 || id >= h->nstreams || h->mark[id] == h->stamp) return FEC_ERR_ARG;
        h->mark[id] = h->stamp;
    }
    return FEC_OK;
}

// This call's staging buffer: the call that used it before has read it (host wait on that call's
// kernel, kStageBufs calls back), and the previous call's kernel -- which read / wrote the windows and
// rings, after every older kernel and so after the last reader of d_stage[b] -- comes before
// anything this call enqueues on `s`, whichever stream the previous call used (device-side wait).
int stage_free(fec_streams* h, hipStream_t s, int* b) {
    if (h->poisoned) return FEC_ERR_HIP;
    *b = h->buf;
    FS_TRY(hipEventSynchronize(h->staged[*b]));
    FS_TRY(hipStreamWaitEvent(s, h->done, 0));
    return FEC_OK;
}

}  // namespace

int fec::stream_encode_one(const CodecView& v, uint8_t* win, const uint8_t* payload, int payload_len, int64_t seq,
                           uint8_t* cw, int32_t* cw_len, uint32_t* done, uint32_t ticket, hipStream_t s) {
    if (v.k > 16 || v.k * v.n > 16 * 32) return FEC_ERR_ARG;  // the kernel's register / LDS bounds
    fec::StreamsEncArgs a;
    a.payload = payload;
    a.len = nullptr;
    a.ids = nullptr;
    a.seq = nullptr;
    a.win = win;
    a.cw = cw;
    a.cw_len = cw_len;
    a.G = v.G;
    a.gf = v.gf;
    a.M = 1;
    a.L = v.L;
    a.k = v.k;
    a.n = v.n;
    a.S = v.S;
    a.CW = v.CW;
    a.SK = v.S * v.k;
    a.W = std::max(1, v.n - 1);
    a.seq1 = seq;
    a.len1 = payload_len;
    a.done = done;
    a.ticket = ticket;
    hipLaunchKernelGGL(fec::fec_streams_encode_kernel, dim3(1), dim3(256), 0, s, a);  // 256: the table loads
    FS_TRY(hipGetLastError());
    return FEC_OK;
}

int fec::stream_decode_one(const CodecView& v, uint8_t* ring, const uint8_t* cw, int64_t seq, int erased,
                           int fate, int clamp, int64_t x, const uint8_t* coef, uint8_t* out, int32_t* out_len,
                           uint32_t* done, uint32_t ticket, hipStream_t s) {
    fec::StreamsDecArgs a;
    a.cw_in = cw;
    a.items = nullptr;
    a.coefs = coef;
    a.ring = ring;
    a.gf = v.gf;
    a.out = out;
    a.out_len = out_len;
    a.M = 1;
    a.L = v.L;
    a.k = v.k;
    a.n = v.n;
    a.CW = v.CW;
    a.RR = kRR;
    a.item1 = fec::StreamItem{0, fate, clamp, 0, seq, x, erased, 0};
    a.done = done;
    a.ticket = ticket;
    hipLaunchKernelGGL(fec::fec_streams_decode_kernel, dim3(1), dim3(256), 0, s, a);  // 256: the table loads
    FS_TRY(hipGetLastError());
    return FEC_OK;
}

extern "C" {

int fec_streams_create(int max_payload, int T, int B, int N, int nstreams, fec_streams** out) {
    if (!out || nstreams <= 0) return FEC_ERR_ARG;
    *out = nullptr;
    try {
        std::unique_ptr<fec_streams> h(new fec_streams());
        if (int st = fec_codec_create(max_payload, T, B, N, &h->codec)) return st;
        fec::CodecView v;
        if (int st = fec::codec_view(h->codec, &v)) return st;
        h->g = fec::Geometry::make(max_payload, T, B, N);
        const fec::Geometry& g = h->g;
        if (g.T + g.k > fec::kRR || g.k > 16 || g.k * g.n > 16 * 32) return FEC_ERR_ARG;
        h->nstreams = nstreams;
        h->W = std::max(1, g.n - 1);
        h->SK = g.S * g.k;
        h->rules = fec::shared_decode_rules(T, B, N);
        h->planners.resize(nstreams);
        for (auto& p : h->planners) p.reset(new fec::StreamPlanner(g, h->rules.get()));
        {
            const int hw = allowed_cpus();  // not hardware_concurrency: the process's cpuset may be smaller
            int nth = std::max(1, std::min(hw > 1 ? hw - 1 : 1, 8));
            if (const char* e = std::getenv("FEC_STREAMS_THREADS")) nth = std::max(1, std::atoi(e));
            if (nth > 1 && nstreams >= 2 * kPoolMinItems) h->pool.reset(new StepPool(nth));
        }
        h->enc_seq.assign(nstreams, 0);
        h->dec_seq.assign(nstreams, 0);
        h->mark.assign(nstreams, 0);
        const size_t wb = static_cast<size_t>(nstreams) * h->W * h->SK;
        const size_t rb = static_cast<size_t>(nstreams) * fec::kRR * g.CW;
        FS_TRY(hipMalloc(&h->d_win, wb));
        FS_TRY(hipMemset(h->d_win, 0, wb));
        FS_TRY(hipMalloc(&h->d_ring, rb));
        FS_TRY(hipMemset(h->d_ring, 0, rb));
        h->stage_bytes = static_cast<size_t>(nstreams) * (sizeof(fec::StreamItem) + g.k * g.n + 16) + 64;
        if (const char* e = std::getenv("FEC_STREAMS_UPLOAD")) h->upload = std::atoi(e) != 0;
        for (int b = 0; b < fec_streams::kStageBufs; ++b) {
            if (h->upload) FS_TRY(hipMalloc(&h->d_stage[b], h->stage_bytes));
            FS_TRY(hipHostMalloc(&h->h_stage[b], h->stage_bytes, hipHostMallocMapped));
            FS_TRY(hipHostGetDevicePointer(&h->m_stage[b], h->h_stage[b], 0));
            FS_TRY(hipEventCreateWithFlags(&h->staged[b], hipEventDisableTiming));
            FS_TRY(hipEventRecord(h->staged[b], nullptr));
        }
        FS_TRY(hipEventCreateWithFlags(&h->done, hipEventDisableTiming));
        FS_TRY(hipEventRecord(h->done, nullptr));
        *out = h.release();
        return FEC_OK;
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}

int fec_streams_destroy(fec_streams* h) {
    delete h;
    return FEC_OK;
}

int fec_streams_encode(fec_streams* h, const int32_t* ids, int M, const uint8_t* d_payload,
                       const int32_t* d_payload_len, uint8_t* d_codeword, int32_t* d_codeword_len,
                       void* stream) {
    if (!h || M < 0 || M > h->nstreams || (M > 0 && (!ids || !d_payload || !d_codeword || !d_codeword_len)))
        return FEC_ERR_ARG;
    if (M == 0) return FEC_OK;
    if (int st = check_ids(h, ids, M)) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    int b = 0;
    if (int st = stage_free(h, s, &b)) return st;
    int64_t* hseq = static_cast<int64_t*>(h->h_stage[b]);
    int32_t* hid = reinterpret_cast<int32_t*>(hseq + M);
    for (int m = 0; m < M; ++m) {
        hseq[m] = h->enc_seq[ids[m]];  // committed below, once the launch is in
        hid[m] = ids[m];
    }
    const size_t bytes = static_cast<size_t>(M) * 12;
    if (h->upload) FS_TRY(hipMemcpyAsync(h->d_stage[b], h->h_stage[b], bytes, hipMemcpyHostToDevice, s));
    const void* rec = h->upload ? h->d_stage[b] : h->m_stage[b];
    fec::CodecView v;
    fec::codec_view(h->codec, &v);
    fec::StreamsEncArgs a;
    a.payload = d_payload;
    a.len = d_payload_len;
    a.seq = static_cast<const int64_t*>(rec);
    a.ids = reinterpret_cast<const int32_t*>(static_cast<const int64_t*>(rec) + M);
    a.win = h->d_win;
    a.cw = d_codeword;
    a.cw_len = d_codeword_len;
    a.G = v.G;
    a.gf = v.gf;
    a.M = M;
    a.L = h->g.L;
    a.k = h->g.k;
    a.n = h->g.n;
    a.S = h->g.S;
    a.CW = h->g.CW;
    a.SK = h->SK;
    a.W = h->W;
    a.seq1 = 0;
    a.len1 = h->g.L;
    a.done = nullptr;
    a.ticket = 0;
    hipLaunchKernelGGL(fec::fec_streams_encode_kernel, dim3((M + 3) / 4), dim3(256), 0, s, a);
    FS_TRY(hipGetLastError());
    FS_TRY(hipEventRecord(h->done, s));
    FS_TRY(hipEventRecord(h->staged[b], s));
    h->buf = (b + 1) % fec_streams::kStageBufs;
    for (int m = 0; m < M; ++m) ++h->enc_seq[ids[m]];
    return FEC_OK;
}

int fec_streams_decode(fec_streams* h, const int32_t* ids, int M, const uint8_t* erasure,
                       const uint8_t* d_codeword, uint8_t* d_payload_out, int32_t* d_payload_len,
                       void* stream) {
    if (!h || M < 0 || M > h->nstreams || (M > 0 && (!ids || !erasure || !d_codeword || !d_payload_out ||
                                                     !d_payload_len)))
        return FEC_ERR_ARG;
    if (M == 0) return FEC_OK;
    static const bool dbg = std::getenv("FEC_STREAMS_DEBUG") != nullptr;  // per-phase host times
    const auto t0 = std::chrono::steady_clock::now();
    if (int st = check_ids(h, ids, M)) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    int b = 0;
    const auto t1 = std::chrono::steady_clock::now();
    if (int st = stage_free(h, s, &b)) return st;
    const auto t2 = std::chrono::steady_clock::now();
    const fec::Geometry& g = h->g;
    // The symbolic decoders advance below, before the upload and the launch; if either fails, the
    // host planners are ahead of the device rings and the group refuses every later call.
    struct Poison {
        fec_streams* h;
        bool armed = true;
        ~Poison() { if (armed) h->poisoned = true; }
    } poison{h};
    fec::StreamItem* items = static_cast<fec::StreamItem*>(h->h_stage[b]);
    uint8_t* coefs = reinterpret_cast<uint8_t*>(items + M);
    const int kn = g.k * g.n;
    std::atomic<int> ncoef_a{0};
    std::atomic<bool> failed{false};
    // one symbolic decoder step per item; the recovered packets' coefficient rows take slots in
    // arrival order (an item carries its slot)
    auto steps = [&](int m0, int m1) {
        try {
            for (int m = m0; m < m1; ++m) {
                const int id = ids[m];
                const bool er = erasure[m] != 0;
                const int64_t seq = h->dec_seq[id]++;
                const fec::StepResult r = h->planners[id]->step(seq, er);
                fec::StreamItem& it = items[m];
                it.id = id;
                it.fate = r.fate;
                it.clamp = r.slow ? 1 : 0;
                it.coef = 0;
                it.seq = seq;
                it.x = r.x;
                it.erased = er ? 1 : 0;
                it.pad = 0;
                if (r.fate == fec::kRecovered) {
                    const int slot = ncoef_a.fetch_add(1, std::memory_order_relaxed);
                    std::memcpy(coefs + static_cast<size_t>(slot) * kn, r.coef, kn);
                    it.coef = slot;
                }
            }
        } catch (...) {
            failed.store(true);
        }
    };
    if (h->pool && M >= 2 * kPoolMinItems) {
        const int np = h->pool->parts();
        h->pool->run([&](int p) { steps(static_cast<int>(static_cast<int64_t>(M) * p / np),
                                        static_cast<int>(static_cast<int64_t>(M) * (p + 1) / np)); });
    } else {
        steps(0, M);
    }
    if (failed.load()) return FEC_ERR_ARG;
    const int ncoef = ncoef_a.load();
    const auto t3 = std::chrono::steady_clock::now();
    const size_t bytes = static_cast<size_t>(M) * sizeof(fec::StreamItem) + static_cast<size_t>(ncoef) * kn;
    if (h->upload) FS_TRY(hipMemcpyAsync(h->d_stage[b], h->h_stage[b], bytes, hipMemcpyHostToDevice, s));
    const void* rec = h->upload ? h->d_stage[b] : h->m_stage[b];
    fec::CodecView v;
    fec::codec_view(h->codec, &v);
    fec::StreamsDecArgs a;
    a.cw_in = d_codeword;
    a.items = static_cast<const fec::StreamItem*>(rec);
    a.coefs = reinterpret_cast<const uint8_t*>(a.items + M);
    a.ring = h->d_ring;
    a.gf = v.gf;
    a.out = d_payload_out;
    a.out_len = d_payload_len;
    a.M = M;
    a.L = g.L;
    a.k = g.k;
    a.n = g.n;
    a.CW = g.CW;
    a.RR = fec::kRR;
    a.done = nullptr;
    a.ticket = 0;
    hipLaunchKernelGGL(fec::fec_streams_decode_kernel, dim3((M + 3) / 4), dim3(256), 0, s, a);
    FS_TRY(hipGetLastError());
    FS_TRY(hipEventRecord(h->done, s));
    FS_TRY(hipEventRecord(h->staged[b], s));
    h->buf = (b + 1) % fec_streams::kStageBufs;
    poison.armed = false;
    if (dbg) {
        const auto t4 = std::chrono::steady_clock::now();
        auto us = [](auto a, auto z) { return std::chrono::duration<double, std::micro>(z - a).count(); };
        std::fprintf(stderr, "streams decode: ids %.1f us, stage wait %.1f, steps %.1f, upload + launch %.1f\n",
                     us(t0, t1), us(t1, t2), us(t2, t3), us(t3, t4));
    }
    return FEC_OK;
}

int fec_streams_state(const fec_streams* h, int id, int64_t* sent, int64_t* received) {
    if (!h || id < 0 || id >= h->nstreams) return FEC_ERR_ARG;
    if (sent) *sent = h->enc_seq[id];
    if (received) *received = h->dec_seq[id];
    return FEC_OK;
}

}  // extern "C"
