// fec_codec.hip -- codec objects, launchers and the C ABI declared in include/fec_amd.h.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "fec_amd.h"
#include "fec_host.h"
#include "fec_kernels.h"
#include "fec_status.h"

using fec::Geometry;

namespace {

constexpr int kLdsBudget = 64 * 1024;
constexpr int kCopyLdsBudget = 32 * 1024;  // decode copy tiles (see the tile choice below)
constexpr int kMaxPayload = 1500;  // UDP MTU; bounds the LDS tiles

inline int round16(int v) { return (v + 15) & ~15; }

#define HIP_TRY(expr)                                  \
    do {                                               \
        if ((expr) != hipSuccess) return FEC_ERR_HIP;  \
    } while (0)

struct EventPair {
    int kernel;
    hipEvent_t a, b;
};

}  // namespace

struct fec_decode_stream {
    int64_t consumed = 0;  // packets pushed so far
    int64_t last_cut = 0;  // where the last push restarted the decode (diagnostics)
};

struct fec_codec {
    Geometry g;
    bool compact_fresh = false;  // the planner's counters were reset and no compaction ran since
    std::vector<uint8_t> G;
    std::shared_ptr<const fec::DecodeRules> rules;  // process-wide cache (shared_decode_rules)
    uint32_t* d_ptab = nullptr;  // [k][n-k][8]
    uint8_t* d_rules = nullptr;
    int64_t* d_wbase = nullptr;  // [n+1]
    uint8_t* d_rules_log = nullptr;  // rules with coefficients in log form (specialised planner)
    const void* plan_fast = nullptr;
    uint8_t* d_gf = nullptr;     // exp[512], log[256]
    uint8_t* d_G = nullptr;      // k x n generator (block mode)
    uint8_t* d_rstate = nullptr; // post-resync block states per phase
    int enc_tp = 0;              // encode tile (packets per workgroup), generic kernel
    int encode_path = 0;         // 0 auto, 1 generic, 5 tile (the ids of round 2's paths are kept)
    int cus = 0;                        // compute units of the device
    const void* tile_kernel = nullptr;  // contiguous-chunk LDS-tile encode (fec_encode_tile.hip)
    int tile_ppw = 0;                   // its packets per wave slice (tile = 4 * tile_ppw packets)
    int tile_lds = 0, tile_lds_len = 0; // its dynamic LDS per workgroup (without / with lengths)
    int tile_per_cu = 0;                // its resident workgroups per CU
    int tile_off[9] = {};               // off_in, in_bytes, off_pw, off_q, off_out, off_len, ngl, nso, off_scratch
    const void* copy_fast = nullptr;  // specialised decode copy kernel (LDS tiles)
    int copyf_tp = 0;
    int copy_path = 0;           // 0 auto, 1 generic, 2 specialised (LDS tiles)
    int plan_path = 0;
    int dedup = 1;               // episode-shape deduplication in the planner
    uint64_t* d_stamps = nullptr;  // diagnostics: phase stamps of the next specialised launch
    int stamp_kernel = -1;
    int copy_tp = 0;             // decode-copy tile
    bool timing = false;
    std::vector<EventPair> events;
    hipStream_t side = nullptr;  // decode plan runs here, forked from the caller's stream
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;

    ~fec_codec() {
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (side) (void)hipStreamDestroy(side);
        for (auto& e : events) {
            (void)hipEventDestroy(e.a);
            (void)hipEventDestroy(e.b);
        }
        if (d_ptab) (void)hipFree(d_ptab);
        if (d_rules) (void)hipFree(d_rules);
        if (d_wbase) (void)hipFree(d_wbase);
        if (d_rules_log) (void)hipFree(d_rules_log);
        if (d_gf) (void)hipFree(d_gf);
        if (d_G) (void)hipFree(d_G);
        if (d_rstate) (void)hipFree(d_rstate);
    }

    int enc_lds(int tp) const {
        const int SP = (g.S + 3) & ~3;
        const int rows = tp + g.n - 1;
        const int Sk = g.S * g.k;
        return round16(g.k * rows * SP) + round16(tp * g.CW) + 2 * ((Sk + 7) & ~7) + 4 * rows;
    }
    int copy_lds(int tp) const { return round16(tp * g.CW) + 2 * ((g.L + 2 + 7) & ~7) + 4 * tp; }
    int ns4() const { return (g.S + 3) / 4; }
    int copyf_raw(int tp) const { return round16(16 + tp * g.CW + 4 * g.n + 16); }
    int copyf_lds(int tp) const { return copyf_raw(tp) + round16(tp * g.L) + 4 * tp + tp + g.T + 16; }

    int begin(int kernel, hipStream_t s, hipEvent_t* stop) {
        *stop = nullptr;
        if (!timing) return FEC_OK;
        EventPair e{kernel, nullptr, nullptr};
        HIP_TRY(hipEventCreate(&e.a));
        HIP_TRY(hipEventCreate(&e.b));
        HIP_TRY(hipEventRecord(e.a, s));
        events.push_back(e);
        *stop = e.b;
        return FEC_OK;
    }
    int end(hipEvent_t stop, hipStream_t s) {
        if (stop) HIP_TRY(hipEventRecord(stop, s));
        return FEC_OK;
    }
    // A launch whose timing events (when on) are bound to the dispatch itself (hipExtLaunchKernel's
    // start / stop events) rather than recorded around it as separate stream packets: the pair then
    // brackets the kernel, not the queue's gap in front of it (tools/ubench/event_timing.hip).
    int launch(int kernel, const void* fn, dim3 grid, dim3 block, void** args, size_t lds, hipStream_t s) {
        if (!timing) {
            HIP_TRY(hipLaunchKernel(fn, grid, block, args, lds, s));
            return FEC_OK;
        }
        EventPair e{kernel, nullptr, nullptr};
        HIP_TRY(hipEventCreate(&e.a));
        HIP_TRY(hipEventCreate(&e.b));
        events.push_back(e);
        HIP_TRY(hipExtLaunchKernel(fn, grid, block, args, lds, s, e.a, e.b, 0));
        return FEC_OK;
    }
};

namespace {

int codec_init(fec_codec* c, int max_payload, int T, int B, int N) {
    c->g = Geometry::make(max_payload, T, B, N);
    const Geometry& g = c->g;
    // n <= 17: decode rules tabulated per (window, erasure mask); n up to 31: computed on demand
    // (host) and by the planner's wave (device)
    if (g.L > kMaxPayload || g.B < g.N || g.n > fec::kMaxN - 1) return FEC_ERR_ARG;
    c->G = fec::make_generator(T, B, N);
    c->rules = fec::shared_decode_rules(T, B, N);
    const fec::Field& F = fec::field();

    // Per parity coefficient: the three register tables of gf_mul4 plus a non-zero flag.
    const std::vector<uint32_t> ptab = fec::parity_mul_tables(c->G, g.k, g.n);
    HIP_TRY(hipMalloc(&c->d_ptab, ptab.size() * 4));
    HIP_TRY(hipMemcpy(c->d_ptab, ptab.data(), ptab.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&c->d_rules, std::max<size_t>(16, c->rules->table.size())));
    HIP_TRY(hipMemcpy(c->d_rules, c->rules->table.data(), c->rules->table.size(), hipMemcpyHostToDevice));
    c->plan_fast = fec::fec_plan_fast_kernel_for(g.k, g.n - g.k);
    if (c->plan_fast) {
        // sel bytes unchanged; coefficient bytes (and padding) -> log2, 0 -> 0xff
        std::vector<uint8_t> lt(c->rules->table);
        const int ES = c->rules->entry_bytes;
        for (size_t e = 0; e + ES <= lt.size(); e += ES)
            for (int o = g.k; o < ES; ++o) lt[e + o] = lt[e + o] ? F.log[lt[e + o]] : 0xff;
        HIP_TRY(hipMalloc(&c->d_rules_log, std::max<size_t>(16, lt.size())));
        HIP_TRY(hipMemcpy(c->d_rules_log, lt.data(), lt.size(), hipMemcpyHostToDevice));
    }
    std::vector<int64_t> wb(c->rules->w_base.begin(), c->rules->w_base.end());
    HIP_TRY(hipMalloc(&c->d_wbase, wb.size() * 8));
    HIP_TRY(hipMemcpy(c->d_wbase, wb.data(), wb.size() * 8, hipMemcpyHostToDevice));
    uint8_t gf[768];
    std::memcpy(gf, F.exp, 512);
    std::memcpy(gf + 512, F.log, 256);
    HIP_TRY(hipMalloc(&c->d_gf, 768));
    HIP_TRY(hipMemcpy(c->d_gf, gf, 768, hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&c->d_G, c->G.size()));
    HIP_TRY(hipMemcpy(c->d_G, c->G.data(), c->G.size(), hipMemcpyHostToDevice));
    const std::vector<uint8_t> rst = fec::build_resync_states(g, *c->rules);
    HIP_TRY(hipMalloc(&c->d_rstate, rst.size()));
    HIP_TRY(hipMemcpy(c->d_rstate, rst.data(), rst.size(), hipMemcpyHostToDevice));

    // Largest power-of-two tiles (<= 64 packets) that fit the LDS budget.
    for (int tp = 64; tp >= 1; tp >>= 1)
        if (c->enc_lds(tp) <= kLdsBudget) {
            c->enc_tp = tp;
            break;
        }
    for (int tp = 64; tp >= 1; tp >>= 1)
        if (c->copy_lds(tp) <= kLdsBudget) {
            c->copy_tp = tp;
            break;
        }
    if (!c->enc_tp || !c->copy_tp) return FEC_ERR_ARG;
    // tuning overrides of the specialised kernels' largest tile (power of two, 8..64)
    auto tile_cap = [](const char* name) {
        const char* v = std::getenv(name);
        const int t = v ? std::atoi(v) : 64;
        return (t >= 8 && t <= 64) ? t : 64;
    };
    {
        int dev = 0;
        HIP_TRY(hipGetDevice(&dev));
        HIP_TRY(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if ((g.L & 3) == 0 && g.n - g.k >= 0) {
        const fec::TileGeom tg = fec::tile_geometry(g.k, g.n - g.k, g.L);
        if (tg.ok) c->tile_kernel = fec::fec_encode_tile_kernel_for(g.k, g.n - g.k, g.L);
        if (c->tile_kernel) {
            c->tile_lds = tg.lds;
            c->tile_lds_len = tg.lds_len;
            c->tile_ppw = tg.PPW;
            c->tile_off[0] = tg.off_in;
            c->tile_off[1] = tg.in_bytes;
            c->tile_off[2] = tg.off_pw;
            c->tile_off[3] = tg.off_q;
            c->tile_off[4] = tg.off_out;
            c->tile_off[5] = tg.off_len;
            c->tile_off[6] = tg.ngl;
            c->tile_off[7] = tg.nso;
            c->tile_off[8] = tg.off_scratch;
        }
        if (c->tile_kernel) {
            HIP_TRY(hipFuncSetAttribute(c->tile_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, c->tile_lds_len));
            int per_cu = 0;
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, c->tile_kernel, 256, c->tile_lds));
            c->tile_per_cu = per_cu;
            if (per_cu <= 0) c->tile_kernel = nullptr;
        }
    }
    if ((g.L & 3) == 0) c->copy_fast = fec::fec_copy_fast_kernel_for(g.k, g.n - g.k);
    // The copy stages its whole tile, converts, then stores (no overlap inside a workgroup), so
    // smaller tiles with more resident workgroups per CU overlap better: at (10,3,3) 32 packets
    // (23 KB LDS) take 135 us per 1M packets against 148 us at 64 and 154 us at 16
    // (profiles/r01/decode_diag/copy_tile_ab.txt, same-process A/B).
    if (c->copy_fast)
        for (int tp = tile_cap("FEC_COPY_TILE"); tp >= 8; tp >>= 1)
            if (c->copyf_lds(tp) <= (tp == 8 ? kLdsBudget : kCopyLdsBudget)) {
                c->copyf_tp = tp;
                break;
            }
    if (!c->copyf_tp) c->copy_fast = nullptr;
    // experiments (FEC_SIDE_CUS / FEC_SIDE_PRIO): the planner's side stream on a CU subset, or at
    // the lowest / highest stream priority
    const char* side_cus = std::getenv("FEC_SIDE_CUS");
    const char* side_prio = std::getenv("FEC_SIDE_PRIO");
    if (side_cus && std::atoi(side_cus) > 0) {
        int dev = 0, cus = 0;
        HIP_TRY(hipGetDevice(&dev));
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        const int want = std::min(cus, std::atoi(side_cus));
        std::vector<uint32_t> mask((cus + 31) / 32, 0u);
        for (int i = 0; i < want; ++i) {
            const int cu = static_cast<int>(static_cast<int64_t>(i) * cus / want);
            mask[cu / 32] |= 1u << (cu % 32);
        }
        HIP_TRY(hipExtStreamCreateWithCUMask(&c->side, static_cast<uint32_t>(mask.size()), mask.data()));
    } else if (side_prio) {
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIP_TRY(hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking,
                                            std::strcmp(side_prio, "high") == 0 ? greatest : least));
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    }
    HIP_TRY(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    return FEC_OK;
}

struct WsLayout {
    size_t counters, erased, src_d, rec_list, sym_ok, coef, work, dups, keys, reps_tr, total;
    int tbits;
};

WsLayout ws_layout(const Geometry& g, int64_t P) {
    auto up = [](size_t v) { return (v + 255) & ~size_t(255); };
    WsLayout w;
    w.counters = 0;
    w.erased = up(64);
    w.src_d = w.erased + up(static_cast<size_t>(P) * 4);
    w.rec_list = w.src_d + up(static_cast<size_t>(P) * 4);
    w.sym_ok = w.rec_list + up(static_cast<size_t>(P) * 8);
    w.coef = w.sym_ok + up(static_cast<size_t>(P) * g.k);
    // episode starts are >= T+2 packets apart
    const size_t maxep = static_cast<size_t>(P) / static_cast<size_t>(g.T + 2) + 2;
    w.tbits = 8;
    while ((size_t(1) << w.tbits) < 2 * maxep) ++w.tbits;
    w.work = w.coef + up(static_cast<size_t>(P) * g.k * g.n);
    w.dups = w.work + up(maxep * 4);
    w.keys = w.dups + up(maxep * 8);
    w.reps_tr = w.keys + up((size_t(1) << w.tbits) * 8);
    w.total = w.reps_tr + up((size_t(1) << w.tbits) * 4);
    return w;
}

struct Ws {
    int32_t* counters;  // [1] erased outputs, [2] recovered, [6] replayed, [7] duplicates
    int32_t* erased;
    int32_t* src_d;
    int32_t* rec_list;
    uint8_t* sym_ok;
    uint8_t* coef;
    int32_t *work, *dups;
    uint64_t* keys;
    int32_t* reps_tr;
    int tbits;
};

Ws ws_carve(const Geometry& g, int64_t P, void* d_ws) {
    const WsLayout w = ws_layout(g, P);
    uint8_t* base = static_cast<uint8_t*>(d_ws);
    auto i32 = [&](size_t o) { return reinterpret_cast<int32_t*>(base + o); };
    return {i32(w.counters), i32(w.erased), i32(w.src_d), i32(w.rec_list), base + w.sym_ok, base + w.coef, i32(w.work),
            i32(w.dups), reinterpret_cast<uint64_t*>(base + w.keys), i32(w.reps_tr), w.tbits};
}


int launch_encode_tile(fec_codec* c, const uint8_t* d_payload, const int32_t* d_len, int64_t history,
                       int64_t P, uint8_t* d_cw, int32_t* d_cwlen, hipStream_t s) {
    const Geometry& g = c->g;
    history = std::min<int64_t>(std::max<int64_t>(0, history), g.n - 1);
    const int R = 4 * c->tile_ppw;
    // 32-bit buffer offsets: batches beyond 2 GB go in chunks of whole tiles (each chunk sees the
    // n-1 rows in front of it as history; the chunk start stays 16-byte aligned in the output)
    const int64_t max_rows = ((int64_t(0x7fffffff) - 65536) / std::max(g.L, g.CW) - g.n) / R * R;
    if (history + P > max_rows) {
        const int64_t chunk = max_rows - R;
        for (int64_t r = 0; r < P; r += chunk) {
            const int64_t h = std::min<int64_t>(history + r, g.n - 1);
            if (int st = launch_encode_tile(c, d_payload + r * g.L, d_len ? d_len + r : nullptr, h,
                                            std::min(chunk, P - r), d_cw + r * g.CW, d_cwlen ? d_cwlen + r : nullptr, s))
                return st;
        }
        return FEC_OK;
    }
    fec::EncTileArgs a;
    a.payload_base = d_payload - history * g.L;
    a.len_base = d_len ? d_len - history : nullptr;
    a.payload_bytes = static_cast<int>((history + P) * g.L);
    a.len_bytes = static_cast<int>((history + P) * 4);
    a.history = static_cast<int>(history);
    a.P = static_cast<int>(P);
    a.cw = d_cw;
    a.cw_bytes = static_cast<int>(P * g.CW);
    a.cw_len = d_cwlen;
    a.ptab = c->d_ptab;
    a.L = g.L;
    a.CW = g.CW;
    a.NS4 = c->ns4();
    a.PPW = c->tile_ppw;
    a.rem = g.S - 4 * (a.NS4 - 1);
    a.nvl = g.L / 4 - g.k * (a.NS4 - 1);
    const int64_t ntiles = (P + R - 1) / R;
    // one wave of resident workgroups, each a contiguous run of tiles (plus the tile in front)
    int64_t slots = static_cast<int64_t>(std::max(1, c->cus)) * c->tile_per_cu;
    if (const char* v = std::getenv("FEC_TILE_WPC"))
        slots = static_cast<int64_t>(std::max(1, c->cus)) * std::max(1, std::min(c->tile_per_cu, std::atoi(v)));
    const int64_t tpw = (ntiles + slots - 1) / slots;
    a.tiles_per_wg = static_cast<int>(tpw);
    a.ntiles = static_cast<int>(ntiles);
    a.off_in = c->tile_off[0];
    a.in_bytes = c->tile_off[1];
    a.off_pw = c->tile_off[2];
    a.off_q = c->tile_off[3];
    a.off_out = c->tile_off[4];
    a.off_len = c->tile_off[5];
    a.ngl = c->tile_off[6];
    a.nso = c->tile_off[7];
    a.off_scratch = c->tile_off[8];
    a.dbg = 0;
#ifdef FEC_ABLATION_BUILD
    // timing ablations (work skipped, codewords wrong by design): only in a diagnostic build,
    // `make EXTRA=-DFEC_ABLATION_BUILD OUT=... BUILD=...`; the product library ignores FEC_TILE_DBG
    if (const char* v = std::getenv("FEC_TILE_DBG")) a.dbg = std::atoi(v);
#endif
    a.seg = nullptr;
    a.cur_rows = a.old_rows = nullptr;
    a.cur_len = a.old_len = nullptr;
    a.W = 0;
    // bit 0: non-temporal codeword stores, bit 1: non-temporal payload loads.  Default 2: the
    // payload rows are read once; 0.2983 - 0.3015 vs 0.3058 - 0.3088 ms per step, encoder 141 - 143
    // vs 145 us (three alternations in one process, profiles/r05/headline/r05zz_tile_nt_ab.txt);
    // non-temporal codeword stores (bit 0) slow the encoder to 170 - 177 us (the copy reads them next)
    a.nt = 2;
    if (const char* v = std::getenv("FEC_TILE_NT")) a.nt = std::atoi(v) & 3;
    const int64_t blocks = (ntiles + tpw - 1) / tpw;
    void* args[] = {&a};
    return c->launch(FEC_KERNEL_ENCODE, c->tile_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), args,
                     d_len ? c->tile_lds_len : c->tile_lds, s);
}

int launch_encode(fec_codec* c, const uint8_t* d_payload, const int32_t* d_len, int64_t history,
                  int64_t P, uint8_t* d_cw, int32_t* d_cwlen, hipStream_t s) {
    if (P <= 0) return FEC_OK;
    {
        const bool tile_ok = c->tile_kernel && (reinterpret_cast<uintptr_t>(d_payload) & 3) == 0 &&
                             (reinterpret_cast<uintptr_t>(d_cw) & 15) == 0;
        if (c->encode_path == 5 && !tile_ok) return FEC_ERR_ARG;
        if (tile_ok && (c->encode_path == 0 || c->encode_path == 5))
            return launch_encode_tile(c, d_payload, d_len, history, P, d_cw, d_cwlen, s);
    }
    if (c->encode_path != 0 && c->encode_path != 1) return FEC_ERR_ARG;
    const Geometry& g = c->g;
    fec::EncArgs a;
    a.payload = d_payload;
    a.len = d_len;
    a.history = std::max<int64_t>(0, history);
    a.P = P;
    a.cw = d_cw;
    a.cw_len = d_cwlen;
    a.ptab = c->d_ptab;
    a.L = g.L;
    a.k = g.k;
    a.n = g.n;
    a.S = g.S;
    a.CW = g.CW;
    a.SP = (g.S + 3) & ~3;
    a.TP = c->enc_tp;
    a.ROWS = a.TP + g.n - 1;
    a.plane = a.ROWS * a.SP;
    a.xin_bytes = round16(g.k * a.plane);
    a.xout_bytes = round16(a.TP * g.CW);
    const int64_t blocks = (P + a.TP - 1) / a.TP;
    if (blocks > 0x7fffffff) return FEC_ERR_ARG;
    hipEvent_t stop;
    if (int st = c->begin(FEC_KERNEL_ENCODE, s, &stop)) return st;
    hipLaunchKernelGGL(fec::fec_encode_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256),
                       c->enc_lds(a.TP), s, a);
    HIP_TRY(hipGetLastError());
    return c->end(stop, s);
}

// The planner's counters (16 words) and shape hash table zeroed in one launch (two runtime fills
// before: 6 us each, on the side stream beside the copy).
__global__ __launch_bounds__(256) void fec_ws_reset_kernel(int32_t* counters, uint64_t* keys, int64_t nkeys) {
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (tid < 16) counters[tid] = 0;
    for (int64_t i = tid; i < nkeys; i += static_cast<int64_t>(gridDim.x) * 256) keys[i] = 0;
}

int check_ws(fec_codec* c, int64_t P, void* d_ws, size_t ws_bytes) {
    if (P > 0x7fffffffLL) return FEC_ERR_ARG;
    if (!d_ws || ws_bytes < ws_layout(c->g, P).total) return FEC_ERR_WORKSPACE;
    return FEC_OK;
}

// Erasure-pattern-only half of the decode: two launches.  fec_episode_kernel finds the resync
// points, the loss episodes and their shapes and lists the erased outputs; the plan kernel replays
// one episode per shape per diagonal and points the other episodes' erased outputs at their
// representative's rows.
int launch_plan(fec_codec* c, const uint8_t* d_er, int64_t P, void* d_ws, size_t ws_bytes,
                hipStream_t s) {
    const Geometry& g = c->g;
    const int64_t Pout = P - g.T;
    if (Pout <= 0) return FEC_OK;
    if (int st = check_ws(c, P, d_ws, ws_bytes)) return st;
    const Ws w = ws_carve(g, P, d_ws);
    const bool fast_ok = c->plan_fast && P < (int64_t(1) << 31) - 1024;
    if (c->plan_path == 2 && !fast_ok) return FEC_ERR_ARG;
    if (g.T >= 64) return FEC_ERR_ARG;  // fec_episode_kernel's resync look-back is one 64-packet word
    {
        const int64_t nkeys = int64_t(1) << w.tbits;
        const int64_t rb = std::max<int64_t>(1, std::min<int64_t>((nkeys + 255) / 256, 256));
        hipLaunchKernelGGL(fec_ws_reset_kernel, dim3(static_cast<unsigned>(rb)), dim3(256), 0, s, w.counters, w.keys, nkeys);
        HIP_TRY(hipGetLastError());
        c->compact_fresh = true;  // counters[2] (the compaction's) is zero until the next compaction
    }
    hipEvent_t stop;
    if (int st = c->begin(FEC_KERNEL_DEC_SCAN, s, &stop)) return st;
    fec::EpisodeArgs ea;
    ea.er = d_er;
    ea.P = P;
    ea.Pout = Pout;
    ea.T = g.T;
    ea.tbits = w.tbits;
    ea.dedup = c->dedup;
    ea.counters = w.counters;
    ea.erased = w.erased;
    ea.src_d = w.src_d;
    ea.work = w.work;
    ea.dups = w.dups;
    ea.keys = w.keys;
    ea.reps_tr = w.reps_tr;
    ea.stamps = (c->stamp_kernel == FEC_KERNEL_DEC_SCAN) ? c->d_stamps : nullptr;
    // a wave per 1024 packets (fec_shapes.hip), at most FEC_EPISODE_GRID waves (A/B switch)
    // one wave per CU: beside the headline copy, 977 waves at 1 M packets took its CUs (0.3224 vs
    // 0.3066 ms per step with 245; 384: 0.3000 - 0.3015 vs 0.2987 - 0.2992, profiles/r06/r06u, r06w)
    int64_t egrid = 256;
    if (const char* v = std::getenv("FEC_EPISODE_GRID")) egrid = std::max(1, std::atoi(v));
    const int64_t sblocks = std::min<int64_t>((P + 1023) / 1024, egrid);
    hipLaunchKernelGGL(fec::fec_episode_kernel, dim3(static_cast<unsigned>(sblocks)), dim3(64), 0, s, ea);
    HIP_TRY(hipGetLastError());
    if (int st = c->end(stop, s)) return st;

    fec::PlanArgs pa;
    pa.er = d_er;
    pa.P = P;
    pa.Pout = Pout;
    pa.rules = c->d_rules;
    pa.G = c->d_G;
    for (int i = 0; i <= fec::kPlanMaxN; ++i)
        pa.wbase[i] = (i < static_cast<int>(c->rules->w_base.size())) ? c->rules->w_base[i] : -1;
    pa.gf = c->d_gf;
    pa.ES = c->rules->entry_bytes;
    pa.k = g.k;
    pa.n = g.n;
    pa.T = g.T;
    pa.counters = w.counters;
    pa.work = w.work;
    pa.dups = w.dups;
    pa.keys = w.keys;
    pa.reps_tr = w.reps_tr;
    pa.src_d = w.src_d;
    pa.rstate = c->d_rstate;
    pa.rs_bytes = fec::resync_state_bytes(g);
    pa.sym_ok = w.sym_ok;
    pa.coef = w.coef;
    if (int st = c->begin(FEC_KERNEL_DEC_PLAN, s, &stop)) return st;
    // The work lists live on the device: (episode, diagonal) replays of one episode per shape
    // (41 x 11 at (10,3,3) on bin/erasure.bin) and one item per duplicate episode.  Graph-replayed
    // plan beside the copy: 8192 / 512 workgroups 175 / 169 us (tools/graph_parts.py).
    int pgrid = 1024;
    if (const char* v = std::getenv("FEC_PLAN_GRID")) pgrid = std::max(1, std::atoi(v));
    if (fast_ok && c->plan_path != 1) {
        pa.rules = c->d_rules_log;
        void* args[] = {&pa};
        HIP_TRY(hipLaunchKernel(c->plan_fast, dim3(pgrid), dim3(64), args, 0, s));
    } else {
        const int plan_lds = 768 + g.n * g.n + 2 * g.k * g.n + 32 * 16 + 32 * 32 + g.k * (1 + g.n);
        hipLaunchKernelGGL(fec::fec_plan_kernel, dim3(pgrid), dim3(64), plan_lds, s, pa);
    }
    HIP_TRY(hipGetLastError());
    return c->end(stop, s);
}

// The two-tiles-per-workgroup copy for this codec, or null: the one test launch_copy and
// fec_codec_info both use (nt = the copy's non-temporal loads, which the paired kernel needs).
const void* copy_pair_kernel(const fec_codec* c, bool nt) {
    const char* pv = std::getenv("FEC_COPY_PAIR");
    if ((pv && pv[0] == '0') || !nt || !c->copy_fast) return nullptr;
    if (16 + c->copyf_tp * c->g.CW + 16 > 6 * 16 * 256) return nullptr;  // the stage of one tile in registers
    return fec::fec_copy_pair_kernel_for(c->g.k, c->g.n - c->g.k);
}

int launch_copy(fec_codec* c, const uint8_t* d_cw, const uint8_t* d_er, int64_t P, uint8_t* d_out,
                int32_t* d_outlen, hipStream_t s, bool skip_erased = false) {
    const Geometry& g = c->g;
    const int64_t Pout = P - g.T;
    if (Pout <= 0) return FEC_OK;
    if (c->copy_path != 0 && c->copy_path != 1 && c->copy_path != 2) return FEC_ERR_ARG;
    const bool fast_ok = c->copy_fast && (reinterpret_cast<uintptr_t>(d_out) & 3) == 0;
    if (c->copy_path == 2 && !fast_ok) return FEC_ERR_ARG;
    if (fast_ok && c->copy_path != 1) {
        fec::CopyFastArgs fa;
        fa.cw = d_cw;
        fa.er = d_er;
        fa.P = P;
        fa.Pout = Pout;
        fa.out = d_out;
        fa.out_len = d_outlen;
        fa.L = g.L;
        fa.CW = g.CW;
        fa.NS4 = c->ns4();
        fa.T = g.T;
        fa.TP = c->copyf_tp;
        fa.raw_bytes = c->copyf_raw(fa.TP);
        fa.out_bytes = round16(fa.TP * g.L);
        fa.stamps = (c->stamp_kernel == FEC_KERNEL_DEC_COPY) ? c->d_stamps : nullptr;
        fa.skip_erased = skip_erased ? 1 : 0;
        // non-temporal codeword loads and payload stores: 0.318 vs 0.338 ms per bench step
        // (tools/step_ab.py, same process, profiles/r02/decode_diag/copy_nt_ab.txt)
        fa.nt = 1;
        if (const char* v = std::getenv("FEC_COPY_NT")) fa.nt = std::atoi(v) ? 1 : 0;
        // (Tried: 32 bytes of LDS padding after every 16 tile rows, which gives the 32 lanes of a
        // ds_read_b32 group distinct banks -- conflict cycles 3.81 M -> 31 k per launch -- but the
        // padded staging made the step 2.2 % slower in the same process, 0.3228 vs 0.3157 ms:
        // profiles/r03/r03v_copy_row_pad_*.txt.  2-way conflicts cost one LDS cycle per 32-lane
        // group; the copy is bound by its HBM traffic and load latency, not by the LDS.)
        // two tiles per workgroup, the second one's loads in flight while the first is converted
        // (copy_pair_kernel: when the stage of one tile fits the registers): 0.3055 vs 0.3126 ms per
        // step, copy 143.6 vs 151.5 us in the step (profiles/r05/headline/r05zu_copy_pair_ab.txt);
        // FEC_COPY_PAIR=0: one tile per workgroup
        const void* pk = copy_pair_kernel(c, fa.nt != 0);
        const int64_t tiles = (Pout + fa.TP - 1) / fa.TP;
        const int64_t blocks = pk ? (tiles + 1) / 2 : tiles;
        // 256 threads (one per (packet, group) item of the tile rounded up to waves, 320 at (10,3,3),
        // measured slower in the step: 0.3402 vs 0.3235 ms, profiles/r03/r03y_copy_threads_ab.txt)
        const int nthr = 256;
        void* args[] = {&fa};
        return c->launch(FEC_KERNEL_DEC_COPY, pk ? pk : c->copy_fast, dim3(static_cast<unsigned>(blocks)), dim3(nthr),
                         args, c->copyf_lds(fa.TP), s);
    }
    fec::CopyArgs ca;
    ca.cw = d_cw;
    ca.er = d_er;
    ca.P = P;
    ca.Pout = Pout;
    ca.out = d_out;
    ca.out_len = d_outlen;
    ca.L = g.L;
    ca.k = g.k;
    ca.n = g.n;
    ca.S = g.S;
    ca.CW = g.CW;
    ca.T = g.T;
    ca.TP = c->copy_tp;
    ca.cwt_bytes = round16(ca.TP * g.CW);
    const int64_t cblocks = (Pout + ca.TP - 1) / ca.TP;
    hipEvent_t stop;
    if (int st = c->begin(FEC_KERNEL_DEC_COPY, s, &stop)) return st;
    hipLaunchKernelGGL(fec::fec_copy_kernel, dim3(static_cast<unsigned>(cblocks)), dim3(256),
                       c->copy_lds(ca.TP), s, ca);
    HIP_TRY(hipGetLastError());
    return c->end(stop, s);
}

// Recovered packets -> rec_list (fec_compact_kernel), on `s` after the plan.
int launch_compact(fec_codec* c, int64_t P, uint8_t* d_out, int32_t* d_outlen, void* d_ws, size_t ws_bytes,
                   hipStream_t s, int64_t row_off = 0, bool zero_lost = false) {
    const Geometry& g = c->g;
    if (P - g.T <= 0) return FEC_OK;
    if (int st = check_ws(c, P, d_ws, ws_bytes)) return st;
    const Ws w = ws_carve(g, P, d_ws);
    fec::CompactArgs ca;
    ca.counters = w.counters;
    ca.erased = w.erased;
    ca.src_d = w.src_d;
    ca.sym_ok = w.sym_ok;
    ca.k = g.k;
    ca.rec_list = w.rec_list;
    // the copy writes every row (zero rows and length 0 for erased packets); recovered rows are
    // overwritten by the recovery, which runs after it
    ca.zero_lost = zero_lost ? 1 : 0;
    ca.out = d_out;
    ca.out_len = d_outlen;
    ca.L = g.L;
    ca.row_off = row_off;
    if (!c->compact_fresh)  // a second compaction of one plan starts over
        HIP_TRY(hipMemsetAsync(w.counters + 2, 0, 4, s));
    c->compact_fresh = false;
    hipLaunchKernelGGL(fec::fec_compact_kernel, dim3(256), dim3(256), 0, s, ca);
    HIP_TRY(hipGetLastError());
    return FEC_OK;
}

// Byte half of the erased packets: one wave per recovered packet of rec_list.  `compacted`: the
// list was built on this stream's side already (launch_decode); otherwise it is built here first.
int launch_recover(fec_codec* c, const uint8_t* d_cw, int64_t P, uint8_t* d_out, int32_t* d_outlen,
                   void* d_ws, size_t ws_bytes, hipStream_t s, int64_t row_off = 0, bool compacted = false) {
    const Geometry& g = c->g;
    const int64_t Pout = P - g.T;
    if (Pout <= 0) return FEC_OK;
    if (int st = check_ws(c, P, d_ws, ws_bytes)) return st;
    if (!compacted)
        if (int st = launch_compact(c, P, d_out, d_outlen, d_ws, ws_bytes, s, row_off)) return st;
    const Ws w = ws_carve(g, P, d_ws);
    fec::RecArgs ra;
    ra.cw = d_cw;
    ra.P = P;
    ra.Pout = Pout;
    ra.counters = w.counters;
    ra.rec_list = w.rec_list;
    ra.coef = w.coef;
    ra.gf = c->d_gf;
    ra.out = d_out;
    ra.out_len = d_outlen;
    ra.L = g.L;
    ra.k = g.k;
    ra.n = g.n;
    ra.S = g.S;
    ra.CW = g.CW;
    hipEvent_t stop;
    if (int st = c->begin(FEC_KERNEL_DEC_RECOVER, s, &stop)) return st;
    ra.row_off = row_off;
    ra.stamps = (c->stamp_kernel == FEC_KERNEL_DEC_RECOVER) ? c->d_stamps : nullptr;
    // the k+n-1 rows a recovered packet reads, staged in LDS when they fit 12 KB per wave
    // (fec_recover_kernel_t's kRecStageChunks)
    const int span = (g.k + g.n - 1) * g.CW + 32;
    ra.stage_bytes = (span <= 12 * 1024 && g.n <= 17) ? ((span + 15) & ~15) : 0;
    if (const char* v = std::getenv("FEC_REC_STAGE")) ra.stage_bytes = std::atoi(v) ? ra.stage_bytes : 0;
    // a wave per recovered packet: up to 4096 waves
    const unsigned rgrid = static_cast<unsigned>(std::min<int64_t>((Pout + 3) / 4, 1024));
    const int maxn = g.n <= 17 ? 17 : 32;
    const int lds = fec::recover_lds_bytes(maxn, ra.stage_bytes);
    if (g.n > 17)
        hipLaunchKernelGGL((fec::fec_recover_kernel_t<32, false>), dim3(rgrid), dim3(256), lds, s, ra);
    else if (ra.stage_bytes)
        hipLaunchKernelGGL((fec::fec_recover_kernel_t<17, true>), dim3(rgrid), dim3(256), lds, s, ra);
    else
        hipLaunchKernelGGL((fec::fec_recover_kernel_t<17, false>), dim3(rgrid), dim3(256), lds, s, ra);
    HIP_TRY(hipGetLastError());
    return c->end(stop, s);
}

// Full decode on `s`: the erasure-only plan runs on the codec's side stream concurrently with the
// systematic copy, joined before the recovery pass (fork/join through events, capturable).
// FEC_RECOVER_BESIDE=1 (A/B switch, off by default): the recovery on the side stream behind the
// planner chain, beside a copy that leaves the erased rows alone (the compaction zeroes the lost
// ones).  Slower wherever it was measured: the headline step 0.3157 - 0.3163 vs 0.3103 - 0.3114 ms,
// config 3 (360 000 packets, whose 56 us copy is shorter than the ~100 us chain) 0.1253 vs 0.1235 ms
// per decode (profiles/r06/r06v, r06w; round 3: profiles/r03/r03y_recover_beside_ab.txt).
bool recover_beside(const fec_codec* c, const uint8_t* d_out) {
    // only the specialised copies leave erased rows alone (fec_copy_fast.hip, skip_erased)
    if (!c->copy_fast || c->copy_path == 1 || (reinterpret_cast<uintptr_t>(d_out) & 3) != 0) return false;
    const char* v = std::getenv("FEC_RECOVER_BESIDE");
    return v && v[0] == '1';
}

int launch_decode(fec_codec* c, const uint8_t* d_cw, const uint8_t* d_er, int64_t P, uint8_t* d_out,
                  int32_t* d_outlen, void* d_ws, size_t ws_bytes, hipStream_t s) {
    if (P - c->g.T <= 0) return FEC_OK;
    if (int st = check_ws(c, P, d_ws, ws_bytes)) return st;
    HIP_TRY(hipEventRecord(c->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(c->side, c->ev_fork, 0));
    if (int st = launch_plan(c, d_er, P, d_ws, ws_bytes, c->side)) return st;
    if (recover_beside(c, d_out)) {
        if (int st = launch_compact(c, P, d_out, d_outlen, d_ws, ws_bytes, c->side, 0, true)) return st;
        if (int st = launch_recover(c, d_cw, P, d_out, d_outlen, d_ws, ws_bytes, c->side, 0, true)) return st;
        HIP_TRY(hipEventRecord(c->ev_join, c->side));
        if (int st = launch_copy(c, d_cw, d_er, P, d_out, d_outlen, s, true)) return st;
        HIP_TRY(hipStreamWaitEvent(s, c->ev_join, 0));
        return FEC_OK;
    }
    if (int st = launch_compact(c, P, d_out, d_outlen, d_ws, ws_bytes, c->side)) return st;
    HIP_TRY(hipEventRecord(c->ev_join, c->side));
    // The copy writes every row (erased ones as zero rows, length 0); the recovery overwrites the
    // recovered ones after the join.  Rounds 2 and 3 measured the alternatives slower in the step
    // (a copy that leaves erased rows to a recovery running beside it: 0.3198 vs 0.3162 ms,
    // profiles/r03/r03y_recover_beside_ab.txt; the plan beside the encoder; profiles/r02/decode_diag).
    if (int st = launch_copy(c, d_cw, d_er, P, d_out, d_outlen, s)) return st;
    HIP_TRY(hipStreamWaitEvent(s, c->ev_join, 0));
    return launch_recover(c, d_cw, P, d_out, d_outlen, d_ws, ws_bytes, s, 0, true);
}

// Continuing decode (fec_decode_stream_push): the next P packets of a stream whose earlier packets
// were pushed before.  The decoder state at the first packet still owed an output depends only on
// the erasure pattern from the start of the episode it lies in, so the decode restarts, as a fresh
// decoder, at a cut c <= that packet where the reference decoder is on its fast path and stays
// there for T more packets (no erasure in [c-T-1, c+T]): from c on a fresh FEC_Decoder and the
// stream's decoder agree (Decoder.cpp:77-133: the fast path reads only the stored codeword, a
// resync replays the last T codewords, which lie after c).  The plan covers [c, end); the copy
// and the recovery write only the rows [next_out, end-T).
int launch_decode_stream(fec_codec* c, fec_decode_stream* st, const uint8_t* d_cw, const uint8_t* d_er,
                         const uint8_t* h_er, int64_t P, int64_t history, uint8_t* d_out, int32_t* d_outlen,
                         int64_t* n_out, void* d_ws, size_t ws_bytes, hipStream_t s) {
    const int T = c->g.T;
    const int64_t s0 = st->consumed;                 // absolute index of the first new packet
    const int64_t next_out = std::max<int64_t>(0, s0 - T);
    const int64_t end = s0 + P;
    const int64_t avail = s0 - history;              // first packet in memory
    *n_out = 0;
    if (P < 0 || history < 0 || avail < 0) return FEC_ERR_ARG;
    if (end - T <= next_out) {  // nothing to output yet (stream shorter than T so far)
        st->consumed = end;
        return FEC_OK;
    }
    if (s0 - next_out > history) return FEC_ERR_HISTORY;  // the copy reads the T packets before s0
    auto er_at = [&](int64_t x) -> bool { return x >= 0 && x < end && h_er[x - s0] != 0; };
    // largest valid cut c <= next_out whose check window [c-T-1, c+T] is known (or the stream start)
    int64_t cut = -1;
    for (int64_t x = next_out; x >= avail; --x) {
        if (x - T - 1 < avail && x - T - 1 >= 0) break;  // flags in front of x are not in memory
        bool ok = true;
        for (int64_t y = x - T - 1; y <= x + T && ok; ++y) ok = !er_at(y);
        if (ok || x == 0) {
            cut = x;
            break;
        }
    }
    if (cut < 0) return FEC_ERR_HISTORY;
    const int64_t Pp = end - cut;
    if (int st2 = check_ws(c, Pp, d_ws, ws_bytes)) return st2;
    const uint8_t* cw_c = d_cw - (s0 - cut) * c->g.CW;
    const uint8_t* er_c = d_er - (s0 - cut);
    HIP_TRY(hipEventRecord(c->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(c->side, c->ev_fork, 0));
    if (int e = launch_plan(c, er_c, Pp, d_ws, ws_bytes, c->side)) return e;
    if (int e = launch_compact(c, Pp, d_out, d_outlen, d_ws, ws_bytes, c->side, next_out - cut)) return e;
    HIP_TRY(hipEventRecord(c->ev_join, c->side));
    // received rows [next_out, end - T): a copy over packets [next_out, end)
    const int64_t Pc = end - next_out;
    const uint8_t* cw_o = d_cw - (s0 - next_out) * c->g.CW;
    const uint8_t* er_o = d_er - (s0 - next_out);
    if (int e = launch_copy(c, cw_o, er_o, Pc, d_out, d_outlen, s)) return e;
    HIP_TRY(hipStreamWaitEvent(s, c->ev_join, 0));
    if (int e2 = launch_recover(c, cw_c, Pp, d_out, d_outlen, d_ws, ws_bytes, s, next_out - cut, true)) return e2;
    *n_out = end - T - next_out;
    st->consumed = end;
    st->last_cut = cut;
    return FEC_OK;
}

template <class F>
int guarded(F&& f) {
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

}  // namespace

// ------------------------------------------------------------------------------------------
// Streaming objects
// ------------------------------------------------------------------------------------------
// One call per packet is one GPU round trip with no DMA command: the caller's packet is written into a
// host-visible staging row (pinned, coherent, mapped), a staging kernel moves it into the device
// window / ring, the coding kernel writes its result straight into a host-visible result row, one
// stream synchronisation.  Everything the coder needs from earlier packets stays on the device.
// A per-packet coder's resident server (fec_server.hip): its mailbox and whether a launch of it
// may still be running.
struct ServerHost {
    fec::ServerBox* h_box = nullptr;  // pinned, coherent, mapped
    fec::ServerBox* m_box = nullptr;  // its device address
    uint64_t* h_req = nullptr;        // sealed request block (fec_kernels.h), pinned, coherent, mapped
    uint64_t* m_req = nullptr;
    int nunits = 0;                   // its units (the decoder's: with the coefficient units)
    bool on = false;                  // this coder runs on a server (else one launch per call)
    bool live = false;                // a server launch may be running on the coder's stream
    bool slot = false;                // it holds one of the process's persistent-server slots
};

struct fec_encoder {
    std::unique_ptr<fec_codec> codec;
    ServerHost sv;
    bool poisoned = false;         // a failed HIP call left host and device state apart
    int64_t origin = -1;           // seq of the first call (the encoder's creation point)
    int64_t next = 0;              // expected seq
    int res_len_off = 0;           // offset of the trimmed size in the result block (4-aligned)
    hipStream_t s = nullptr;
    uint8_t* d_win = nullptr;      // the n-1 windows in front, a ring by seq % (n-1) (fec_streams layout)
    uint8_t* h_stage = nullptr;    // pinned, coherent: payload row (read by the kernel)
    uint8_t* h_res = nullptr;      // pinned, coherent: codeword (CW) | trimmed size (written by the kernel)
    uint8_t* m_stage = nullptr;    // device addresses of h_stage / h_res
    uint8_t* m_res = nullptr;
    uint8_t* h_done = nullptr;     // pinned, coherent: completion word (ticket of the last finished call)
    uint8_t* m_done = nullptr;
    uint32_t ticket = 0;
    ~fec_encoder();
};

struct fec_decoder {
    static constexpr int RR = 64;  // ring rows (>= T + k)
    std::unique_ptr<fec_codec> codec;
    ServerHost sv;
    std::vector<uint8_t> h_ring;   // server mode: the received codewords, zero-padded (RR x CW; zero
                                   // rows for missing packets) -- the decoder's own copies
    std::vector<uint32_t> req;     // server mode: request words (fields, window rows, coefficients)
    int win_units = 0;             // ceil((k+n-1) * CW / 4)
    bool poisoned = false;         // a failed HIP call left host and device state apart
    std::unique_ptr<fec::StreamPlanner> planner;
    int64_t origin = -1;           // seq of the first call; the planner runs on seq - origin
    int64_t next = 0;
    int res_len_off = 0;
    hipStream_t s = nullptr;
    uint8_t* d_ring = nullptr;     // RR x CW
    uint8_t* d_coef = nullptr;     // k x n coefficients of a recovered packet
    uint8_t* h_cw = nullptr;       // pinned, coherent: CW-byte staging row
    uint8_t* h_coef = nullptr;     // pinned, coherent: k x n (read by the output kernel)
    uint8_t* h_res = nullptr;      // pinned, coherent: payload (L) | length (written by the kernel)
    uint8_t* m_cw = nullptr;       // device addresses of h_cw / h_coef / h_res
    uint8_t* m_coef = nullptr;
    uint8_t* m_res = nullptr;
    uint8_t* h_done = nullptr;     // pinned, coherent: completion word (ticket of the last finished call)
    uint8_t* m_done = nullptr;
    uint32_t ticket = 0;
    ~fec_decoder();
};

namespace {
// The server ends on its stop word; the stream then holds no running launch.
void server_slot_give(ServerHost& sv);
void server_stop(ServerHost& sv, hipStream_t s) {
    if (sv.live && sv.h_box && s) {
        reinterpret_cast<volatile fec::ServerBox*>(sv.h_box)->stop = 1;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        (void)hipStreamSynchronize(s);
        sv.live = false;
    }
    server_slot_give(sv);
}
}  // namespace

fec_encoder::~fec_encoder() {
    server_stop(sv, s);
    if (s) (void)hipStreamDestroy(s);
    if (d_win) (void)hipFree(d_win);
    for (void* p : {static_cast<void*>(h_stage), static_cast<void*>(h_res), static_cast<void*>(h_done),
                    static_cast<void*>(sv.h_box), static_cast<void*>(sv.h_req)})
        if (p) (void)hipHostFree(p);
}

fec_decoder::~fec_decoder() {
    server_stop(sv, s);
    if (s) (void)hipStreamDestroy(s);
    for (void* p : {static_cast<void*>(d_ring), static_cast<void*>(d_coef)})
        if (p) (void)hipFree(p);
    for (void* p : {static_cast<void*>(h_cw), static_cast<void*>(h_coef), static_cast<void*>(h_res),
                    static_cast<void*>(h_done), static_cast<void*>(sv.h_box), static_cast<void*>(sv.h_req)})
        if (p) (void)hipHostFree(p);
}

namespace fec {
namespace {
std::mutex g_err_mu;
char g_err[512] = "";
}  // namespace
int hip_failed(hipError_t e, const char* site) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    std::snprintf(g_err, sizeof(g_err), "%s (%d) at %s", hipGetErrorName(e), static_cast<int>(e), site);
    return FEC_ERR_HIP;
}
}  // namespace fec

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
// The batch encode without the trimmed wire sizes where the kernel can skip them (the runtime-L
// tile kernels and the generic one: fec_relay_vr's batches, whose zero-length gap rows made that
// scan most of their encode); the L-specialised kernels write them to d_cwlen_fallback.
namespace fec {
int encode_batch_nolen(fec_codec* c, const uint8_t* d_payload, const int32_t* d_len, int64_t history, int64_t P,
                       uint8_t* d_cw, int32_t* d_cwlen_fallback, hipStream_t s) {
    if (!c || P < 0 || (P > 0 && (!d_payload || !d_cw || !d_cwlen_fallback))) return FEC_ERR_ARG;
    const bool skip = !c->tile_kernel || c->tile_kernel == fec_encode_tile_kernel_for(c->g.k, c->g.n - c->g.k, 0);
    return launch_encode(c, d_payload, d_len, history, P, d_cw, skip ? nullptr : d_cwlen_fallback, s);
}
}  // namespace fec

extern "C" {

int fec_last_error(char* buf, size_t size) {
    std::lock_guard<std::mutex> lk(fec::g_err_mu);
    const int n = static_cast<int>(std::strlen(fec::g_err));
    if (buf && size) std::snprintf(buf, size, "%s", fec::g_err);
    return n;
}

const char* fec_strerror(int status) {
    switch (status) {
        case FEC_OK: return "ok";
        case FEC_ERR_ARG: return "invalid argument or unsupported (max_payload,T,B,N)";
        case FEC_ERR_HIP: return "HIP runtime error";
        case FEC_ERR_NOMEM: return "out of memory";
        case FEC_ERR_WORKSPACE: return "decode workspace too small";
        case FEC_ERR_SEQUENCE: return "sequence numbers must be consecutive from the first call's";
        case FEC_ERR_HISTORY: return "continuing decode: not enough earlier packets kept in memory";
        default: return "unknown error";
    }
}

int fec_version(void) { return FEC_AMD_ABI_VERSION; }

int fec_codec_create(int max_payload, int T, int B, int N, fec_codec** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<fec_codec> c(new fec_codec());
        if (int st = codec_init(c.get(), max_payload, T, B, N)) return st;
        *out = c.release();
        return FEC_OK;
    });
}

int fec_codec_destroy(fec_codec* codec) {
    delete codec;
    return FEC_OK;
}

int fec_codec_geometry(const fec_codec* c, int* k, int* n, int* S, int* CW) {
    if (!c) return FEC_ERR_ARG;
    if (k) *k = c->g.k;
    if (n) *n = c->g.n;
    if (S) *S = c->g.S;
    if (CW) *CW = c->g.CW;
    return FEC_OK;
}

int fec_codec_generator(const fec_codec* c, uint8_t* G) {
    if (!c || !G) return FEC_ERR_ARG;
    std::memcpy(G, c->G.data(), c->G.size());
    return FEC_OK;
}

int fec_encode_batch(fec_codec* c, const uint8_t* d_payload, const int32_t* d_len, int64_t history,
                     int64_t P, uint8_t* d_cw, int32_t* d_cwlen, void* stream) {
    if (!c || P < 0 || (P > 0 && (!d_payload || !d_cw || !d_cwlen))) return FEC_ERR_ARG;
    return launch_encode(c, d_payload, d_len, history, P, d_cw, d_cwlen,
                         static_cast<hipStream_t>(stream));
}

size_t fec_decode_workspace_bytes(const fec_codec* c, int64_t P) {
    if (!c || P < 0) return 0;
    return ws_layout(c->g, P).total;
}

int fec_decode_batch(fec_codec* c, const uint8_t* d_cw, const uint8_t* d_er, int64_t P,
                     uint8_t* d_out, int32_t* d_outlen, void* d_ws, size_t ws_bytes, void* stream) {
    if (!c || P < 0) return FEC_ERR_ARG;
    if (P > c->g.T && (!d_cw || !d_er || !d_out || !d_outlen)) return FEC_ERR_ARG;
    return launch_decode(c, d_cw, d_er, P, d_out, d_outlen, d_ws, ws_bytes,
                         static_cast<hipStream_t>(stream));
}

int fec_decode_stream_create(fec_decode_stream** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    return guarded([&] {
        *out = new fec_decode_stream();
        return FEC_OK;
    });
}

int fec_decode_stream_destroy(fec_decode_stream* st) {
    delete st;
    return FEC_OK;
}

int fec_decode_stream_state(const fec_decode_stream* st, int64_t* consumed, int64_t* last_cut) {
    if (!st) return FEC_ERR_ARG;
    if (consumed) *consumed = st->consumed;
    if (last_cut) *last_cut = st->last_cut;
    return FEC_OK;
}

int fec_decode_stream_push(fec_codec* c, fec_decode_stream* st, const uint8_t* d_cw, const uint8_t* d_er,
                           const uint8_t* h_er, int64_t P, int64_t history, uint8_t* d_out, int32_t* d_outlen,
                           int64_t* n_out, void* d_ws, size_t ws_bytes, void* stream) {
    if (!c || !st || !d_cw || !d_er || !h_er || !n_out || !d_out || !d_outlen) return FEC_ERR_ARG;
    return guarded([&] {
        return launch_decode_stream(c, st, d_cw, d_er, h_er, P, history, d_out, d_outlen, n_out, d_ws, ws_bytes,
                                    static_cast<hipStream_t>(stream));
    });
}

int fec_decode_plan(fec_codec* c, const uint8_t* d_er, int64_t P, void* d_ws, size_t ws_bytes,
                    void* stream) {
    if (!c || P < 0 || (P > c->g.T && !d_er)) return FEC_ERR_ARG;
    return launch_plan(c, d_er, P, d_ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int fec_decode_apply(fec_codec* c, const uint8_t* d_cw, const uint8_t* d_er, int64_t P,
                     uint8_t* d_out, int32_t* d_outlen, void* d_ws, size_t ws_bytes, void* stream) {
    if (!c || P < 0) return FEC_ERR_ARG;
    if (P > c->g.T && (!d_cw || !d_er || !d_out || !d_outlen)) return FEC_ERR_ARG;
    if (int st = check_ws(c, P, d_ws, ws_bytes)) return P > c->g.T ? st : FEC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (int st = launch_copy(c, d_cw, d_er, P, d_out, d_outlen, s)) return st;
    return launch_recover(c, d_cw, P, d_out, d_outlen, d_ws, ws_bytes, s);
}

int fec_decode_copy(fec_codec* c, const uint8_t* d_cw, const uint8_t* d_er, int64_t P, uint8_t* d_out,
                    int32_t* d_outlen, void* stream) {
    if (!c || P < 0) return FEC_ERR_ARG;
    if (P > c->g.T && (!d_cw || !d_er || !d_out || !d_outlen)) return FEC_ERR_ARG;
    return launch_copy(c, d_cw, d_er, P, d_out, d_outlen, static_cast<hipStream_t>(stream));
}

int fec_decode_recover(fec_codec* c, const uint8_t* d_cw, int64_t P, uint8_t* d_out,
                       int32_t* d_outlen, void* d_ws, size_t ws_bytes, void* stream) {
    if (!c || P < 0) return FEC_ERR_ARG;
    if (P > c->g.T && (!d_cw || !d_out || !d_outlen)) return FEC_ERR_ARG;
    return launch_recover(c, d_cw, P, d_out, d_outlen, d_ws, ws_bytes,
                          static_cast<hipStream_t>(stream));
}

int fec_decode_counters(const void* d_ws, int64_t* episodes, int64_t* recovered, int64_t* lost) {
    if (!d_ws) return FEC_ERR_ARG;
    int32_t h[8];
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(h, d_ws, sizeof(h), hipMemcpyDeviceToHost));
    if (episodes) *episodes = h[6] + h[7];  // every episode is replayed or a duplicate
    if (recovered) *recovered = h[2];
    if (lost) *lost = h[1] - h[2];  // erased outputs that were not recovered
    return FEC_OK;
}

int fec_codec_info(const fec_codec* c, char* buf, size_t size) {
    if (!c || !buf || size == 0) return FEC_ERR_ARG;
    // kernel symbol the encoder launches for a 16-byte aligned payload (rocprofv3 naming)
    char enc[64];
    const int np = c->g.n - c->g.k;
    if (c->tile_kernel && (c->encode_path == 0 || c->encode_path == 5))
        std::snprintf(enc, sizeof(enc), "fec_encode_tile_kernel<%d, %d, %d, false>", c->g.k, np,
                      c->tile_kernel == fec::fec_encode_tile_kernel_for(c->g.k, np, 0) ? 0 : c->g.L);
    else
        std::snprintf(enc, sizeof(enc), "fec_encode_kernel");
    char cpy[64];
    const char* ntv = std::getenv("FEC_COPY_NT");
    const bool pair = copy_pair_kernel(c, !(ntv && !std::atoi(ntv))) != nullptr;
    if (c->copy_fast && c->copy_path != 1 && pair)
        std::snprintf(cpy, sizeof(cpy), "fec_copy_pair_kernel<%d, %d>", c->g.k, np);
    else if (c->copy_fast && c->copy_path != 1)
        std::snprintf(cpy, sizeof(cpy), "fec_copy_fast_kernel<%d, %d>", c->g.k, np);
    else
        std::snprintf(cpy, sizeof(cpy), "fec_copy_kernel");
    std::snprintf(buf, size,
                  "{\"k\": %d, \"n\": %d, \"S\": %d, \"CW\": %d, \"encode_kernel\": \"%s\", "
                  "\"copy_kernel\": \"%s\", \"encode_tile_packets\": %d, \"encode_tile_workgroups_per_cu\": %d, "
                  "\"copy_tile\": %d, \"plan_specialised\": %d}",
                  c->g.k, c->g.n, c->g.S, c->g.CW, enc, cpy, 4 * c->tile_ppw, c->tile_per_cu, c->copyf_tp,
                  c->plan_fast ? 1 : 0);
    return FEC_OK;
}

int fec_decode_plan_stats(const void* d_ws, int64_t* replayed, int64_t* filled) {
    if (!d_ws) return FEC_ERR_ARG;
    int32_t h[8];
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(h, d_ws, sizeof(h), hipMemcpyDeviceToHost));
    if (replayed) *replayed = h[6];
    if (filled) *filled = h[7];
    return FEC_OK;
}

int fec_debug_stamps(fec_codec* c, int kernel, void* d_stamps) {
    if (!c) return FEC_ERR_ARG;
    c->stamp_kernel = d_stamps ? kernel : -1;
    c->d_stamps = static_cast<uint64_t*>(d_stamps);
    return FEC_OK;
}

int fec_codec_set_episode_dedup(fec_codec* c, int on) {
    if (!c) return FEC_ERR_ARG;
    c->dedup = on ? 1 : 0;
    return FEC_OK;
}

int fec_codec_set_plan_path(fec_codec* c, int path) {
    if (!c || path < 0 || path > 2) return FEC_ERR_ARG;
    if (path == 2 && !c->plan_fast) return FEC_ERR_ARG;
    c->plan_path = path;
    return FEC_OK;
}

int fec_codec_set_copy_path(fec_codec* c, int path) {
    if (!c || path < 0 || path > 2) return FEC_ERR_ARG;
    if (path == 2 && !c->copy_fast) return FEC_ERR_ARG;
    c->copy_path = path;
    return FEC_OK;
}

int fec_codec_set_encode_path(fec_codec* c, int path) {
    if (!c || !(path == 0 || path == 1 || path == 5)) return FEC_ERR_ARG;
    if (path == 5 && !c->tile_kernel) return FEC_ERR_ARG;
    c->encode_path = path;
    return FEC_OK;
}

int fec_timing_enable(fec_codec* c, int enable) {
    if (!c) return FEC_ERR_ARG;
    c->timing = enable != 0;
    return FEC_OK;
}

int fec_timing_collect(fec_codec* c, double* total_ms, int64_t* launches) {
    if (!c || !total_ms || !launches) return FEC_ERR_ARG;
    for (int i = 0; i < FEC_KERNEL_COUNT; ++i) {
        total_ms[i] = 0.0;
        launches[i] = 0;
    }
    for (auto& e : c->events) {
        HIP_TRY(hipEventSynchronize(e.b));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, e.a, e.b));
        total_ms[e.kernel] += ms;
        launches[e.kernel] += 1;
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    c->events.clear();
    return FEC_OK;
}

// ---- streaming encoder --------------------------------------------------------------------
namespace {
// Pinned host memory the kernels read and write directly (coherent: never cached in the GPU's L2, so a
// row the host rewrote between calls is seen fresh, and a result row is complete at the stream
// synchronisation).
hipError_t host_mapped(uint8_t** host, uint8_t** dev, size_t bytes) {
    if (hipError_t e = hipHostMalloc(reinterpret_cast<void**>(host), bytes,
                                     hipHostMallocMapped | hipHostMallocCoherent))
        return e;
    std::memset(*host, 0, bytes);
    return hipHostGetDevicePointer(reinterpret_cast<void**>(dev), *host, 0);
}

// End of a streaming call: the call's last kernel stores `ticket` into the host-visible completion
// word after its results; the host polls that word (a stream synchronisation's wake-up costs several
// microseconds more).  A call that takes longer than 20 ms, or FEC_STREAM_SPIN=0, falls back to
// hipStreamSynchronize, which also reports a failed kernel.
hipError_t wait_done(const uint8_t* h_done, uint32_t ticket, hipStream_t s) {
    static const bool spin = [] {
        const char* v = std::getenv("FEC_STREAM_SPIN");
        return !v || std::atoi(v) != 0;
    }();
    if (spin) {
        const volatile uint32_t* w = reinterpret_cast<const volatile uint32_t*>(h_done);
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t i = 1;; ++i) {
            if (*w == ticket) {
                std::atomic_thread_fence(std::memory_order_acquire);
                return hipSuccess;
            }
            if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
            __builtin_ia32_pause();
        }
    }
    return hipStreamSynchronize(s);
}

// Resident servers (fec_server.hip).  FEC_SERVER=0 restores one launch per call.
bool server_enabled() {
    static const bool on = [] {
        const char* v = std::getenv("FEC_SERVER");
        return !v || std::atoi(v) != 0;
    }();
    return on;
}
constexpr int64_t kServerIdleTicks = 5000000;  // 50 ms of the 100 MHz counter without a request

// Persistent servers per process.  A live server occupies its stream's hardware queue until it
// idles out, and a process has few queues (GPU_MAX_HW_QUEUES, 4 by default): streams beyond that
// share queues, and work queued behind a live server waits for it.  Which streams share a queue is
// the runtime's choice, so no two servers are ever live at once: every server launch first stops
// the other live servers (their stop word; they write their state back and end).  At most
// FEC_SERVER_MAX (default 1; 0 = none) coders keep a persistent server; the others serve each call
// with a one-shot launch of the same kernel (idle limit 0: it serves the posted request and exits,
// and the call waits for the launch to end).  A stopped server's coder relaunches it at its next
// call.  A coder gives its slot back at its next call after its server ended, or when it is
// destroyed.
// The coders' streams (the servers and one-shot launches run there) are created with the greatest
// stream priority: the runtime keeps high-priority streams on hardware queues of their own, apart
// from the normal-priority streams of torch, the batched calls and the caller, so a live server never
// holds a launch of those behind it (a plain stream shares one of GPU_MAX_HW_QUEUES queues with the
// others: a 50 ms server held a launch on another stream for 49.9 ms; on a high-priority stream the
// worst of 13 launches, the null stream's included, took 18-23 us, profiles/r05/r05q_queue_prio.txt).
// FEC_CODER_PLAIN_STREAMS=1 (diagnostic) creates them plainly.
hipError_t coder_stream_create(hipStream_t* s) {
    static const bool plain = [] {
        const char* v = std::getenv("FEC_CODER_PLAIN_STREAMS");
        return v && v[0] == '1';
    }();
    if (plain) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

std::atomic<int> g_server_slots{0};
std::mutex g_server_mu;
std::vector<ServerHost*> g_server_live;  // persistent servers launched and not seen ended

int server_slot_cap() {
    static const int cap = [] {
        const char* v = std::getenv("FEC_SERVER_MAX");
        const int c = v ? std::atoi(v) : 1;
        return c < 0 ? 0 : c;
    }();
    return cap;
}
bool server_slot_take(ServerHost& sv) {
    if (sv.slot) return true;
    int c = g_server_slots.load();
    while (c < server_slot_cap())
        if (g_server_slots.compare_exchange_weak(c, c + 1)) {
            sv.slot = true;
            return true;
        }
    return false;
}
void server_unregister(ServerHost& sv) {
    std::lock_guard<std::mutex> lk(g_server_mu);
    g_server_live.erase(std::remove(g_server_live.begin(), g_server_live.end(), &sv), g_server_live.end());
}
void server_slot_give(ServerHost& sv) {
    server_unregister(sv);
    if (sv.slot) {
        g_server_slots.fetch_sub(1);
        sv.slot = false;
    }
}
// At the start of a call: whether this call's server is (or becomes) persistent.
bool server_persistent(ServerHost& sv) {
    if (!sv.live) server_slot_give(sv);
    return sv.live || server_slot_take(sv);
}
// Before a server launch: every other coder's persistent server stops (it writes its state back
// and ends; its coder sees exited = 1 and relaunches at its next call).
void server_stop_others(const ServerHost& self) {
    std::lock_guard<std::mutex> lk(g_server_mu);
    for (ServerHost* o : g_server_live)
        if (o != &self) reinterpret_cast<volatile fec::ServerBox*>(o->h_box)->stop = 1;
    g_server_live.erase(std::remove_if(g_server_live.begin(), g_server_live.end(),
                                       [&](ServerHost* o) { return o != &self; }),
                        g_server_live.end());
    std::atomic_thread_fence(std::memory_order_seq_cst);
}

using ServerLaunch = std::function<hipError_t(uint32_t last, int64_t idle_ticks)>;

hipError_t server_start(ServerHost& sv, uint32_t last, bool persistent, const ServerLaunch& launch) {
    volatile fec::ServerBox* b = sv.h_box;
    server_stop_others(sv);
    b->stop = 0;
    b->exited = 0;
    b->alive = 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (hipError_t e = launch(last, persistent ? kServerIdleTicks : 0)) return e;
    sv.live = true;
    if (persistent) {
        std::lock_guard<std::mutex> lk(g_server_mu);
        if (std::find(g_server_live.begin(), g_server_live.end(), &sv) == g_server_live.end())
            g_server_live.push_back(&sv);
    }
    return hipSuccess;
}

// After reading alive = 0: the server is exiting.  Wait until it revived for this request
// (alive = 1), answered it, or made its exit final (exited = 1: then the launch is drained).
hipError_t server_settle(ServerHost& sv, uint32_t ticket, hipStream_t s, bool* ended) {
    const volatile fec::ServerBox* b = sv.h_box;
    *ended = false;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
        if (b->exited) break;
        if (b->alive || b->done == ticket) return hipSuccess;
        if ((i & 4095) == 0) {
            if (hipError_t e = hipStreamQuery(s); e != hipSuccess && e != hipErrorNotReady) return e;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) break;
        }
        __builtin_ia32_pause();
    }
    // exited = 1 is the launch's last write to the box (its state write-back, if any, goes to device
    // memory and is ordered before the stream's next launch): the box is free without a stream
    // synchronisation.  Only the time limit above falls back to one.
    const hipError_t e = b->exited ? hipSuccess : hipStreamSynchronize(s);
    sv.live = false;
    server_unregister(sv);
    *ended = true;
    return e;
}

// Post request `ticket` (its sealed units are written) and make sure a server serves it.
hipError_t server_post(ServerHost& sv, uint32_t ticket, hipStream_t s, bool persistent, const ServerLaunch& launch) {
    volatile fec::ServerBox* b = sv.h_box;
    if (!sv.live)
        if (hipError_t e = server_start(sv, ticket - 1, persistent, launch)) return e;
    std::atomic_thread_fence(std::memory_order_release);
    b->req = ticket;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (b->alive == 0) {
        bool ended = false;
        if (hipError_t e = server_settle(sv, ticket, s, &ended)) return e;
        if (ended && b->done != ticket)
            if (hipError_t e = server_start(sv, ticket - 1, persistent, launch)) return e;
    }
    return hipSuccess;
}

// The request `words` (n dwords) into the sealed request block from unit `first` on, stamped with
// `ticket`: one 8-byte store per unit, in decreasing order (the server takes a request when the
// units of its head carry the ticket, fec_kernels.h; units written earlier are then visible too).
void server_seal(ServerHost& sv, int first, const uint32_t* words, int n, uint32_t ticket) {
    volatile uint64_t* u = sv.h_req + first;
    const uint64_t tk = static_cast<uint64_t>(ticket) << 32;
    for (int i = n - 1; i >= 0; --i) u[i] = tk | words[i];
}

// Wait for the server's done ticket (in host memory: no PCIe round trip per poll).  A server whose
// exit became final before answering (stopped by another coder's one-shot, or idled out in the
// exit race) is relaunched for the request, a few times at most; a failed launch is reported after
// the stream is drained; ten seconds without an answer are reported as an error.  A one-shot launch
// is drained after its answer.
hipError_t server_wait(ServerHost& sv, uint32_t ticket, hipStream_t s, bool persistent, const ServerLaunch& launch) {
    const volatile fec::ServerBox* b = sv.h_box;
    const auto t0 = std::chrono::steady_clock::now();
    int relaunches = 0;
    for (uint32_t i = 1;; ++i) {
        if (b->done == ticket) {
            std::atomic_thread_fence(std::memory_order_acquire);
            if (!persistent) {
                // a one-shot launch answers, then makes its exit final (exited = 1) as its last
                // write to the box; whatever it does after that (an encoder's state write-back)
                // goes to its own device memory, ordered before the next launch on its stream.
                // So the box is free once exited = 1: no stream synchronisation on the call path.
                for (uint32_t j = 1; !b->exited; ++j) {
                    if ((j & 4095) == 0) {
                        if (hipError_t e = hipStreamQuery(s); e != hipSuccess && e != hipErrorNotReady) return e;
                        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
                            return hipErrorLaunchTimeOut;
                    }
                    __builtin_ia32_pause();
                }
                sv.live = false;
            }
            return hipSuccess;
        }
        if ((i & 1023) == 0) {
            if (b->exited) {  // the server is gone without this request's answer (exited = 1: its last box write)
                std::atomic_thread_fence(std::memory_order_acquire);
                sv.live = false;
                server_unregister(sv);
                if (b->done == ticket) continue;
                if (hipError_t e = hipStreamQuery(s); e != hipSuccess && e != hipErrorNotReady) return e;
                // a server stopped by another coder's launch (its stop word) is contention, not a
                // failure: relaunched without limit (the ten-second bound below still holds); only
                // exits of its own (the idle exit race) count toward the limit
                if (b->stop == 0 && ++relaunches > 8) return hipErrorLaunchFailure;
                if (hipError_t e2 = server_start(sv, ticket - 1, persistent, launch)) return e2;
                continue;
            }
            if (hipError_t e = hipStreamQuery(s); e != hipSuccess && e != hipErrorNotReady) return e;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) return hipErrorLaunchTimeOut;
        }
        __builtin_ia32_pause();
    }
}
}  // namespace

int fec_encoder_create(int max_payload, int T, int B, int N, fec_encoder** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<fec_encoder> e(new fec_encoder());
        fec_codec* c = nullptr;
        if (int st = fec_codec_create(max_payload, T, B, N, &c)) return st;
        e->codec.reset(c);
        const Geometry& g = c->g;
        if (g.k > 16 || g.k * g.n > 16 * 32) return FEC_ERR_ARG;  // fec_streams_encode_kernel's bounds
        e->res_len_off = (g.CW + 3) & ~3;
        HIP_TRY(coder_stream_create(&e->s));
        const size_t wb = static_cast<size_t>(std::max(1, g.n - 1)) * g.S * g.k;
        HIP_TRY(hipMalloc(&e->d_win, wb));
        HIP_TRY(hipMemset(e->d_win, 0, wb));
        HIP_TRY(host_mapped(&e->h_stage, &e->m_stage, (g.L + 3) & ~3));
        HIP_TRY(host_mapped(&e->h_res, &e->m_res, e->res_len_off + 4));
        HIP_TRY(host_mapped(&e->h_done, &e->m_done, 4));
        const int W = std::max(1, g.n - 1), SK = g.S * g.k;
        e->sv.on = server_enabled() && g.CW <= 2048 && g.L <= 1500 && g.k * g.n <= 16 * 32 &&
                   static_cast<int64_t>(W) * SK <= 48 * 1024;
        if (e->sv.on) {
            HIP_TRY(host_mapped(reinterpret_cast<uint8_t**>(&e->sv.h_box), reinterpret_cast<uint8_t**>(&e->sv.m_box),
                                sizeof(fec::ServerBox)));
            e->sv.nunits = fec::kEncReqFields + (g.L + 3) / 4;
            HIP_TRY(host_mapped(reinterpret_cast<uint8_t**>(&e->sv.h_req), reinterpret_cast<uint8_t**>(&e->sv.m_req),
                                sizeof(uint64_t) * e->sv.nunits));
        }
        HIP_TRY(hipDeviceSynchronize());  // the window is zero before the first call's kernel
        *out = e.release();
        return FEC_OK;
    });
}

int fec_encoder_destroy(fec_encoder* e) {
    delete e;
    return FEC_OK;
}

int fec_encoder_transmit(fec_encoder* e, const uint8_t* data, int payload, int seq, uint8_t* cw_out,
                         int* cw_size) {
    if (!e || !cw_out || !cw_size || payload < 0 || (payload > 0 && !data) || seq < 0) return FEC_ERR_ARG;
    // The reference coder indexes its diagonals by seq % n and starts from an all-zero state, so
    // it accepts any first seq (Variable_Rate_FEC_Encoder creates encoders mid-stream,
    // Variable_Rate_FEC_Encoder.cpp:126/144/185); the first call fixes the origin, later calls
    // must be consecutive.
    if (e->origin < 0) {
        e->origin = seq;
        e->next = seq;
    }
    if (seq != e->next) return FEC_ERR_SEQUENCE;
    if (e->poisoned) return FEC_ERR_HIP;
    const Geometry& g = e->codec->g;
    if (payload > g.L) payload = g.L;
    fec::CodecView v;
    if (int st = fec::codec_view(e->codec.get(), &v)) return st;
    // from here on a failed HIP call leaves the window ring (device) and e->next (host) apart
    struct Poison {
        bool& p;
        bool ok = false;
        ~Poison() {
            if (!ok) p = true;
        }
    } poison{e->poisoned};
    if (e->sv.on) {
        // the resident server: the request, sealed with its ticket, into the mailbox; no launch
        // (fec_server.hip)
        const uint32_t ticket = ++e->ticket;
        {
            uint32_t w[fec::kEncReqFields + 375];
            const int64_t rel = seq - e->origin;
            w[0] = static_cast<uint32_t>(payload);
            w[1] = static_cast<uint32_t>(rel);
            w[2] = static_cast<uint32_t>(rel >> 32);
            const int nw = e->sv.nunits - fec::kEncReqFields;
            w[fec::kEncReqFields + nw - 1] = 0;
            if (payload > 0) std::memcpy(w + fec::kEncReqFields, data, payload);
            std::memset(reinterpret_cast<uint8_t*>(w + fec::kEncReqFields) + payload, 0, 4 * nw - payload);
            server_seal(e->sv, 0, w, e->sv.nunits, ticket);
        }
        const bool persistent = server_persistent(e->sv);
        auto launch = [&](uint32_t last, int64_t idle_ticks) -> hipError_t {
            fec::EncServerArgs a;
            a.box = e->sv.m_box;
            a.req = e->sv.m_req;
            a.nunits = e->sv.nunits;
            a.stage = e->m_stage;
            a.res = e->m_res;
            a.res_len_off = e->res_len_off;
            a.win_home = e->d_win;
            a.G = v.G;
            a.gf = v.gf;
            a.L = g.L;
            a.k = g.k;
            a.n = g.n;
            a.S = g.S;
            a.CW = g.CW;
            a.SK = g.S * g.k;
            a.W = std::max(1, g.n - 1);
            a.last = last;
            a.idle_ticks = idle_ticks;
            return fec::server_encode_launch(a, e->s) == FEC_OK ? hipSuccess : hipErrorLaunchFailure;
        };
        HIP_TRY(server_post(e->sv, ticket, e->s, persistent, launch));
        HIP_TRY(server_wait(e->sv, ticket, e->s, persistent, launch));
        std::memcpy(cw_out, e->h_res, g.CW);
        std::memcpy(cw_size, e->h_res + e->res_len_off, 4);
        ++e->next;
        poison.ok = true;
        return FEC_OK;
    }
    // one launch: the closed form over the device-resident window (fec_streams_encode_kernel reads
    // the payload from the mapped staging row, writes codeword and size into the mapped result row,
    // then the completion word)
    if (e->ticket) HIP_TRY(wait_done(e->h_done, e->ticket, e->s));  // h_stage is free again
    if (payload > 0) std::memcpy(e->h_stage, data, payload);
    const uint32_t ticket = ++e->ticket;
    if (int st = fec::stream_encode_one(v, e->d_win, e->m_stage, payload, seq - e->origin, e->m_res,
                                        reinterpret_cast<int32_t*>(e->m_res + e->res_len_off),
                                        reinterpret_cast<uint32_t*>(e->m_done), ticket, e->s))
        return st;
    HIP_TRY(wait_done(e->h_done, ticket, e->s));
    std::memcpy(cw_out, e->h_res, g.CW);
    std::memcpy(cw_size, e->h_res + e->res_len_off, 4);
    ++e->next;
    poison.ok = true;
    return FEC_OK;
}

// ---- streaming decoder --------------------------------------------------------------------
int fec_decoder_create(int max_payload, int T, int B, int N, fec_decoder** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<fec_decoder> d(new fec_decoder());
        fec_codec* c = nullptr;
        if (int st = fec_codec_create(max_payload, T, B, N, &c)) return st;
        d->codec.reset(c);
        const Geometry& g = c->g;
        if (g.T + g.k > fec_decoder::RR) return FEC_ERR_ARG;
        d->planner.reset(new fec::StreamPlanner(g, c->rules.get()));
        d->res_len_off = (g.L + 3) & ~3;
        HIP_TRY(coder_stream_create(&d->s));
        HIP_TRY(hipMalloc(&d->d_ring, static_cast<size_t>(fec_decoder::RR) * g.CW));
        HIP_TRY(hipMemset(d->d_ring, 0, static_cast<size_t>(fec_decoder::RR) * g.CW));
        HIP_TRY(hipMalloc(&d->d_coef, g.k * g.n));
        HIP_TRY(host_mapped(&d->h_cw, &d->m_cw, (g.CW + 3) & ~3));
        HIP_TRY(host_mapped(&d->h_coef, &d->m_coef, (g.k * g.n + 3) & ~3));
        HIP_TRY(host_mapped(&d->h_res, &d->m_res, d->res_len_off + 4));
        HIP_TRY(host_mapped(&d->h_done, &d->m_done, 4));
        const int Wn = g.k + g.n - 1;
        d->sv.on = server_enabled() && g.k * g.n <= 16 * 32 && static_cast<int64_t>(Wn) * g.CW <= 48 * 1024;
        if (d->sv.on) {
            HIP_TRY(host_mapped(reinterpret_cast<uint8_t**>(&d->sv.h_box), reinterpret_cast<uint8_t**>(&d->sv.m_box),
                                sizeof(fec::ServerBox)));
            d->win_units = (Wn * g.CW + 3) / 4;
            d->sv.nunits = fec::kDecReqFields + d->win_units + (g.k * g.n + 3) / 4;
            HIP_TRY(host_mapped(reinterpret_cast<uint8_t**>(&d->sv.h_req), reinterpret_cast<uint8_t**>(&d->sv.m_req),
                                sizeof(uint64_t) * d->sv.nunits));
            d->h_ring.assign(static_cast<size_t>(fec_decoder::RR) * g.CW, 0);
            d->req.assign(static_cast<size_t>(d->sv.nunits), 0);
        }
        HIP_TRY(hipDeviceSynchronize());  // the ring is zero before the first call's kernel
        *out = d.release();
        return FEC_OK;
    });
}

int fec_decoder_destroy(fec_decoder* d) {
    delete d;
    return FEC_OK;
}

namespace {
// Server mode, packet x received (fate kCopy): its systematic bytes from the decoder's own copy of
// its codeword -- the fast path's copy (Decoder.cpp:77-108) and the slow path's output for a
// received packet (its sub-streams' data symbols; the length clamped, Decoder.cpp:148-149).  No GF
// work: the same formula as the device copy kernels (fec_streams.hip stream_decode_one).
void host_copy_out(const Geometry& g, const uint8_t* cwx, bool clamp, uint8_t* payload_out, int* payload) {
    auto byte_at = [&](int h) -> uint8_t {
        const int s = h / g.k, i = h - s * g.k;
        return cwx[s * g.n + i];
    };
    const int hdr = byte_at(0) * 256 + byte_at(1);
    const int ln = clamp ? std::min(hdr, g.L) : hdr;
    const int cp = std::min(ln, g.L);
    // data byte h = symbol (h / k, h % k): runs of up to k contiguous bytes per sub-stream
    for (int b = 0, h = 2; b < cp;) {
        const int s = h / g.k, i = h - s * g.k;
        const int run = std::min(g.k - i, cp - b);
        std::memcpy(payload_out + b, cwx + s * g.n + i, run);
        b += run;
        h += run;
    }
    std::memset(payload_out + cp, 0, g.L - cp);
    *payload = ln;
}
}  // namespace

int fec_decoder_receive(fec_decoder* d, const uint8_t* cw, int cw_size, int seq, int erasure,
                        uint8_t* payload_out, int* payload) {
    if (!d || !payload_out || !payload || seq < 0) return FEC_ERR_ARG;
    // first call = origin (Variable_Rate_FEC_Decoder creates decoders mid-stream,
    // Variable_Rate_FEC_Decoder.cpp:2472/2559); the decoder state is a function of seq - origin
    // (all diagonal blocks start identical, so relabelling them by the origin is exact)
    if (d->origin < 0) {
        d->origin = seq;
        d->next = seq;
    }
    if (seq != d->next) return FEC_ERR_SEQUENCE;
    if (d->poisoned) return FEC_ERR_HIP;
    const int64_t rel = seq - d->origin;
    const Geometry& g = d->codec->g;
    const bool er = erasure != 0 || cw == nullptr;
    // the previous call's kernel has read h_cw / h_coef (its completion word is set); server-mode
    // calls are synchronous
    if (d->ticket && !d->sv.on) HIP_TRY(wait_done(d->h_done, d->ticket, d->s));
    if (d->sv.on) {  // FEC_Decoder.cpp:55-63: the decoder's zero-padded copy of the wire codeword
        uint8_t* row = d->h_ring.data() + (rel % fec_decoder::RR) * g.CW;
        const int sz = er ? 0 : std::max(0, std::min(cw_size, g.CW));
        if (sz) std::memcpy(row, cw, sz);
        std::memset(row + sz, 0, g.CW - sz);
    }
    fec::StepResult r;
    int st = guarded([&] {
        r = d->planner->step(rel, er);
        return FEC_OK;
    });
    if (st) return st;
    ++d->next;
    // from here on a failed HIP call leaves the planner (host) ahead of the device ring
    struct Poison {
        bool& p;
        bool ok = false;
        ~Poison() {
            if (!ok) p = true;
        }
    } poison{d->poisoned};
    const bool no_output = r.fate == fec::kNone || r.fate == fec::kLost;
    if (no_output) {
        std::memset(payload_out, 0, g.L);
        *payload = 0;
        if (er || d->sv.on) {  // nothing to keep on the device, nothing to compute
            poison.ok = true;
            return FEC_OK;
        }
    }
    if (d->sv.on) {
        const uint8_t* ring = d->h_ring.data();
        if (r.fate == fec::kCopy) {
            host_copy_out(g, ring + (r.x % fec_decoder::RR) * g.CW, r.slow, payload_out, payload);
            poison.ok = true;
            return FEC_OK;
        }
        // a recovered packet: the coefficients and the k+n-1 codewords they read (packets
        // x-k+1 .. x+n-1, zero rows before the origin or not yet received), sealed into the
        // mailbox of the resident server (fec_server.hip)
        fec::CodecView v;
        if (int e = fec::codec_view(d->codec.get(), &v)) return e;
        const uint32_t ticket = ++d->ticket;
        uint32_t* w = d->req.data();
        std::fill(w, w + fec::kDecReqFields, 0u);
        w[0] = static_cast<uint32_t>(r.fate);
        w[1] = r.slow ? 1u : 0u;
        uint8_t* wb = reinterpret_cast<uint8_t*>(w + fec::kDecReqFields);
        const int Wn = g.k + g.n - 1;
        for (int row = 0; row < Wn; ++row) {
            const int64_t sp = r.x - (g.k - 1) + row;
            uint8_t* dst = wb + static_cast<size_t>(row) * g.CW;
            if (sp < 0 || sp > rel) std::memset(dst, 0, g.CW);
            else std::memcpy(dst, ring + (sp % fec_decoder::RR) * g.CW, g.CW);
        }
        std::memset(wb + static_cast<size_t>(Wn) * g.CW, 0, 4 * d->win_units - static_cast<size_t>(Wn) * g.CW);
        uint8_t* cfb = reinterpret_cast<uint8_t*>(w + fec::kDecReqFields + d->win_units);
        const int ncf = (g.k * g.n + 3) / 4;
        std::memset(cfb, 0, 4 * ncf);
        std::memcpy(cfb, r.coef, g.k * g.n);
        server_seal(d->sv, 0, w, d->sv.nunits, ticket);
        const bool persistent = server_persistent(d->sv);
        auto launch = [&](uint32_t last, int64_t idle_ticks) -> hipError_t {
            fec::DecServerArgs a;
            a.box = d->sv.m_box;
            a.req = d->sv.m_req;
            a.nunits = d->sv.nunits;
            a.win_units = d->win_units;
            a.res = d->m_res;
            a.res_len_off = d->res_len_off;
            a.gf = v.gf;
            a.L = g.L;
            a.k = g.k;
            a.n = g.n;
            a.CW = g.CW;
            a.Wn = Wn;
            a.last = last;
            a.idle_ticks = idle_ticks;
            return fec::server_decode_launch(a, d->s) == FEC_OK ? hipSuccess : hipErrorLaunchFailure;
        };
        HIP_TRY(server_post(d->sv, ticket, d->s, persistent, launch));
        HIP_TRY(server_wait(d->sv, ticket, d->s, persistent, launch));
        std::memcpy(payload_out, d->h_res, g.L);
        std::memcpy(payload, d->h_res + d->res_len_off, 4);
        poison.ok = true;
        return FEC_OK;
    }
    if (!er) {  // FEC_Decoder.cpp:55-63: keep a zero-padded copy of the wire codeword
        const int sz = std::max(0, std::min(cw_size, g.CW));
        std::memset(d->h_cw, 0, (g.CW + 3) & ~3);
        if (sz) std::memcpy(d->h_cw, cw, sz);
    }
    const uint8_t* coef = nullptr;
    if (r.fate == fec::kRecovered) {
        std::memcpy(d->h_coef, r.coef, g.k * g.n);
        HIP_TRY(hipMemcpyAsync(d->d_coef, d->h_coef, g.k * g.n, hipMemcpyHostToDevice, d->s));
        coef = d->d_coef;
    }
    // one launch (fec_streams_decode_kernel): the codeword into the device ring, packet r.x into the
    // mapped result row, then the completion word
    fec::CodecView v;
    if (int e = fec::codec_view(d->codec.get(), &v)) return e;
    const uint32_t ticket = ++d->ticket;
    if (int e = fec::stream_decode_one(v, d->d_ring, er ? nullptr : d->m_cw, rel, er ? 1 : 0, r.fate, r.slow ? 1 : 0,
                                       r.x, coef, d->m_res, reinterpret_cast<int32_t*>(d->m_res + d->res_len_off),
                                       reinterpret_cast<uint32_t*>(d->m_done), ticket, d->s))
        return e;
    if (no_output) {  // the codeword is stored asynchronously; the next call waits for it
        poison.ok = true;
        return FEC_OK;
    }
    HIP_TRY(wait_done(d->h_done, ticket, d->s));
    std::memcpy(payload_out, d->h_res, g.L);
    std::memcpy(payload, d->h_res + d->res_len_off, 4);
    poison.ok = true;
    return FEC_OK;
}

int fec_plan_host(int max_payload, int T, int B, int N, const uint8_t* erasure, int64_t P,
                  uint8_t* fate) {
    if (!erasure || !fate || P < 0) return FEC_ERR_ARG;
    return guarded([&] {
        const Geometry g = Geometry::make(max_payload, T, B, N);
        if (g.B < g.N || g.n > fec::kMaxN - 1) return FEC_ERR_ARG;
        const auto rules = fec::shared_decode_rules(T, B, N);
        fec::StreamPlanner pl(g, rules.get());
        for (int64_t t = 0; t < P; ++t) {
            const fec::StepResult r = pl.step(t, erasure[t] != 0);
            if (r.x >= 0) fate[r.x] = static_cast<uint8_t>(r.fate);
        }
        return FEC_OK;
    });
}

}  // extern "C"

int fec::codec_view(const fec_codec* c, fec::CodecView* v) {
    if (!c || !v) return FEC_ERR_ARG;
    const Geometry& g = c->g;
    v->L = g.L;
    v->T = g.T;
    v->B = g.B;
    v->N = g.N;
    v->k = g.k;
    v->n = g.n;
    v->S = g.S;
    v->CW = g.CW;
    v->G = c->d_G;
    v->gf = c->d_gf;
    v->rules = c->d_rules;
    v->wbase_n = c->rules->w_base[g.n];
    v->ES = c->rules->entry_bytes;
    return FEC_OK;
}

extern "C" {

// ---- block mode (fec_block.hip) ------------------------------------------------------------
static int launch_block(fec_codec* c, bool decode, const uint8_t* d_in, const uint8_t* d_er, int64_t nblk,
                        uint8_t* d_out, uint8_t* d_er_out, void* stream) {
    if (!c || nblk < 0 || (nblk > 0 && (!d_in || !d_out || (decode && !d_er)))) return FEC_ERR_ARG;
    if (nblk == 0) return FEC_OK;
    const Geometry& g = c->g;
    if (decode && c->rules->lazy) return FEC_ERR_ARG;  // block decode reads the window-n rule table
    fec::BlockArgs a;
    a.in = d_in;
    a.er = d_er;
    a.out = d_out;
    a.er_out = d_er_out;
    a.nblk = nblk;
    a.k = g.k;
    a.n = g.n;
    a.G = c->d_G;
    a.gf = c->d_gf;
    a.rules = c->d_rules;
    a.wbase_n = c->rules->w_base[g.n];
    a.ES = c->rules->entry_bytes;
    const int64_t grid = std::min<int64_t>((nblk + 255) / 256, 4096);
    const size_t lds = decode ? 768 + 2 * 256 * g.n : 768 + 1024 + 256 * (g.k + g.n);
    if (decode)
        hipLaunchKernelGGL(fec::fec_block_decode_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), lds,
                           static_cast<hipStream_t>(stream), a);
    else
        hipLaunchKernelGGL(fec::fec_block_encode_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), lds,
                           static_cast<hipStream_t>(stream), a);
    HIP_TRY(hipGetLastError());
    return FEC_OK;
}

int fec_block_encode_batch(fec_codec* c, const uint8_t* d_data, int64_t nblk, uint8_t* d_codeword, void* stream) {
    return launch_block(c, false, d_data, nullptr, nblk, d_codeword, nullptr, stream);
}

int fec_block_decode_batch(fec_codec* c, const uint8_t* d_codeword, const uint8_t* d_erasure, int64_t nblk,
                           uint8_t* d_out, uint8_t* d_erasure_out, void* stream) {
    return launch_block(c, true, d_codeword, d_erasure, nblk, d_out, d_erasure_out, stream);
}

int fec_util_fill_payload(uint8_t* d_out, int64_t t0, int64_t count, int L, uint64_t seed,
                          void* stream) {
    if (!d_out || count < 0 || L <= 0) return FEC_ERR_ARG;
    if (count == 0) return FEC_OK;
    const int64_t blocks = std::min<int64_t>((count * L + 255) / 256, 8192);
    hipLaunchKernelGGL(fec::fec_fill_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_out, t0, count, L, seed);
    HIP_TRY(hipGetLastError());
    return FEC_OK;
}

}  // extern "C"
