// fec_relay_vr.hip -- the relay chain under variable rate, batched: RELAYING_TYPE 2 / 3 through
// a schedule of code switches (fec_amd.h, fec_relay_vr_*).
//
// What the reference does (Variable_Rate_FEC_Decoder.cpp:600-740 at the relay, :1423-1600 and
// :1772-1873 at the destination): at a switch to a new code (T, N) at seq s the relay and the
// destination each create a fresh Decoder_Symbol_Wise for it; for the T_TOT + 1 double-coded seqs
// s .. s + T_TOT the old object takes the old codeword and the new one the new codeword, the relay
// sends [BE16 size_cur][new code's part][old code's part], the destination's old object reports
// and the new one only decodes; at s + T_TOT + 1 both nodes copy the new object into the main one
// (copy_elements, Decoder_Symbol_Wise.cpp:88-117) and go on with it.
//
// So every code instance i -- a fresh object at its start seq a_i that runs through b_i = the end
// of the next switch's double coding -- is one fixed-rate relay chain over seqs [a_i, b_i] with its
// own source encoder (also fresh at a_i, Variable_Rate_FEC_Encoder.cpp:74-235).  The batch lays
// the instances of one code end to end in one stream of rows, each behind kGap rows of zero
// codewords on received flags: a window reaching in front of an instance then sees exactly what a
// fresh object holds (zero rows, received flags), so one fixed-rate batch per code (fec_swdf /
// fec_sdswdf, the state-dependent planners reset at each instance's first row) runs all its
// instances at once.  The gap rows' codewords and frames are zeroed between the stages; the relay
// frames and the destination's reported rows are then gathered back into seq order, with the
// double-coding layout.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "fec_amd.h"
#include "fec_status.h"

namespace fec {
int encode_batch_nolen(fec_codec* c, const uint8_t* d_payload, const int32_t* d_len, int64_t history, int64_t P,
                       uint8_t* d_cw, int32_t* d_cwlen_fallback, hipStream_t s);  // fec_codec.hip
namespace {

constexpr int kTT = 10;         // T_TOT (FEC_Macro.h)
constexpr int kGap = 3 * kTT + 3;  // zero rows in front of an instance (>= every window's reach)
constexpr int kMaxCodes = 16;
constexpr int kGatherLanes = 32;  // lanes per seq in the gather (64: 340 us, 32: 207 us, 16: 210 us; r06ze, r06zf)

struct RvTupleDev {             // one code's batch buffers, for the gather kernel
    const uint8_t* frames;      // rows of F bytes
    const uint8_t* out;         // rows of ostride bytes
    const uint8_t* flag;        // per row: the destination's loss flag (type 2; null for type 3)
    int F, part, hdr;           // frame row bytes, part bytes (from byte 2), of which header bytes (11 / 0)
    int ostride, outb;          // out row bytes, bytes reported
    const uint8_t* frames_end;  // one past the frames buffer (R rows of F bytes)
    const uint8_t* out_end;     // one past the out buffer (R rows of ostride bytes)
};
struct RvGatherArgs {
    RvTupleDev tup[kMaxCodes];
    const int32_t* map;         // [P][6]: new (code, row), old (code, row) or -1, reporting (code, row)
    int64_t P;
    uint8_t* frames;            // [P][fstride]
    int64_t fstride;
    int32_t* frame_len;
    uint8_t* out;               // [P][out_stride]
    int64_t out_stride;
    uint8_t* flag;              // [P]: the reporting object's flag (type 2), or null
};

// Bytes [0, n) of src to dst + doff (doff in 0..3, dst 4-byte aligned), a lane per destination
// dword, four dwords per lane per round with every load issued before the round's stores (a seq's
// copies are short: their load latency, not bandwidth, is the cost): two source dword loads (the
// source's own alignment) and v_alignbyte for an interior dword, byte loads at the run's two ends
// (the neighbouring bytes belong to other fields).
template <int NL>  // lanes per run
__device__ __forceinline__ void copy_run(uint8_t* dst, int doff, const uint8_t* src, int n, int lane) {
    const int nd = (doff + n + 3) >> 2;  // destination dwords touched
    const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
    for (int w0 = 0; w0 < nd; w0 += 4 * NL) {
        uint32_t v[4];
        bool whole[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int w = w0 + lane + NL * i;
            const int b0 = 4 * w - doff;  // source byte of the dword's first byte
            const uint32_t sh = static_cast<uint32_t>((sa + b0) & 3);
            // both aligned source dwords inside the run (no read past its last byte)
            whole[i] = w < nd && b0 >= 0 && b0 + 4 <= n && (sh == 0 || b0 - static_cast<int>(sh) + 8 <= n);
            v[i] = 0;
            if (whole[i]) {
                const uint32_t* p = reinterpret_cast<const uint32_t*>((sa + b0) & ~uintptr_t(3));
                const uint32_t lo = p[0], hi = sh ? p[1] : 0u;
                v[i] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int w = w0 + lane + NL * i;
            if (whole[i]) {
                *reinterpret_cast<uint32_t*>(dst + 4 * w) = v[i];
            } else if (w < nd) {
                const int b0 = 4 * w - doff;
                for (int x = 0; x < 4; ++x) {
                    const int bb = b0 + x;
                    if (bb >= 0 && bb < n) dst[4 * w + x] = src[bb];
                }
            }
        }
    }
}

// A frame without an old part is its code's frame row verbatim but for the BE16 size in front
// (Variable_Rate_FEC_Decoder.cpp:1502-1571): F bytes from any byte of the code's rows to a 16-byte
// aligned row, a lane per 16-byte chunk -- the two aligned source chunks that cover it, shifted --
// where copy_run takes two dword loads and a store per dword.  A lane whose second source chunk would
// pass the buffer's end reads bytes.  Bytes past F in the last chunk (the next row's) land in the
// destination row's padding, past frame_len.
__device__ __forceinline__ uint32_t keep_low(int c) { return c >= 4 ? 0xffffffffu : (1u << (8 * c)) - 1u; }

// The 16 bytes at s0 (any alignment): the two aligned chunks that cover them, shifted; bytes where
// the second chunk would pass src_end one by one.
__device__ __forceinline__ void load16_any(const uint8_t* s0, const uint8_t* src_end, uint32_t (&o)[4]) {
    const uintptr_t A = reinterpret_cast<uintptr_t>(s0) & ~uintptr_t(15);
    const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(s0) - A);
    if (reinterpret_cast<const uint8_t*>(A) + 32 <= src_end) {
        const uint4 lo = *reinterpret_cast<const uint4*>(A), hi = *reinterpret_cast<const uint4*>(A + 16);
        const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const int q = sh >> 2;
        const uint32_t r = static_cast<uint32_t>(sh & 3);
        uint32_t x[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) x[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = r ? __builtin_amdgcn_alignbyte(x[j + 1], x[j], r) : x[j];
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            o[j] = 0;
            for (int e = 0; e < 4; ++e)
                if (s0 + 4 * j + e < src_end) o[j] |= static_cast<uint32_t>(s0[4 * j + e]) << (8 * e);
        }
    }
}

template <int NL>
__device__ __forceinline__ void copy_row16(uint8_t* dst, const uint8_t* src, int n, const uint8_t* src_end,
                                           int size, int lane) {
    for (int c = lane; 16 * c < n; c += NL) {
        uint32_t o[4];
        load16_any(src + 16 * c, src_end, o);
        if (c == 0) o[0] = (o[0] & 0xffff0000u) | static_cast<uint32_t>(size / 256) | (static_cast<uint32_t>(size % 256) << 8);
        *reinterpret_cast<uint4*>(dst + 16 * c) = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// The reported row: bytes [0, n) of src, zero up to `stride` (a multiple of 4, dst 4-byte aligned),
// a lane per 16 bytes read as two aligned chunks, written as dwords.
template <int NL>
__device__ __forceinline__ void copy_out16(uint8_t* dst, const uint8_t* src, int n, int stride, const uint8_t* src_end,
                                           int lane) {
    for (int c = lane; 16 * c < stride; c += NL) {
        uint32_t o[4] = {0u, 0u, 0u, 0u};
        if (16 * c < n) load16_any(src + 16 * c, src_end, o);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int b = 16 * c + 4 * j;
            if (b >= stride) break;
            const uint32_t v = b + 4 <= n ? o[j] : (b >= n ? 0u : o[j] & keep_low(n - b));
            *reinterpret_cast<uint32_t*>(dst + b) = v;
        }
    }
}

// Half a wave (kGatherLanes) per seq: the frame [BE16 size of the new part's code bytes][new part][old part] and
// the reporting destination's row (its blocks*k bytes, zero after).  Frame rows and output rows are
// 4-byte aligned, the parts' sources at any byte; a frame without an old part (97 % of the seqs) is
// its code's row verbatim but for the size in front, copied 16 bytes a lane (copy_row16), the
// reported row likewise (copy_out16), and a double-coded frame a dword a lane (copy_run).  A frame
// of the fast codes is 27 - 54 such chunks and a reported row 21: a whole wave per seq left most of
// its lanes idle (207 vs 340 us per 360 000 seqs, profiles/r06/r06ze).  (Before: eight seqs per wave
// with their map entries loaded at once was slower, 489 vs 403 us; a wave per (seq, row) too, 518 vs
// 476 us, r06s; every load of a seq's three runs before their stores too, 620 vs 476 us, r06za.)
__global__ __launch_bounds__(256) void fec_relay_vr_gather_kernel(RvGatherArgs a) {
    __shared__ RvTupleDev stup[kMaxCodes];  // per-lane indices into the tuples: from LDS
    if (threadIdx.x < kMaxCodes) stup[threadIdx.x] = a.tup[threadIdx.x];
    __syncthreads();
    constexpr int NL = kGatherLanes, SPB = 256 / NL;  // lanes per seq, seqs per workgroup and pass
    const int lane = threadIdx.x & (NL - 1);
    const int64_t slot = static_cast<int64_t>(blockIdx.x) * SPB + threadIdx.x / NL;
    for (int64_t t = slot; t < a.P; t += static_cast<int64_t>(gridDim.x) * SPB) {
        const int32_t* m = a.map + 6 * t;
        const int m0 = m[0], m1 = m[1], m2 = m[2], m3 = m[3], m4 = m[4], m5 = m[5];
        const RvTupleDev& tn = stup[m0];
        uint8_t* fr = a.frames + t * a.fstride;
        const uint8_t* pn = tn.frames + static_cast<int64_t>(m1) * tn.F + 2;
        const int size_cur = tn.part - tn.hdr;  // the new code's codeword_r_d_size (:997-999, :1502-1571)
        int len = 2 + tn.part;
        if (m2 < 0) {  // no old part: the row as it is, its size in front
            copy_row16<NL>(fr, pn - 2, len, tn.frames_end, size_cur, lane);
        } else {
            if (lane == 0) {
                fr[0] = static_cast<uint8_t>(size_cur / 256);
                fr[1] = static_cast<uint8_t>(size_cur % 256);
            }
            copy_run<NL>(fr, 2, pn, tn.part, lane);
            const RvTupleDev& to = stup[m2];
            const uint8_t* po = to.frames + static_cast<int64_t>(m3) * to.F + 2;
            copy_run<NL>(fr + (len & ~3), len & 3, po, to.part, lane);
            len += to.part;
        }
        if (lane == 0) a.frame_len[t] = len;
        const RvTupleDev& tr = stup[m4];
        const uint8_t* src = tr.out + static_cast<int64_t>(m5) * tr.ostride;
        uint8_t* dst = a.out + t * a.out_stride;
        copy_out16<NL>(dst, src, tr.outb, static_cast<int>(a.out_stride), tr.out_end, lane);
        if (a.flag && lane == 0) a.flag[t] = tr.flag[m5];
    }
}

// Payload rows into an instance-ordered stream (src[r] < 0: a gap row, zero with length 0), and
// (er1 non-null) the rows' hop erasure flags from the seq-ordered patterns (gap rows received).
// A wave per 4 rows: with L a multiple of 4 and at most 512 bytes, every row's dwords are loaded
// before any is stored (the copy is latency-bound at one row per wave); bytes otherwise.
__global__ __launch_bounds__(256) void fec_relay_vr_payload_kernel(const uint8_t* payload, int L, const int64_t* src,
                                                                   int64_t R, uint8_t* dst, int32_t* len,
                                                                   const uint8_t* e1, const uint8_t* e2, uint8_t* er1,
                                                                   uint8_t* er2) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = static_cast<int64_t>(gridDim.x) * 4;
    for (int64_t r0 = (static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6)) * 4; r0 < R; r0 += nw * 4) {
        int64_t sv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) sv[i] = r0 + i < R ? src[r0 + i] : -2;
        if ((L & 3) == 0 && L <= 512) {
            uint32_t v[4][2];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int w = lane + 64 * j;
                    v[i][j] = (sv[i] >= 0 && w < L / 4) ? reinterpret_cast<const uint32_t*>(payload + sv[i] * L)[w] : 0u;
                }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int w = lane + 64 * j;
                    if (sv[i] > -2 && w < L / 4) reinterpret_cast<uint32_t*>(dst + (r0 + i) * L)[w] = v[i][j];
                }
        } else {
            for (int i = 0; i < 4; ++i) {
                if (sv[i] == -2) break;
                const int64_t r = r0 + i;
                for (int b = lane; b < L; b += 64) dst[r * L + b] = sv[i] < 0 ? 0 : payload[sv[i] * L + b];
            }
        }
        if (lane < 4 && sv[lane] > -2) {
            const int64_t r = r0 + lane, s = sv[lane];
            len[r] = s < 0 ? 0 : L;
            if (er1) {
                er1[r] = s < 0 ? 0 : (e1[s] ? 1 : 0);
                er2[r] = s < 0 ? 0 : (e2[s] ? 1 : 0);
            }
        }
    }
}

// Zero the gap rows of rows of W bytes: the kGap rows in front of instance b's first row
// starts[b] are one contiguous run of kGap * W bytes, a workgroup per instance, dword stores
// inside the run and byte stores at its two unaligned ends.  (A wave per row over all R rows,
// reading the row map to find the gap rows, took 20 - 38 us for the large codes.)
__global__ __launch_bounds__(256) void fec_relay_vr_zero_kernel(const int64_t* starts, int ninst, uint8_t* rows, int W) {
    if (static_cast<int>(blockIdx.x) >= ninst) return;
    const int64_t b0 = (starts[blockIdx.x] - kGap) * static_cast<int64_t>(W), b1 = b0 + static_cast<int64_t>(kGap) * W;
    const int64_t a0 = (b0 + 3) & ~int64_t(3), a1 = b1 & ~int64_t(3);
    const int tid = threadIdx.x;
    for (int64_t o = a0 + 4 * tid; o < a1; o += 4 * 256) *reinterpret_cast<uint32_t*>(rows + o) = 0u;
    if (tid < a0 - b0) rows[b0 + tid] = 0;
    if (tid < b1 - a1) rows[a1 + tid] = 0;
}

unsigned grid_rows(int64_t R) { return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((R + 3) / 4, 65536))); }

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t n) {
        if (n <= cap) return FEC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, std::max<size_t>(n, 16)) != hipSuccess) return FEC_ERR_NOMEM;
        cap = n;
        return FEC_OK;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct Code {
    int T = 0, N = 0, k = 0, n = 0, S = 0, CW = 0, rd = 0, part = 0, F = 0, ostride = 0, outb = 0;
    std::vector<int64_t> src;     // per row: source seq, or -1 (gap)
    std::vector<int64_t> starts;  // each instance's first row
    int64_t R = 0;
    fec_codec* codec = nullptr;
    fec_swdf* sw = nullptr;
    fec_sdswdf* sd = nullptr;
    DevBuf d_src, d_starts, d_pay, d_len, d_cw, d_cwlen, d_er1, d_er2, d_frames, d_out, d_flag, d_work;
    std::vector<uint8_t> h_er1, h_er2, h_flag;
    bool src_up = false;
    Code() = default;
    Code(const Code&) = delete;
    Code& operator=(const Code&) = delete;
    ~Code() {
        if (codec) fec_codec_destroy(codec);
        if (sw) fec_swdf_destroy(sw);
        if (sd) fec_sdswdf_destroy(sd);
    }
};

}  // namespace
}  // namespace fec

struct fec_relay_vr {
    static constexpr int kStreams = fec::kMaxCodes;  // type 3: a stream per code (its chains run side by side)
    static constexpr int kQueues = 4;                // type 2: the chains on this many streams
    int type = 2, L = 0;
    int64_t P = 0;
    hipStream_t st[kStreams] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kStreams] = {};
    ~fec_relay_vr() {
        for (int i = 0; i < kStreams; ++i) {
            if (st[i]) {
                (void)hipStreamSynchronize(st[i]);
                (void)hipStreamDestroy(st[i]);
            }
            if (ev_join[i]) (void)hipEventDestroy(ev_join[i]);
        }
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (h_pin) (void)hipHostFree(h_pin);
    }
    std::vector<std::unique_ptr<fec::Code>> codes;
    std::vector<int32_t> map;   // [P][6]
    int fstride = 0, ostride = 0;
    fec::DevBuf d_map, d_e1, d_e2, d_flag;  // the hop patterns (seq order) and, type 2, the flags out
    uint8_t* h_pin = nullptr;  // page-locked staging: e1, e2 up and the flags down (3 x P bytes)
    bool map_up = false;
};

extern "C" {

int fec_relay_vr_create(int type, int max_payload, const int32_t* sched, int nsw, int64_t P, fec_relay_vr** out) {
    if (!out) return FEC_ERR_ARG;
    *out = nullptr;
    if ((type != 2 && type != 3) || max_payload < 1 || max_payload > 65535 || !sched || nsw < 1 || P < 1 ||
        sched[0] != 0)
        return FEC_ERR_ARG;
    for (int i = 0; i < nsw; ++i) {
        const int s = sched[3 * i], T = sched[3 * i + 1], N = sched[3 * i + 2];
        if (T < 1 || T > fec::kTT || N < 0 || N > T || s < 0 || s >= P) return FEC_ERR_ARG;
        if (i > 0 && s < sched[3 * (i - 1)] + fec::kTT + 1) return FEC_ERR_ARG;  // one transition at a time
    }
    try {
        std::unique_ptr<fec_relay_vr> r(new fec_relay_vr());
        r->type = type;
        r->L = max_payload;
        r->P = P;
        std::map<int, int> code_of;  // T * 64 + N -> code index
        struct Inst {
            int64_t a, b, row0;
            int c;
        };
        std::vector<Inst> inst;
        for (int i = 0; i < nsw; ++i) {
            const int T = sched[3 * i + 1], N = sched[3 * i + 2];
            const int key = T * 64 + N;
            auto it = code_of.find(key);
            if (it == code_of.end()) {
                if (static_cast<int>(r->codes.size()) >= fec::kMaxCodes) return FEC_ERR_ARG;
                std::unique_ptr<fec::Code> c(new fec::Code());
                c->T = T;
                c->N = N;
                int st;
                if (type == 2) {
                    st = fec_swdf_create(max_payload, T, N, T, N, &c->sw);
                    int F = 0;
                    if (!st) st = fec_swdf_geometry(c->sw, &c->k, &c->n, nullptr, &c->S, &F, nullptr);
                    c->F = F;
                    c->part = F - 2;
                } else {
                    st = fec_sdswdf_create(max_payload, T, N, T, N, 0, &c->sd);
                    int F = 0;
                    if (!st) st = fec_sdswdf_geometry(c->sd, &c->k, &c->n, nullptr, &c->S, nullptr, &F, nullptr);
                    c->F = F;
                    c->part = F - 2;
                }
                if (st) return st;
                if ((st = fec_codec_create(max_payload, T, N, N, &c->codec))) return st;
                c->CW = c->S * c->n;
                c->ostride = c->S * c->k;
                c->outb = (max_payload / c->k + 1) * c->k;  // extract_data's blocks * k (:653-661)
                it = code_of.emplace(key, static_cast<int>(r->codes.size())).first;
                r->codes.push_back(std::move(c));
            }
            const int64_t a = sched[3 * i];
            const int64_t b = i + 1 < nsw ? std::min<int64_t>(sched[3 * (i + 1)] + fec::kTT, P - 1) : P - 1;
            inst.push_back({a, b, 0, it->second});
        }
        for (auto& in : inst) {  // rows: per code, its instances in seq order, each behind kGap zero rows
            fec::Code& c = *r->codes[static_cast<size_t>(in.c)];
            for (int g = 0; g < fec::kGap; ++g) c.src.push_back(-1);
            in.row0 = static_cast<int64_t>(c.src.size());
            c.starts.push_back(in.row0);
            for (int64_t t = in.a; t <= in.b; ++t) c.src.push_back(t);
        }
        int part_max = 0, ostride = max_payload + 32;
        for (auto& c : r->codes) {
            c->R = static_cast<int64_t>(c->src.size());
            part_max = std::max(part_max, c->part);
            ostride = std::max(ostride, c->outb);
        }
        r->fstride = (2 + 2 * part_max + 15) & ~15;
        r->ostride = (ostride + 3) & ~3;  // output rows 4-byte aligned (the gather's dword stores)
        // per seq: the newest instance, the old one during double coding, the reporting one
        r->map.assign(static_cast<size_t>(P) * 6, -1);
        for (size_t i = 0; i < inst.size(); ++i) {
            const Inst& in = inst[i];
            const bool has_next = i + 1 < inst.size();
            const int64_t next = has_next ? inst[i + 1].a : P;
            for (int64_t t = in.a; t <= in.b; ++t) {
                int32_t* m = &r->map[static_cast<size_t>(t) * 6];
                const int32_t row = static_cast<int32_t>(in.row0 + (t - in.a));
                const bool dc_new = i > 0 && t <= in.a + fec::kTT;  // the new object of a transition
                if (t < next) {  // newest instance at t
                    m[0] = in.c;
                    m[1] = row;
                } else {  // the old object of the next switch's double coding
                    m[2] = in.c;
                    m[3] = row;
                }
                // reporting: the old object during the next switch's transition, else this one unless
                // it is the new object of its own transition
                if (t >= next || !dc_new) {
                    m[4] = in.c;
                    m[5] = row;
                }
            }
        }
        *out = r.release();
        return FEC_OK;
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}

int fec_relay_vr_destroy(fec_relay_vr* r) {
    if (r) (void)hipDeviceSynchronize();
    delete r;
    return FEC_OK;
}

int fec_relay_vr_geometry(const fec_relay_vr* r, int* frame_stride, int* out_stride, int* codes) {
    if (!r) return FEC_ERR_ARG;
    if (frame_stride) *frame_stride = r->fstride;
    if (out_stride) *out_stride = r->ostride;
    if (codes) *codes = static_cast<int>(r->codes.size());
    return FEC_OK;
}

int fec_relay_vr_run(fec_relay_vr* r, const uint8_t* d_payload, const uint8_t* h_e1, const uint8_t* h_e2,
                     uint8_t* d_frames, int32_t* d_frame_len, uint8_t* d_out, uint8_t* h_flag, void* hip_stream) {
    if (!r || !d_payload || !h_e1 || !h_e2 || !d_frames || !d_frame_len || !d_out) return FEC_ERR_ARG;
    hipStream_t caller = static_cast<hipStream_t>(hip_stream);
    try {
        const int L = r->L;
        if (!r->ev_fork) {
            FEC_HIP(hipEventCreateWithFlags(&r->ev_fork, hipEventDisableTiming));
            for (int i = 0; i < fec_relay_vr::kStreams; ++i) {
                FEC_HIP(hipStreamCreateWithFlags(&r->st[i], hipStreamNonBlocking));
                FEC_HIP(hipEventCreateWithFlags(&r->ev_join[i], hipEventDisableTiming));
            }
        }
        if (r->type == 2) {  // the hop patterns, for the device-side row gathers (type 3's planners read them on the host)
            if (int st = r->d_e1.reserve(static_cast<size_t>(r->P))) return st;
            if (int st = r->d_e2.reserve(static_cast<size_t>(r->P))) return st;
            if (int st = r->d_flag.reserve(static_cast<size_t>(r->P))) return st;
            const size_t P = static_cast<size_t>(r->P);
            if (!r->h_pin) FEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&r->h_pin), 3 * P, hipHostMallocDefault));
            std::memcpy(r->h_pin, h_e1, P);  // (the previous run's copies are done: it ended synchronised)
            std::memcpy(r->h_pin + P, h_e2, P);
            FEC_HIP(hipMemcpyAsync(r->d_e1.p, r->h_pin, P, hipMemcpyHostToDevice, caller));
            FEC_HIP(hipMemcpyAsync(r->d_e2.p, r->h_pin + P, P, hipMemcpyHostToDevice, caller));
        }
        FEC_HIP(hipEventRecord(r->ev_fork, caller));
        // the streams this run uses: type 2's chains go to kQueues of them, type 3's codes one each (the
        // fork, the join and the drain touch only these: joining idle streams too cost the gather's
        // start ~60 us behind the last chain, profiles/r06/r06zd_*)
        const bool per_code = r->type == 3 || std::getenv("FEC_RELAY_VR_PER_CODE") != nullptr;  // (A/B for type 2)
        const int nst = std::min<int>(per_code ? fec_relay_vr::kStreams : fec_relay_vr::kQueues,
                                      static_cast<int>(r->codes.size()));
        // any return before the join below (an error) drains the side streams first: otherwise the
        // caller's stream is not ordered after their work and the next run could rewrite buffers
        // those kernels still read
        struct SideDrain {
            fec_relay_vr* r;
            int n;
            bool armed = true;
            ~SideDrain() {
                if (armed)
                    for (int i = 0; i < n; ++i) (void)hipStreamSynchronize(r->st[i]);
            }
        } drain{r, nst};
        for (int i = 0; i < nst; ++i)
            FEC_HIP(hipStreamWaitEvent(r->st[i], r->ev_fork, 0));
        // one code's chain on its own stream; type 3's host planners make its batches synchronous,
        // so its codes run on threads of their own (each code has its own planner objects)
        auto run_code = [&](size_t ci, hipStream_t s) -> int {
            fec::Code& c = *r->codes[ci];
            const int64_t R = c.R;
            if (r->type == 3) {  // the planners' erasure rows, on the host
                c.h_er1.resize(static_cast<size_t>(R));
                c.h_er2.resize(static_cast<size_t>(R));
                for (int64_t q = 0; q < R; ++q) {
                    const int64_t t = c.src[static_cast<size_t>(q)];
                    c.h_er1[static_cast<size_t>(q)] = t < 0 ? 0 : (h_e1[t] ? 1 : 0);
                    c.h_er2[static_cast<size_t>(q)] = t < 0 ? 0 : (h_e2[t] ? 1 : 0);
                }
            } else {
                if (int st = c.d_er1.reserve(static_cast<size_t>(R))) return st;
                if (int st = c.d_er2.reserve(static_cast<size_t>(R))) return st;
            }
            if (int st = c.d_src.reserve(static_cast<size_t>(R) * 8)) return st;
            if (int st = c.d_starts.reserve(c.starts.size() * 8)) return st;
            if (int st = c.d_pay.reserve(static_cast<size_t>(R) * L)) return st;
            if (int st = c.d_len.reserve(static_cast<size_t>(R) * 4)) return st;
            if (int st = c.d_cw.reserve(static_cast<size_t>(R) * c.CW)) return st;
            if (int st = c.d_cwlen.reserve(static_cast<size_t>(R) * 4)) return st;
            if (int st = c.d_frames.reserve(static_cast<size_t>(R) * c.F)) return st;
            if (int st = c.d_out.reserve(static_cast<size_t>(R) * c.ostride)) return st;
            if (!c.src_up) {  // the row map depends on the schedule alone: uploaded once
                FEC_HIP(hipMemcpyAsync(c.d_src.p, c.src.data(), static_cast<size_t>(R) * 8, hipMemcpyHostToDevice, s));
                FEC_HIP(hipMemcpyAsync(c.d_starts.p, c.starts.data(), c.starts.size() * 8, hipMemcpyHostToDevice, s));
                c.src_up = true;
            }
            const bool t2 = r->type == 2;
            hipLaunchKernelGGL(fec::fec_relay_vr_payload_kernel, dim3(fec::grid_rows((R + 3) / 4)), dim3(256), 0, s, d_payload, L,
                               c.d_src.as<const int64_t>(), R, c.d_pay.as<uint8_t>(), c.d_len.as<int32_t>(),
                               t2 ? r->d_e1.as<const uint8_t>() : nullptr, t2 ? r->d_e2.as<const uint8_t>() : nullptr,
                               t2 ? c.d_er1.as<uint8_t>() : nullptr, t2 ? c.d_er2.as<uint8_t>() : nullptr);
            FEC_HIP(hipGetLastError());
            // each instance a fresh source encoder: its rows behind kGap zero-length packets (>= n-1)
            // (without the trimmed wire sizes: nothing here reads them)
            if (int st = fec::encode_batch_nolen(c.codec, c.d_pay.as<uint8_t>(), c.d_len.as<int32_t>(), 0, R,
                                                 c.d_cw.as<uint8_t>(), c.d_cwlen.as<int32_t>(), s))
                return st;
            const int ninst = static_cast<int>(c.starts.size());
            const dim3 zgrid(static_cast<unsigned>(std::max(1, ninst)));
            hipLaunchKernelGGL(fec::fec_relay_vr_zero_kernel, zgrid, dim3(256), 0, s, c.d_starts.as<const int64_t>(), ninst,
                               c.d_cw.as<uint8_t>(), c.CW);
            FEC_HIP(hipGetLastError());
            if (r->type == 2) {
                if (int st = c.d_flag.reserve(static_cast<size_t>(R))) return st;
                const size_t wb = fec_swdf_workspace_bytes(c.sw, R);
                if (int st = c.d_work.reserve(wb)) return st;
                if (int st = fec_swdf_relay_batch(c.sw, c.d_cw.as<uint8_t>(), c.CW, c.d_er1.as<uint8_t>(), R,
                                                  c.d_frames.as<uint8_t>(), nullptr, c.d_work.p, wb, s))
                    return st;
                hipLaunchKernelGGL(fec::fec_relay_vr_zero_kernel, zgrid, dim3(256), 0, s, c.d_starts.as<const int64_t>(),
                                   ninst, c.d_frames.as<uint8_t>(), c.F);
                FEC_HIP(hipGetLastError());
                if (int st = fec_swdf_destination_batch(c.sw, c.d_frames.as<uint8_t>(), c.d_er2.as<uint8_t>(), R,
                                                        c.d_out.as<uint8_t>(), c.d_flag.as<uint8_t>(), s))
                    return st;
            } else {
                const int ns = static_cast<int>(c.starts.size());
                if (int st = fec_sdswdf_relay_batch_starts(c.sd, c.d_cw.as<uint8_t>(), c.CW, c.h_er1.data(), R,
                                                           c.starts.data(), ns, c.d_frames.as<uint8_t>(), s))
                    return st;
                hipLaunchKernelGGL(fec::fec_relay_vr_zero_kernel, zgrid, dim3(256), 0, s, c.d_starts.as<const int64_t>(),
                                   ninst, c.d_frames.as<uint8_t>(), c.F);
                FEC_HIP(hipGetLastError());
                c.h_flag.resize(static_cast<size_t>(R));
                if (int st = fec_sdswdf_destination_batch_starts(c.sd, c.d_frames.as<uint8_t>(), c.h_er2.data(), R,
                                                                 c.starts.data(), ns, c.d_out.as<uint8_t>(),
                                                                 c.h_flag.data(), s))
                    return st;
            }
            return static_cast<int>(FEC_OK);
        };
        if (r->type == 2) {
            // the codes' chains on kQueues streams (the device's hardware queues: more streams
            // share them, and a chain queued behind another on one waits for it), longest first,
            // each on the least loaded stream.  A chain's cost in microseconds (profiles/r06/r06q):
            // about 60 for its six launches plus 2 per 1000 rows with the specialised relay kernels;
            // about 250 whatever its rows without them (k < 4: the generic encoder and decoder, a
            // few hundred rows on bin/erasure.bin).
            std::vector<size_t> order(r->codes.size());
            for (size_t i = 0; i < order.size(); ++i) order[i] = i;
            auto cost = [&](size_t i) {
                const fec::Code& c = *r->codes[i];
                return c.k >= 4 ? 60 + c.R / 500 : 250 + c.R / 500;
            };
            std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return cost(x) > cost(y); });
            int64_t load[fec_relay_vr::kQueues] = {};
            for (size_t ci : order) {
                if (per_code) {
                    if (int st = run_code(ci, r->st[ci])) return st;
                    continue;
                }
                int q = 0;
                for (int j = 1; j < nst; ++j)
                    if (load[j] < load[q]) q = j;
                load[q] += cost(ci);
                if (int st = run_code(ci, r->st[q])) return st;
            }
        } else {
            std::vector<int> status(r->codes.size(), FEC_OK);
            std::vector<std::thread> th;
            for (size_t ci = 0; ci < r->codes.size(); ++ci)
                th.emplace_back([&, ci] {
                    try {
                        status[ci] = run_code(ci, r->st[ci]);
                    } catch (const std::bad_alloc&) {
                        status[ci] = FEC_ERR_NOMEM;
                    } catch (...) {
                        status[ci] = FEC_ERR_ARG;
                    }
                });
            for (auto& t : th) t.join();
            for (int st : status)
                if (st) return st;
        }
        hipStream_t s = caller;
        for (int i = 0; i < nst; ++i) {
            FEC_HIP(hipEventRecord(r->ev_join[i], r->st[i]));
            FEC_HIP(hipStreamWaitEvent(s, r->ev_join[i], 0));
        }
        drain.armed = false;  // the caller's stream now waits for every side stream
        if (!r->map_up) {
            if (int st = r->d_map.reserve(r->map.size() * 4)) return st;
            FEC_HIP(hipMemcpyAsync(r->d_map.p, r->map.data(), r->map.size() * 4, hipMemcpyHostToDevice, s));
            r->map_up = true;
        }
        fec::RvGatherArgs a{};
        for (size_t i = 0; i < r->codes.size(); ++i) {
            const fec::Code& c = *r->codes[i];
            a.tup[i] = {c.d_frames.as<const uint8_t>(), c.d_out.as<const uint8_t>(),
                        r->type == 2 ? c.d_flag.as<const uint8_t>() : nullptr, c.F, c.part, r->type == 3 ? 11 : 0,
                        c.ostride, c.outb, c.d_frames.as<const uint8_t>() + c.R * static_cast<int64_t>(c.F),
                        c.d_out.as<const uint8_t>() + c.R * static_cast<int64_t>(c.ostride)};
        }
        a.map = r->d_map.as<const int32_t>();
        a.P = r->P;
        a.frames = d_frames;
        a.fstride = r->fstride;
        a.frame_len = d_frame_len;
        a.out = d_out;
        a.out_stride = r->ostride;
        a.flag = r->type == 2 ? r->d_flag.as<uint8_t>() : nullptr;
        hipLaunchKernelGGL(fec::fec_relay_vr_gather_kernel, dim3(fec::grid_rows((r->P * fec::kGatherLanes + 63) / 64)), dim3(256), 0, s, a);
        FEC_HIP(hipGetLastError());
        if (r->type == 2 && h_flag)  // the reporting objects' flags, gathered by the kernel in seq order
            FEC_HIP(hipMemcpyAsync(r->h_pin + 2 * r->P, r->d_flag.p, static_cast<size_t>(r->P), hipMemcpyDeviceToHost, s));
        FEC_HIP(hipStreamSynchronize(s));
        if (r->type == 2 && h_flag) std::memcpy(h_flag, r->h_pin + 2 * r->P, static_cast<size_t>(r->P));
        if (r->type == 3 && h_flag)
            for (int64_t t = 0; t < r->P; ++t) {
                const int32_t* m = &r->map[static_cast<size_t>(t) * 6];
                h_flag[t] = r->codes[static_cast<size_t>(m[4])]->h_flag[static_cast<size_t>(m[5])];
            }
        return FEC_OK;
    } catch (const std::bad_alloc&) {
        return FEC_ERR_NOMEM;
    } catch (...) {
        return FEC_ERR_ARG;
    }
}

}  // extern "C"
