// fec_server.hip -- the per-packet coders' resident servers: one workgroup per FEC_Encoder /
// FEC_Decoder that stays on the GPU between calls and takes each call's packet from a host-visible
// mailbox, so that a call costs no kernel launch.
//
// The reference's contract is synchronous and per packet (FEC_Encoder::onTransmit,
// FEC_Encoder.cpp:42-68; FEC_Decoder::onReceive, FEC_Decoder.cpp:49-72): the codeword (payload)
// comes back from the call.  A launch per call costs more than the reference's whole CPU encode
// (DESIGN.md §4), so the coder keeps a server workgroup polling its mailbox instead:
//   host:   the request (fields and payload / codeword) -> the sealed request block, every 8-byte
//           unit stamped with the request's ticket (fec_kernels.h), then the request word;
//   server: one poll reads the block's head and sees the whole request in it (the fields and the
//           packet arrive with the ticket: no second round trip), does the packet's byte work (the
//           encoder against the n-1 windows it keeps in LDS for its whole life, Encoder.cpp:73-95;
//           the decoder's recovery against the window of codewords the request carries), writes the
//           result row, then the done ticket;
//   host:   polls the done ticket in its own (coherent) memory.
// Every poll also reads a stop word (set when the coder is destroyed), and a server that has seen
// no request for `idle_ticks` of the 100 MHz real-time counter writes its state back to HBM and
// exits; the next call launches a new one.  So every launch ends: on the stop word, on idle, or on
// the process's exit.  The exit handshake (alive = 0, then one more look at the request word, then
// exited = 1 if none) and the host's check of `alive` after posting are Dekker-ordered by
// sequentially consistent fences on both sides; a host that sees alive = 0 waits for alive = 1
// (revived for its request), its done ticket, or exited = 1 (then it waits for the launch to end and
// relaunches), so a request is never served twice and a revived server is never waited out.
// A server launched with idle_ticks = 0 serves the request already posted and exits (one-shot: the
// host's fallback when the process's persistent-server slots are taken, fec_codec.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fec_amd.h"
#include "fec_host.h"
#include "fec_kernels.h"

namespace fec {
namespace {

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t sys_load64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint8_t sgmul(const uint8_t* gexp, const uint8_t* glog, uint8_t a, uint8_t b) {
    return (a && b) ? gexp[glog[a] + glog[b]] : 0;
}

enum : uint32_t { kCmdIdle = 0, kCmdStop = 1, kCmdWork = 2 };

// Wave 0 waits for request last + 1: each poll reads the head of the sealed request block (lane l:
// units l, l + 64, l + 128) and the stop word in one round trip, and takes the request when every
// head unit carries the new ticket; the head's request dwords land in reqw (LDS).  On the stop word
// or the idle limit it ends the launch (exit handshake: announce, then one more look at the request
// word; a request posted meanwhile is served, its units complete since they were written first).
__device__ __forceinline__ uint32_t server_wait(ServerBox* box, const uint64_t* req, int nhead, uint32_t last,
                                                int64_t idle_ticks, uint32_t* reqw, uint32_t* cmd) {
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const uint32_t want = last + 1;
        uint32_t c = kCmdIdle;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            uint64_t u[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int i = lane + 64 * q;
                u[q] = i < nhead ? sys_load64(req + i) : static_cast<uint64_t>(want) << 32;
            }
            const uint32_t st = sys_load(&box->stop);
            bool ok = true;
#pragma unroll
            for (int q = 0; q < 3; ++q) ok = ok && static_cast<uint32_t>(u[q] >> 32) == want;
            if (st) {  // stopped (the coder's destruction, or another coder needs the queue)
                if (lane == 0) {
                    sys_store(&box->alive, 0u);
                    sys_store(&box->exited, 1u);
                }
                c = kCmdStop;
                break;
            }
            if (__all(ok)) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int i = lane + 64 * q;
                    if (i < nhead) reqw[i] = static_cast<uint32_t>(u[q]);
                }
                c = kCmdWork;
                break;
            }
            if (static_cast<int64_t>(__builtin_amdgcn_s_memrealtime() - t0) > idle_ticks) {
                if (lane == 0) sys_store(&box->alive, 0u);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                if (sys_load(&box->req) == want && !sys_load(&box->stop)) {
                    if (lane == 0) sys_store(&box->alive, 1u);
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        const int i = lane + 64 * q;
                        if (i < nhead) reqw[i] = static_cast<uint32_t>(sys_load64(req + i));
                    }
                    c = kCmdWork;
                } else if (lane == 0) {
                    sys_store(&box->exited, 1u);  // final: no request will be served by this launch
                }
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (c == kCmdWork) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the units past the head
        if (lane == 0) *cmd = c;
    }
    __syncthreads();
    return *cmd;
}

// After every thread's result stores: the done ticket, behind a system-scope release.
__device__ __forceinline__ void server_done(ServerBox* box, uint32_t ticket) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sys_store(&box->done, ticket);
    }
}

}  // namespace

// Encoder server.  Per request (seq relative to the coder's origin, payload size): the codeword
// of the closed form (Encoder.cpp:65-98 -> codingOperations.cpp:131-147) over the LDS windows, a
// thread per codeword byte; then the packet's own window row replaces row seq - W.
__global__ __launch_bounds__(256) void fec_encoder_server_kernel(EncServerArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t win[];  // W x SK window ring (slot seq % W)
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t Gs[16 * 32];
    __shared__ uint32_t reqw[kEncReqFields + 375];  // the request: fields, payload words (L <= 1500)
    __shared__ uint32_t cwl[512];   // codeword (CW <= 2048)
    __shared__ int ro[32];          // window offset of packet seq - d (-1: before the coder's origin)
    __shared__ int last_nz;
    __shared__ uint32_t cmd;
    const int tid = threadIdx.x;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW, SK = a.SK, W = a.W;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    for (int i = tid; i < k * n; i += 256) Gs[i] = a.G[i];
    for (int b = tid; b < W * SK; b += 256) win[b] = a.win_home[b];
    __syncthreads();
    uint32_t last = a.last;
    const int nhead = min(a.nunits, kServerHeadUnits);
    while (server_wait(a.box, a.req, nhead, last, a.idle_ticks, reqw, &cmd) == kCmdWork) {
        const uint32_t tk = last + 1;
        for (int i = nhead + tid; i < a.nunits; i += 256) reqw[i] = static_cast<uint32_t>(sys_load64(a.req + i));
        if (tid == 0) last_nz = -1;
        __syncthreads();
        const int ln = min(max(static_cast<int>(reqw[0]), 0), L);
        const int64_t seq = static_cast<int64_t>(reqw[1]) | (static_cast<int64_t>(reqw[2]) << 32);
        if (tid < 32) ro[tid] = (tid >= 1 && seq - tid >= 0) ? static_cast<int>((seq - tid) % W) * SK : -1;
        __syncthreads();
        const uint8_t* pay = reinterpret_cast<const uint8_t*>(reqw + kEncReqFields);
        auto xbyte = [&](int b) -> uint8_t {  // [len_hi, len_lo, payload, zero pad] (Encoder.cpp:75-83)
            return b == 0 ? static_cast<uint8_t>(ln >> 8)
                          : b == 1 ? static_cast<uint8_t>(ln & 0xff) : (b - 2 < ln ? pay[b - 2] : 0);
        };
        uint8_t* cwb = reinterpret_cast<uint8_t*>(cwl);
        int lastc = -1;
        for (int c = tid; c < CW; c += 256) {
            const int s = c / n, j = c - s * n;
            uint8_t v = 0;
            if (j < k) {
                v = xbyte(s * k + j);
            } else {  // parity: XOR_i G[i][j] * X_{t-(j-i)}[s][i], rows before the origin = 0
                for (int i = 0; i < k; ++i) {
                    const int r = ro[j - i];
                    if (r >= 0) v ^= sgmul(gexp, glog, Gs[i * n + j], win[r + s * k + i]);
                }
            }
            cwb[c] = v;
            if (v) lastc = c;
        }
        for (int c = CW + tid; c < ((CW + 3) & ~3); c += 256) cwb[c] = 0;  // the row's dword padding
        if (lastc >= 0) atomicMax(&last_nz, lastc);
        __syncthreads();  // codeword complete; window slot seq % W (row seq - W) has been read
        const int own = static_cast<int>(seq % W) * SK;
        for (int b = tid; b < SK; b += 256) win[own + b] = xbyte(b);
        for (int w = tid; 4 * w < CW; w += 256) reinterpret_cast<uint32_t*>(a.res)[w] = cwl[w];
        if (tid == 0) *reinterpret_cast<int32_t*>(a.res + a.res_len_off) = last_nz + 1;  // FEC_Encoder.cpp:55-60
        server_done(a.box, tk);
        last = tk;
        __syncthreads();  // the window row is in place before the next request's reads
    }
    // stop or idle: the windows go back to HBM for the next launch (kernel end makes them visible)
    for (int b = tid; b < W * SK; b += 256) a.win_home[b] = win[b];
}

// Decoder server.  Per request (a packet x the host planner recovers): the k+n-1 received
// codewords around x and the k x n coefficients arrive in the sealed request; the server applies
// the coefficients (the byte half of decodeBlock, codingOperations.cpp:149-232) and writes the
// payload of packet x into the result row.  It keeps no state: the systematic copies of the fast
// path (Decoder.cpp:77-108) are done by the host, which holds the received codewords anyway
// (FEC_Decoder.cpp:55-63).
__global__ __launch_bounds__(256) void fec_decoder_server_kernel(DecServerArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t win[];  // Wn x CW: packets x-k+1 .. x+n-1
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t coef[16 * 32];
    __shared__ uint32_t reqw[kServerHeadUnits];
    __shared__ uint32_t cmd;
    __shared__ int s_hdr;
    const int tid = threadIdx.x;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    __syncthreads();
    uint32_t last = a.last;
    const int nhead = min(a.nunits, kServerHeadUnits);
    while (server_wait(a.box, a.req, nhead, last, a.idle_ticks, reqw, &cmd) == kCmdWork) {
        const uint32_t tk = last + 1;
        auto unit = [&](int u) -> uint32_t { return u < nhead ? reqw[u] : static_cast<uint32_t>(sys_load64(a.req + u)); };
        for (int w = tid; w < a.win_units; w += 256) reinterpret_cast<uint32_t*>(win)[w] = unit(kDecReqFields + w);
        for (int w = tid; 4 * w < k * n; w += 256)
            reinterpret_cast<uint32_t*>(coef)[w] = unit(kDecReqFields + a.win_units + w);
        __syncthreads();
        const int clamp = static_cast<int>(reqw[1]);
        // data byte h of packet x: sum_q coef[i][q] * symbol (s, q) of packet x-i+q (window row k-1-i+q)
        auto byte_at = [&](int h) -> uint8_t {
            const int s = h / k, i = h - s * k;
            uint8_t acc = 0;
            for (int q = 0; q < n; ++q) {
                const uint8_t c = coef[i * n + q];
                if (c) acc ^= sgmul(gexp, glog, c, win[(k - 1 - i + q) * CW + s * n + q]);
            }
            return acc;
        };
        if (tid == 0) s_hdr = byte_at(0) * 256 + byte_at(1);
        __syncthreads();
        const int ln = clamp ? min(s_hdr, L) : s_hdr;
        const int cp = min(ln, L);
        uint8_t* orow = a.res;
        for (int w = tid; 4 * w < L; w += 256) {
            uint32_t v = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int b = 4 * w + e;
                if (b < cp) v |= static_cast<uint32_t>(byte_at(b + 2)) << (8 * e);
            }
            reinterpret_cast<uint32_t*>(orow)[w] = v;
        }
        if (tid == 0) *reinterpret_cast<int32_t*>(a.res + a.res_len_off) = ln;
        server_done(a.box, tk);
        last = tk;
        __syncthreads();
    }
}

int server_encode_launch(const EncServerArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(fec_encoder_server_kernel, dim3(1), dim3(256), static_cast<size_t>(a.W) * a.SK, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int server_decode_launch(const DecServerArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(fec_decoder_server_kernel, dim3(1), dim3(256), static_cast<size_t>(a.win_units) * 4, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // namespace fec
