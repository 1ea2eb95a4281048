// fec_kernels.hip -- see fec_kernels.h for the map from reference functions to kernels.
#include "fec_kernels.h"

namespace fec {

// ------------------------------------------------------------------------------------------
// GF(2^8) multiply of four packed bytes by one constant c, without tables in memory: c*x is
// linear over XOR, so c*x = c*(x & 0x07) ^ c*(x & 0x38) ^ c*(x & 0xC0).  Each term is an 8-, 8-
// and 4-entry table of c-multiples held in registers and indexed per byte by v_perm_b32
// (selector bytes 0-3 pick from the second operand, 4-7 from the first).
//   tab[0..1] = c*{0..7}, tab[2..3] = c*({0..7}<<3), tab[4] = c*({0..3}<<6).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t gf_mul4(const uint32_t* tab, uint32_t x) {
    const uint32_t g0 = x & 0x07070707u;
    const uint32_t g1 = (x >> 3) & 0x07070707u;
    const uint32_t g2 = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_perm(tab[1], tab[0], g0) ^ __builtin_amdgcn_perm(tab[3], tab[2], g1) ^
           __builtin_amdgcn_perm(tab[4], tab[4], g2);
}

__device__ __forceinline__ uint8_t gf_mul_lds(const uint8_t* gexp, const uint8_t* glog, uint8_t a,
                                              uint8_t b) {
    return (a && b) ? gexp[glog[a] + glog[b]] : 0;
}

// ------------------------------------------------------------------------------------------
// Encode.  Closed form of the reference's diagonal interleaving (verified bit-exact against the
// oracle): for packet t, sub-stream s, with X_t[s][i] = byte s*k+i of [len_hi, len_lo, payload,
// zero pad],
//     cw_t[s*n + j] = X_t[s][j]                                   j <  k
//     cw_t[s*n + j] = XOR_{i<k} G[i][j] * X_{t-(j-i)}[s][i]       j >= k
// One workgroup = TP packets.  LDS holds the tile's inputs plus an (n-1)-packet halo in a
// position-major layout xin[i][row][s] so that one dword = one position of four sub-streams:
// every parity term is then one conflict-free ds_read_b32 + one packed gf_mul4.  Outputs are
// assembled in LDS and leave in 16-byte coalesced stores.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fec_encode_kernel(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* xin = smem;
    uint8_t* xout = smem + a.xin_bytes;
    uint16_t* hmap = reinterpret_cast<uint16_t*>(xout + a.xout_bytes);
    const int Sk = a.S * a.k;
    int32_t* rowlen = reinterpret_cast<int32_t*>(hmap + ((Sk + 7) & ~7));

    const int tid = threadIdx.x;
    const int k = a.k, n = a.n, S = a.S, L = a.L, SP = a.SP, H = n - 1;
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * a.TP;
    const int ntile = static_cast<int>(min<int64_t>(a.TP, a.P - t0));
    const int rows = ntile + H;

    // Phase 0: zero the input planes, byte h -> (plane h%k, column h/k) map, row lengths.
    for (int o = tid * 16; o < a.xin_bytes; o += 256 * 16)
        *reinterpret_cast<uint4*>(xin + o) = make_uint4(0, 0, 0, 0);
    for (int h = tid; h < Sk; h += 256) hmap[h] = static_cast<uint16_t>((h % k) * a.plane + h / k);
    for (int r = tid; r < rows; r += 256) {
        const int64_t pk = t0 - H + r;
        int ln = -1;  // -1: packet before the encoder's first packet (all-zero row)
        if (pk >= -a.history) {
            ln = a.len ? a.len[pk] : L;
            ln = ln < 0 ? 0 : (ln > L ? L : ln);
        }
        rowlen[r] = ln;
    }
    __syncthreads();

    // Phase 1: scatter [len_hi, len_lo, payload] of every row into the planes.
    int rlo = 0;
    while (rlo < rows && rowlen[rlo] < 0) ++rlo;  // uniform: leading rows before the stream
    for (int r = rlo + tid; r < rows; r += 256) {
        const int ln = rowlen[r];
        xin[hmap[0] + r * SP] = static_cast<uint8_t>(ln >> 8);
        xin[hmap[1] + r * SP] = static_cast<uint8_t>(ln & 0xff);
    }
    const uint8_t* src = a.payload + (t0 - H + rlo) * L;
    const int nrows = rows - rlo;
    if ((L & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 3) == 0) {
        const int L4 = L >> 2;
        const int nd = nrows * L4;
        for (int f = tid; f < nd; f += 256) {
            const int rr = f / L4;
            const int b = (f - rr * L4) * 4;
            const int r = rlo + rr;
            const int ln = rowlen[r];
            if (b >= ln) continue;
            const uint32_t v = *reinterpret_cast<const uint32_t*>(src + static_cast<int64_t>(rr) * L + b);
            uint8_t* row = xin + r * SP;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (b + e < ln) row[hmap[b + e + 2]] = static_cast<uint8_t>(v >> (8 * e));
        }
    } else {
        const int nb = nrows * L;
        for (int f = tid; f < nb; f += 256) {
            const int rr = f / L;
            const int b = f - rr * L;
            const int r = rlo + rr;
            if (b < rowlen[r]) xin[r * SP + hmap[b + 2]] = src[static_cast<int64_t>(rr) * L + b];
        }
    }
    __syncthreads();

    // Phase 2: one task = (packet, group of 4 sub-streams).
    const int NS4 = SP >> 2;
    const uint32_t* x32 = reinterpret_cast<const uint32_t*>(xin);
    const int plane4 = a.plane >> 2, SP4 = SP >> 2;
    for (int task = tid; task < ntile * NS4; task += 256) {
        const int tl = task / NS4;
        const int s4 = task - tl * NS4;
        const int r0 = tl + H;
        uint8_t* orow = xout + tl * a.CW;
        const int sb = s4 * 4;
        const int ns = min(4, S - sb);
        for (int i = 0; i < k; ++i) {
            const uint32_t v = x32[i * plane4 + r0 * SP4 + s4];
            for (int e = 0; e < ns; ++e) orow[(sb + e) * n + i] = static_cast<uint8_t>(v >> (8 * e));
        }
        for (int j = k; j < n; ++j) {
            uint32_t acc = 0;
            for (int i = 0; i < k; ++i) {
                const uint32_t* tab = a.ptab + (i * (n - k) + (j - k)) * 8;
                if (!tab[5]) continue;  // zero coefficient (burst structure of G)
                acc ^= gf_mul4(tab, x32[i * plane4 + (r0 - (j - i)) * SP4 + s4]);
            }
            for (int e = 0; e < ns; ++e) orow[(sb + e) * n + j] = static_cast<uint8_t>(acc >> (8 * e));
        }
    }
    __syncthreads();

    // Phase 3: coalesced store of the tile + trimmed wire sizes (FEC_Encoder.cpp:55-60).
    const int bytes = ntile * a.CW;
    uint8_t* dst = a.cw + t0 * a.CW;
    if ((bytes & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (int o = tid * 16; o < bytes; o += 256 * 16)
            *reinterpret_cast<uint4*>(dst + o) = *reinterpret_cast<const uint4*>(xout + o);
    } else {
        for (int o = tid; o < bytes; o += 256) dst[o] = xout[o];
    }
    for (int tl = tid; tl < ntile; tl += 256) {
        const uint8_t* row = xout + tl * a.CW;
        int z = a.CW - 1;
        while (z >= 0 && row[z] == 0) --z;
        a.cw_len[t0 + tl] = z + 1;
    }
}

// ------------------------------------------------------------------------------------------
// Decode, step 1: resynchronisation points.  The reference decoder is in its fast path at a
// received packet t iff no packet of [t-T, t-1] was erased; at an erased packet it resyncs iff it
// was in the fast path just before, i.e. no erasure in [t-T-1, t-1] (Decoder.cpp:80-83, 109-133).
// Every resync starts an independent episode.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fec_scan_kernel(const uint8_t* er, int64_t P, int T,
                                                       int32_t* counters, int32_t* episodes) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < P; t += stride) {
        if (!er[t]) continue;
        bool resync = true;
        for (int d = 1; d <= T + 1 && t - d >= 0; ++d)
            if (er[t - d]) {
                resync = false;
                break;
            }
        if (resync) episodes[atomicAdd(&counters[0], 1)] = static_cast<int32_t>(t);
    }
}

// ------------------------------------------------------------------------------------------
// Decode, step 2: one wavefront replays one episode of the reference's block decoders
// symbolically.  State per diagonal block b (n of them): erased-position mask er[b], and for
// every stored codeword symbol p / data symbol i its GF coefficient vector over the symbols q of
// the block's current round (lane q holds coefficient q).  Each episode starts from the decoders'
// initial state: the resync overwrites every position that an output of the episode can reach
// ("episode independence").
// ------------------------------------------------------------------------------------------
namespace {
struct PlanState {
    const PlanArgs* a;
    uint8_t* gexp;
    uint8_t* glog;
    uint32_t* er;
    uint8_t* cwc;    // [b][p][q]
    uint8_t* datc;   // [b][i][q]
    uint8_t* fresh;  // [i][q]
    int lane, k, n, T;

    __device__ uint8_t* cw(int b, int p) { return cwc + (b * n + p) * n; }
    __device__ uint8_t* dat(int b, int i) { return datc + (b * k + i) * n; }

    // decodeBlock (codingOperations.cpp:149-232) on coefficient vectors.
    __device__ void decode_block(int b, int t) {
        const uint32_t mall = er[b];
        if (t < k && !((mall >> t) & 1u) && lane < n) dat(b, t)[lane] = cw(b, t)[lane];
        const int w = min(t + T + 1, n);
        const uint32_t full = (1u << w) - 1u;
        const uint32_t m = mall & full;
        if (m == full) return;
        if (!(m & ((1u << k) - 1u))) return;
        const uint8_t* ent = a->rules + a->wbase[w] + static_cast<int64_t>(m) * a->ES;
        const int selv = lane < k ? ent[lane] : 0xFF;
        uint32_t got = 0;
        for (int i = 0; i < k; ++i) {
            if (!((m >> i) & 1u)) continue;
            const int s = __shfl(selv, i);
            if (s == 0xFF) continue;
            const int colv = lane < w ? ent[k + i * n + lane] : 0;
            uint8_t acc = 0;
            for (int c = 0; c < w; ++c) {
                const int f = __shfl(colv, c);
                if (!f || ((m >> c) & 1u)) continue;
                if (lane < n) acc ^= gf_mul_lds(gexp, glog, static_cast<uint8_t>(f), cw(b, c)[lane]);
            }
            if (lane < n) fresh[i * n + lane] = acc;
            got |= 1u << i;
        }
        if (!got) return;
        for (int i = 0; i < k; ++i) {
            if (!((got >> i) & 1u)) continue;
            if (lane < n) {
                const uint8_t v = fresh[i * n + lane];
                dat(b, i)[lane] = v;
                cw(b, i)[lane] = v;
            }
        }
        er[b] = mall & ~got;  // every lane stores the same value
    }

    // Decoder_Block_Code::decodeSymbol (Decoder_Block_Code.cpp:61-78).
    __device__ void decode_symbol(int b, int p, bool erased) {
        if (erased) {
            er[b] = er[b] | (1u << p);
        } else {
            er[b] = er[b] & ~(1u << p);
            if (lane < n) cw(b, p)[lane] = (lane == p) ? 1 : 0;
        }
        if (p < T) return;
        decode_block(b, p - T);
        if (p == n - 1)
            for (int j = p - T + 1; j < k; ++j) decode_block(b, j);
    }

    // Decoder_Basic::decodeStream, input half: symbol p of the packet fed at `time` goes to
    // block (time - p) mod n.
    __device__ void feed(int64_t time, bool erased) {
        const int r = static_cast<int>(time % n);
        for (int p = 0; p < n; ++p) {
            int b = r - p;
            if (b < 0) b += n;
            decode_symbol(b, p, erased);
        }
    }
};
}  // namespace

__global__ __launch_bounds__(64) void fec_plan_kernel(PlanArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    PlanState st;
    st.a = &a;
    st.gexp = smem;
    st.glog = smem + 512;
    st.er = reinterpret_cast<uint32_t*>(smem + 768);
    st.cwc = smem + 768 + 128;
    st.datc = st.cwc + a.n * a.n * a.n;
    st.fresh = st.datc + a.n * a.k * a.n;
    st.lane = threadIdx.x;
    st.k = a.k;
    st.n = a.n;
    st.T = a.T;
    const int lane = threadIdx.x, k = a.k, n = a.n, T = a.T;
    for (int i = lane; i < 768; i += 64) smem[i] = a.gf[i];
    __syncthreads();
    const int nep = a.counters[0];
    const int state_bytes = n * n * n + n * k * n;
    for (int ep = blockIdx.x; ep < nep; ep += gridDim.x) {
        const int64_t tr = a.episodes[ep];
        for (int i = lane; i < 32; i += 64) st.er[i] = 0;
        for (int i = lane; i < state_bytes; i += 64) st.cwc[i] = 0;
        __syncthreads();
        int64_t latest = -1;
        for (int64_t t = tr; t < a.P; ++t) {
            const bool e = a.er[t] != 0;
            if (!e) {
                if (t - latest > T) break;  // Decoder.cpp:80-83: back to the fast path
            } else {
                if (latest == -1) {  // resync, Decoder.cpp:111-133
                    for (int i = 0; i < n - T; ++i) st.feed(t + i, true);
                    for (int i = 0; i < T; ++i)
                        if (t - T + i >= 0) st.feed(t - T + i, false);
                }
                latest = t;
            }
            st.feed(t, e);
            const int64_t x = t - T;
            if (x < 0 || x >= a.Pout || !a.er[x]) continue;
            // Decoder_Basic::decodeStream output half (Decoder_Basic.cpp:68-86).
            bool lost = false;
            for (int i = 0; i < k; ++i) {
                const int b = static_cast<int>(((x - i) % n + n) % n);
                if ((st.er[b] >> i) & 1u) lost = true;
            }
            if (lost) {
                if (lane == 0) atomicAdd(&a.counters[2], 1);
                continue;
            }
            int r = 0;
            if (lane == 0) r = atomicAdd(&a.counters[1], 1);
            r = __shfl(r, 0);
            if (lane == 0) a.rec_list[r] = static_cast<int32_t>(x);
            if (lane < n) {
                for (int i = 0; i < k; ++i) {
                    const int b = static_cast<int>(((x - i) % n + n) % n);
                    a.coef[(static_cast<int64_t>(r) * k + i) * n + lane] = st.dat(b, i)[lane];
                }
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Decode, step 3: every received packet's systematic bytes (fast path Decoder.cpp:77-108; the
// slow path outputs received packets unchanged too).  Tile of TP packets: codewords in via
// 16-byte loads, payload out via 16-byte stores, the (n-k)-byte gaps squeezed out through LDS.
// Erased packets get length 0 / zero bytes here and are overwritten by fec_recover_kernel.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fec_copy_kernel(CopyArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* cwt = smem;
    uint16_t* omap = reinterpret_cast<uint16_t*>(smem + a.cwt_bytes);
    int32_t* clen = reinterpret_cast<int32_t*>(omap + ((a.L + 2 + 7) & ~7));
    const int tid = threadIdx.x;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW;
    const int64_t x0 = static_cast<int64_t>(blockIdx.x) * a.TP;
    const int ntile = static_cast<int>(min<int64_t>(a.TP, a.Pout - x0));

    for (int h = tid; h < L + 2; h += 256) omap[h] = static_cast<uint16_t>((h / k) * n + h % k);
    const int bytes = ntile * CW;
    const uint8_t* src = a.cw + x0 * CW;
    if ((bytes & 15) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        for (int o = tid * 16; o < bytes; o += 256 * 16)
            *reinterpret_cast<uint4*>(cwt + o) = *reinterpret_cast<const uint4*>(src + o);
    } else {
        for (int o = tid; o < bytes; o += 256) cwt[o] = src[o];
    }
    __syncthreads();
    for (int tl = tid; tl < ntile; tl += 256) {
        const int64_t x = x0 + tl;
        int ln = 0, copy = 0;
        if (!a.er[x]) {
            const uint8_t* row = cwt + tl * CW;
            const int hdr = row[omap[0]] * 256 + row[omap[1]];
            bool slow = false;
            for (int d = 0; d <= a.T; ++d) slow = slow || a.er[x + d];
            ln = slow ? min(hdr, L) : hdr;  // Decoder.cpp:148-149 clamps in the slow path only
            copy = min(ln, L);
        }
        clen[tl] = copy;
        a.out_len[x] = ln;
    }
    __syncthreads();
    const int obytes = ntile * L;
    uint8_t* dst = a.out + x0 * L;
    const bool vec = (obytes & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
    if (vec) {
        for (int o = tid * 16; o < obytes; o += 256 * 16) {
            int tl = o / L;
            int b = o - tl * L;
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t acc = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t v = (b < clen[tl]) ? cwt[tl * CW + omap[b + 2]] : 0u;
                    acc |= v << (8 * e);
                    if (++b == L) {
                        b = 0;
                        ++tl;
                    }
                }
                w[q] = acc;
            }
            *reinterpret_cast<uint4*>(dst + o) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    } else {
        for (int o = tid; o < obytes; o += 256) {
            const int tl = o / L;
            const int b = o - tl * L;
            dst[o] = (b < clen[tl]) ? cwt[tl * CW + omap[b + 2]] : 0;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Decode, step 4: recovered packets.  Byte h of packet x (sub-stream s = h/k, position i = h%k)
// = XOR_q coef[i][q] * cw[x-i+q][s*n+q]  over the received symbols q of its diagonal.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fec_recover_kernel(RecArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t cf[16 * 32];
    __shared__ uint8_t ob[4096];
    const int tid = threadIdx.x;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    const int nrec = a.counters[1];
    for (int r = blockIdx.x; r < nrec; r += gridDim.x) {
        const int64_t x = a.rec_list[r];
        for (int i = tid; i < k * n; i += 256) cf[i] = a.coef[static_cast<int64_t>(r) * k * n + i];
        __syncthreads();
        for (int h = tid; h < L + 2; h += 256) {
            const int s = h / k, i = h - (h / k) * k;
            uint8_t acc = 0;
            for (int q = 0; q < n; ++q) {
                const uint8_t c = cf[i * n + q];
                if (!c) continue;
                const int64_t sp = x - i + q;
                if (sp < 0 || sp >= a.P) continue;
                acc ^= gf_mul_lds(gexp, glog, c, a.cw[sp * CW + s * n + q]);
            }
            ob[h] = acc;
        }
        __syncthreads();
        const int ln = min(ob[0] * 256 + ob[1], L);
        for (int b = tid; b < L; b += 256) a.out[x * L + b] = (b < ln) ? ob[b + 2] : 0;
        if (tid == 0) a.out_len[x] = ln;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Streaming decoder output of one packet: same formula with an identity matrix for a copy.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fec_stream_out_kernel(StreamOutArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t ob[4096];
    const int tid = threadIdx.x;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    __syncthreads();
    for (int h = tid; h < L + 2; h += 256) {
        const int s = h / k, i = h - (h / k) * k;
        uint8_t acc = 0;
        for (int q = 0; q < n; ++q) {
            const uint8_t c = a.coef[i * n + q];
            if (!c) continue;
            const int64_t sp = a.x - i + q;
            const int64_t row = ((sp % a.RR) + a.RR) % a.RR;
            acc ^= gf_mul_lds(gexp, glog, c, a.ring[row * CW + s * n + q]);
        }
        ob[h] = acc;
    }
    __syncthreads();
    const int hdr = ob[0] * 256 + ob[1];
    const int ln = a.clamp ? min(hdr, L) : hdr;
    const int cp = min(ln, L);
    for (int b = tid; b < L; b += 256) a.out[b] = (b < cp) ? ob[b + 2] : 0;
    if (tid == 0) *a.out_len = ln;
}

}  // namespace fec

namespace fec {
// Synthetic payloads for tests and bench.py (not part of the coding path): byte b of packet t =
// splitmix64(seed ^ (t*L + b)) & 0xff -- the same generator as oracle/fec_oracle.c.
__global__ __launch_bounds__(256) void fec_fill_kernel(uint8_t* out, int64_t t0, int64_t count, int L,
                                                       uint64_t seed) {
    const int64_t total = count * L;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t o = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; o < total; o += stride) {
        uint64_t z = (seed ^ static_cast<uint64_t>(t0 * L + o)) + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        out[o] = static_cast<uint8_t>((z ^ (z >> 31)) & 0xff);
    }
}
}  // namespace fec
