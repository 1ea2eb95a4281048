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
// Decode, step 1: resynchronisation points and the list of erased packets.  The reference
// decoder is in its fast path at a received packet t iff no packet of [t-T, t-1] was erased; at an
// erased packet it resyncs iff it was in the fast path just before, i.e. no erasure in
// [t-T-1, t-1] (Decoder.cpp:80-83, 109-133).  Every resync starts an independent episode.
// ------------------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ uint32_t nz_bytes_mask(uint32_t w) {  // bit e: byte e of w non-zero
    return (((w & 0xffu) != 0) ? 1u : 0u) | (((w & 0xff00u) != 0) ? 2u : 0u) |
           (((w & 0xff0000u) != 0) ? 4u : 0u) | (((w & 0xff000000u) != 0) ? 8u : 0u);
}
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o);
        if (lane >= o) v += y;
    }
    return v;
}
}  // namespace

// 16 packets per lane (one 16-byte load), 4096 per workgroup; both lists (erased outputs,
// episode starts) get one atomic per workgroup.
__global__ __launch_bounds__(256) void fec_scan_kernel(const uint8_t* er, int64_t P, int64_t Pout,
                                                       int T, int32_t* counters, int32_t* episodes,
                                                       int32_t* erased) {
    __shared__ int wtot[2][4];
    __shared__ int bbase[2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int64_t kPerBlock = 256 * 16;
    for (int64_t blk0 = static_cast<int64_t>(blockIdx.x) * kPerBlock; blk0 < P;
         blk0 += static_cast<int64_t>(gridDim.x) * kPerBlock) {
        const int64_t t0 = blk0 + tid * 16;
        uint32_t m = 0;  // bit e: packet t0+e erased
        if (t0 + 15 < P && (reinterpret_cast<uintptr_t>(er + t0) & 15) == 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(er + t0);
            m = nz_bytes_mask(v.x) | (nz_bytes_mask(v.y) << 4) | (nz_bytes_mask(v.z) << 8) |
                (nz_bytes_mask(v.w) << 12);
        } else {
            for (int e = 0; e < 16; ++e)
                if (t0 + e < P && er[t0 + e]) m |= 1u << e;
        }
        uint32_t resm = 0;
        for (uint32_t rest = m; rest; rest &= rest - 1) {
            const int e = __builtin_ctz(rest);
            const int64_t t = t0 + e;
            // resync iff no erasure in [t-T-1, t-1] (Decoder.cpp:80-83, 109-133)
            const int lo = e - T - 1;
            uint32_t inside = m & ((1u << e) - 1u);
            if (lo > 0) inside &= ~((1u << lo) - 1u);
            bool rs = inside == 0;
            if (rs && lo < 0)
                for (int64_t u = t0 - 1; u >= 0 && u >= t - T - 1; --u)
                    if (er[u]) {
                        rs = false;
                        break;
                    }
            if (rs) resm |= 1u << e;
        }
        uint32_t outm = m;
        if (t0 + 16 > Pout) outm &= (t0 >= Pout) ? 0u : ((1u << (Pout - t0)) - 1u);
        const int nout = __builtin_popcount(outm), nres = __builtin_popcount(resm);
        const int io = wave_incl_scan(nout, lane), ir = wave_incl_scan(nres, lane);
        if (lane == 63) {
            wtot[0][wave] = io;
            wtot[1][wave] = ir;
        }
        __syncthreads();
        if (tid == 0) {
            const int to = wtot[0][0] + wtot[0][1] + wtot[0][2] + wtot[0][3];
            const int tr = wtot[1][0] + wtot[1][1] + wtot[1][2] + wtot[1][3];
            bbase[0] = to ? atomicAdd(&counters[1], to) : 0;
            bbase[1] = tr ? atomicAdd(&counters[0], tr) : 0;
        }
        __syncthreads();
        int so = bbase[0] + io - nout, sr = bbase[1] + ir - nres;
        for (int w = 0; w < wave; ++w) {
            so += wtot[0][w];
            sr += wtot[1][w];
        }
        for (uint32_t rest = outm; rest; rest &= rest - 1)
            erased[so++] = static_cast<int32_t>(t0 + __builtin_ctz(rest));
        for (uint32_t rest = resm; rest; rest &= rest - 1)
            episodes[sr++] = static_cast<int32_t>(t0 + __builtin_ctz(rest));
        __syncthreads();
    }
}

// Packets whose k symbols were all recovered -> rec_list (one atomic per wave).
__global__ __launch_bounds__(256) void fec_compact_kernel(int32_t* counters, const int32_t* erased,
                                                          const uint8_t* sym_ok, int k,
                                                          int32_t* rec_list) {
    const int ner = counters[1];
    const int lane = threadIdx.x & 63;
    const int stride = gridDim.x * blockDim.x;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx - lane < ner; idx += stride) {
        bool ok = false;
        int64_t x = 0;
        if (idx < ner) {
            x = erased[idx];
            ok = true;
            for (int i = 0; i < k; ++i) ok = ok && sym_ok[x * k + i];
        }
        const unsigned long long bal = __ballot(ok);
        if (!bal) continue;
        int base = 0;
        if (lane == 0) base = atomicAdd(&counters[2], __popcll(bal));
        base = __shfl(base, 0);
        if (ok) rec_list[base + __popcll(bal & ((1ull << lane) - 1ull))] = static_cast<int32_t>(x);
    }
}

// ------------------------------------------------------------------------------------------
// Decode, step 2: symbolic replay.  The reference's decoder is S x n independent diagonal block
// decoders (Decoder_Basic / Decoder_Block_Code); all S sub-streams see the same erasure flags, and
// the n diagonals never interact.  One wavefront replays ONE diagonal b through ONE episode
// (resync .. return to the fast path), tracking the erased-position mask (wave-uniform) and, for
// every stored symbol, its GF coefficient vector over the n symbols of the block's current round
// (lane q holds coefficient q; LDS columns are lane-private).  Each episode starts from the
// decoders' initial state: the resync overwrites every position an output of the episode can
// reach ("episode independence").  For each erased packet x output in the episode the
// diagonal holding its symbol i = (x-b) mod n < k writes sym_ok[x][i] and coef[x][i][:].
// ------------------------------------------------------------------------------------------
namespace {
struct BlockReplay {
    const PlanArgs* a;
    const uint8_t* gexp;
    const uint8_t* glog;
    uint8_t* cwc;    // [p][q]
    uint8_t* datc;   // [i][q]
    uint8_t* fresh;  // [i][q]
    uint8_t* rv;     // wave rule: matrix columns [w][16]
    uint8_t* ra;     // wave rule: action columns [w][32]
    uint8_t* rent;   // wave rule: the entry {sel[k], col[k][n]}
    int lane, k, n, T;
    uint32_t er;     // erased positions of the block (uniform)

    __device__ uint8_t mul(uint8_t f, uint8_t v) const {
        return v ? gexp[glog[f] + glog[v]] : 0;
    }
    __device__ static void wsync() {  // LDS written by other lanes of this wave is visible
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }

    // The decode rule of (window w, erasure mask m) computed by the wave (codecs with n > 17 have
    // no rule table): gf256_rref_matrix (basicOperations.cpp:43-122) on the k x w matrix G[:, :w]
    // with erased columns zeroed, column by column -- pivot in row i+offset, a zero pivot swapped
    // with the first later column non-zero in that row (ballot), a row without one bumps the
    // offset, the pivot column normalised and eliminated from every other column (lane = column,
    // element-parallel swaps and scaling) -- then codingOperations.cpp:204-230's unit-column test
    // per erased data symbol (lane = symbol).  Same result as fec_host.cpp decode_rule.
    __device__ void wave_rule(int w, uint32_t m) {
        if (lane < w) {
            const bool e = (m >> lane) & 1u;
            for (int r = 0; r < k; ++r) rv[lane * 16 + r] = e ? 0 : a->G[r * n + lane];
            for (int r = 0; r < w; ++r) ra[lane * 32 + r] = r == lane ? 1 : 0;
        }
        wsync();
        int row = 0;
        for (int i = 0; i < w && row < k;) {
            if (rv[i * 16 + row] == 0) {
                const bool cand = lane > i && lane < w && rv[lane * 16 + row] != 0;
                const uint64_t bal = __builtin_amdgcn_ballot_w64(cand);
                if (!bal) {
                    ++row;
                    continue;
                }
                const int j = static_cast<int>(__builtin_ctzll(bal));
                if (lane < 16) {
                    const uint8_t x = rv[i * 16 + lane], y = rv[j * 16 + lane];
                    rv[i * 16 + lane] = y;
                    rv[j * 16 + lane] = x;
                }
                if (lane < 32) {
                    const uint8_t x = ra[i * 32 + lane], y = ra[j * 32 + lane];
                    ra[i * 32 + lane] = y;
                    ra[j * 32 + lane] = x;
                }
                wsync();
            }
            const uint8_t p = rv[i * 16 + row];
            const uint8_t s = gexp[255 - glog[p]];  // gf_inv
            wsync();
            if (lane < k) rv[i * 16 + lane] = mul(s, rv[i * 16 + lane]);
            if (lane < w) ra[i * 32 + lane] = mul(s, ra[i * 32 + lane]);
            wsync();
            if (lane < w && lane != i) {
                const uint8_t f = rv[lane * 16 + row];
                if (f) {
                    for (int r = 0; r < k; ++r) rv[lane * 16 + r] ^= mul(f, rv[i * 16 + r]);
                    for (int r = 0; r < w; ++r) ra[lane * 32 + r] ^= mul(f, ra[i * 32 + r]);
                }
            }
            wsync();
            ++i;
            ++row;
        }
        if (lane < k) {
            const int i = lane;
            uint8_t sel = 0xff;
            int j = i;
            while (j < k && rv[j * 16 + i] != 1) ++j;
            if (j < k) {
                bool unit = true;
                for (int r = i + 1; r < k; ++r) unit = unit && rv[j * 16 + r] == 0;
                if (unit) sel = static_cast<uint8_t>(j);
            }
            rent[i] = sel;
            for (int c = 0; c < w; ++c) rent[k + i * n + c] = sel == 0xff ? 0 : ra[j * 32 + c];
        }
        wsync();
    }

    // decodeBlock (codingOperations.cpp:149-232) on coefficient vectors.
    __device__ void decode_block(int t) {
        if (t < k && !((er >> t) & 1u) && lane < n) datc[t * n + lane] = cwc[t * n + lane];
        const int w = min(t + T + 1, n);
        const uint32_t full = (1u << w) - 1u;
        const uint32_t m = er & full;
        if (m == full || !(m & ((1u << k) - 1u))) return;
        uint32_t ev = 0, ev2 = 0;
        const bool tab = a->wbase[w] >= 0;
        if (tab) {
            // the whole rule entry {sel[k], col[k][n]} in one wave-wide load
            const uint32_t* ent = reinterpret_cast<const uint32_t*>(
                a->rules + a->wbase[w] + static_cast<int64_t>(m) * a->ES);
            // entries reach 4*77 bytes (k = 15, n = 17): two dwords per lane
            ev = (lane < (a->ES >> 2)) ? ent[lane] : 0u;
            ev2 = (lane + 64 < (a->ES >> 2)) ? ent[lane + 64] : 0u;
        } else {
            wave_rule(w, m);
        }
        auto rd = [&](int idx) -> uint32_t {
            if (!tab) return rent[idx];
            const int d = idx >> 2;
            const uint32_t wv = d < 64 ? __builtin_amdgcn_readlane(ev, d) : __builtin_amdgcn_readlane(ev2, d - 64);
            return (wv >> ((idx & 3) * 8)) & 0xffu;
        };
        uint32_t got = 0;
        for (int i = 0; i < k; ++i) {
            if (!((m >> i) & 1u)) continue;
            const uint32_t sel = rd(i);
            if (sel == 0xffu) continue;
            uint8_t acc = 0;
            const int base = k + i * n;
            for (int c = 0; c < w; ++c) {
                const int idx = base + c;
                const uint32_t f = rd(idx);
                if (!f || ((m >> c) & 1u)) continue;
                if (lane < n) acc ^= mul(static_cast<uint8_t>(f), cwc[c * n + lane]);
            }
            if (lane < n) fresh[i * n + lane] = acc;
            got |= 1u << i;
        }
        if (!got) return;
        for (int i = 0; i < k; ++i)
            if (((got >> i) & 1u) && lane < n) {
                const uint8_t v = fresh[i * n + lane];
                datc[i * n + lane] = v;
                cwc[i * n + lane] = v;
            }
        er &= ~got;
    }

    // Decoder_Block_Code::decodeSymbol (Decoder_Block_Code.cpp:61-78) at position p.
    __device__ void symbol(int p, bool erased) {
        if (erased) {
            er |= 1u << p;
        } else {
            er &= ~(1u << p);
            if (lane < n) cwc[p * n + lane] = (lane == p) ? 1 : 0;
        }
        if (p < T) return;
        decode_block(p - T);
        if (p == n - 1)
            for (int j = p - T + 1; j < k; ++j) decode_block(j);
    }

    // the packet fed at `time` reaches this block (b) at position (time - b) mod n
    __device__ void feed(int64_t time, int b, bool erased) {
        int p = static_cast<int>((time - b) % n);
        if (p < 0) p += n;
        symbol(p, erased);
    }
};
}  // namespace

// Erasure flags of 256 consecutive packets held in one register per lane (4 per lane), read with
// v_readlane: the serial replay then needs no dependent global load per packet.
struct ErWindow {
    const uint8_t* er;
    int64_t P;
    int64_t base = 0;
    uint32_t v = 0;
    int lane;
    __device__ void load(int64_t b) {
        base = b;
        const int64_t i = b + lane * 4;
        if (i >= 0 && i + 3 < P && ((reinterpret_cast<uintptr_t>(er + i) & 3) == 0)) {
            v = *reinterpret_cast<const uint32_t*>(er + i);
        } else {
            v = 0;
            for (int e = 0; e < 4; ++e)
                if (i + e >= 0 && i + e < P && er[i + e]) v |= 1u << (8 * e);
        }
    }
    __device__ bool get(int64_t t) const {  // t in [base, base + 256)
        const int d = static_cast<int>(t - base);
        return ((__builtin_amdgcn_readlane(v, d >> 2) >> ((d & 3) * 8)) & 0xffu) != 0;
    }
};

__global__ __launch_bounds__(64) void fec_plan_kernel(PlanArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x, k = a.k, n = a.n, T = a.T;
    BlockReplay br;
    br.a = &a;
    br.gexp = smem;
    br.glog = smem + 512;
    br.cwc = smem + 768;
    br.datc = br.cwc + n * n;
    br.fresh = br.datc + k * n;
    br.rv = br.fresh + k * n;
    br.ra = br.rv + 32 * 16;
    br.rent = br.ra + 32 * 32;
    br.lane = lane;
    br.k = k;
    br.n = n;
    br.T = T;
    for (int i = lane; i < 768; i += 64) smem[i] = a.gf[i];
    __syncthreads();
    const int64_t pairs = static_cast<int64_t>(a.counters[3]) * n;
    for (int64_t pr = blockIdx.x; pr < pairs; pr += gridDim.x) {
        const int64_t tr = a.episodes[a.work[pr / n]];
        const int b = static_cast<int>(pr % n);
        if (tr < 0 || tr >= a.P) continue;  // defensive: the scan only lists packets of the batch
        if (tr >= T) {
            // resync at tr (Decoder.cpp:111-133) from the initial state: precomputed per phase
            int phi = static_cast<int>((tr - b) % n);
            if (phi < 0) phi += n;
            const uint8_t* st = a.rstate + static_cast<int64_t>(phi) * a.rs_bytes;
            br.er = *reinterpret_cast<const uint32_t*>(st);
            if (lane < n) {
                for (int p = 0; p < n; ++p) br.cwc[p * n + lane] = st[4 + p * n + lane];
                for (int i = 0; i < k; ++i) br.datc[i * n + lane] = st[4 + n * n + i * n + lane];
            }
        } else {
            // startup: the replayed slots before packet 0 are empty (NULL), replay explicitly
            if (lane < n) {  // initial state of a Decoder_Block_Code: zeros, nothing erased
                for (int p = 0; p < n; ++p) br.cwc[p * n + lane] = 0;
                for (int i = 0; i < k; ++i) br.datc[i * n + lane] = 0;
            }
            br.er = 0;
            for (int i = 0; i < n - T; ++i) br.feed(tr + i, b, true);
            for (int i = 0; i < T; ++i)
                if (tr - T + i >= 0) br.feed(tr - T + i, b, false);
        }
        ErWindow win;
        win.er = a.er;
        win.P = a.P;
        win.lane = lane;
        win.load((tr - T) & ~static_cast<int64_t>(3));
        // positions are tracked incrementally (no 64-bit modulo per packet):
        //   p  = (t - b) mod n      position of packet t in this block's round
        //   ix = (t - T - b) mod n  position (= symbol index) of the output packet x = t - T
        int p = static_cast<int>((tr - b) % n);
        if (p < 0) p += n;
        int ix = p - (T % n);
        if (ix < 0) ix += n;
        const int Pi = static_cast<int>(a.P), Pouti = static_cast<int>(a.Pout);
        int latest = -1;
        for (int t = static_cast<int>(tr); t < Pi; ++t) {
            if (t >= win.base + 256) win.load((t - T) & ~3);
            const bool e = win.get(t);
            if (!e) {
                if (t - latest > T) break;  // Decoder.cpp:80-83: back to the fast path
            } else {
                latest = t;
            }
            br.symbol(p, e);
            const int x = t - T;
            const int i = ix;
            if (++p == n) p = 0;
            if (++ix == n) ix = 0;
            if (x < 0 || x >= Pouti || i >= k || !win.get(x)) continue;
            const bool ok = !((br.er >> i) & 1u);  // Decoder_Basic.cpp:76-79
            if (lane == 0) a.sym_ok[static_cast<int64_t>(x) * k + i] = ok ? 1 : 0;
            if (ok && lane < n) a.coef[(static_cast<int64_t>(x) * k + i) * n + lane] = br.datc[i * n + lane];
        }
    }
}

// ------------------------------------------------------------------------------------------
// Decode, step 4: erased packets.  A packet is recovered iff all k of its symbols are
// (Decoder_Basic.cpp:76-79); byte h (sub-stream s = h/k, position i = h%k) is then
// XOR_q coef[x][i][q] * cw[x-i+q][s*n+q] over the received symbols q of its diagonal.
// ------------------------------------------------------------------------------------------
constexpr int kRecMaxK = 16;  // = kMaxK (fec_host.h)
constexpr int kRecRounds = 5;  // 64-byte rounds per pass of fec_recover_kernel (L = 300: one pass)

// kRecMaxN = 17 (codecs with a rule table, the common case) or 32 (n up to 31)
template <int kRecMaxN>
__global__ __launch_bounds__(256) void fec_recover_kernel_t(RecArgs a) {
    // One wave per recovered packet (fec_compact_kernel's list), no workgroup barrier after the
    // table load: lane h computes bytes h, h+64, ... of [len_hi, len_lo, payload]; its n sources
    // are byte loads straight from the diagonal's rows (a ~(k+n)*CW-byte window, L2-resident), all
    // issued before the lookups.
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t lcf[4][kRecMaxK * kRecMaxN];  // per wave: coefficient logs, 255 = zero coefficient
    const int tid = threadIdx.x;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int lane = tid & 63, wl = tid >> 6;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW;
    const int nrec = a.counters[2];
    uint8_t* lc = lcf[wl];
    const int waves = gridDim.x * 4;
    if (a.zero_lost) {  // lost packets: payload 0 (FEC_Decoder returns no data), zero row
        const int ner = a.counters[1];
        for (int r = blockIdx.x * 4 + wl; r < ner; r += waves) {
            const int64_t x = a.erased[r];
            if (x < a.row_off) continue;
            bool ok = true;
            for (int i = 0; i < k; ++i) ok = ok && a.sym_ok[x * k + i];
            if (ok) continue;
            for (int b = lane; b < L; b += 64) a.out[(x - a.row_off) * L + b] = 0;
            if (lane == 0) a.out_len[x - a.row_off] = 0;
        }
    }
    for (int r = blockIdx.x * 4 + wl; r < nrec; r += waves) {
        const int64_t x = a.rec_list[r];
        if (x < a.row_off) continue;  // before the caller's first output row (wave-uniform)
        for (int i = lane; i < k * n; i += 64) {
            const uint8_t c = a.coef[x * k * n + i];
            lc[i] = c ? glog[c] : 255;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        // kRecRounds rounds of 64 bytes per pass: every source byte of the pass is loaded before
        // the first lookup, so the pass costs one memory round trip instead of one per round
        const uint8_t* __restrict__ cwp = a.cw;
        uint8_t* __restrict__ outp = a.out;
        int ln = 0;
        for (int h0 = 0; h0 < L + 2; h0 += 64 * kRecRounds) {
            uint8_t v[kRecRounds][kRecMaxN];
            int iw[kRecRounds];
#pragma unroll
            for (int rr = 0; rr < kRecRounds; ++rr) {
                const int h = h0 + 64 * rr + lane;
                const int sidx = h / k, i = h - sidx * k;
                iw[rr] = i;
#pragma unroll
                for (int q = 0; q < kRecMaxN; ++q) {
                    v[rr][q] = 0;
                    if (q < n && h < L + 2) {
                        const int64_t row = x - i + q;
                        if (lc[i * n + q] != 255 && row >= 0 && row < a.P) v[rr][q] = cwp[row * CW + sidx * n + q];
                    }
                }
            }
#pragma unroll
            for (int rr = 0; rr < kRecRounds; ++rr) {
                const int h = h0 + 64 * rr + lane;
                const int i = iw[rr];
                uint8_t acc = 0;
#pragma unroll
                for (int q = 0; q < kRecMaxN; ++q) {
                    if (q < n && v[rr][q]) {
                        const int lq = lc[i * n + q];
                        if (lq != 255) acc ^= gexp[lq + glog[v[rr][q]]];
                    }
                }
                if (h0 == 0 && rr == 0) {  // recovered length (Decoder.cpp:141-149): bytes 0, 1, clamped to L
                    const int hi = __builtin_amdgcn_readlane(static_cast<int>(acc), 0);
                    const int lo = __builtin_amdgcn_readlane(static_cast<int>(acc), 1);
                    ln = min(hi * 256 + lo, L);
                }
                const int b = h - 2;
                if (b >= 0 && b < L) outp[(x - a.row_off) * L + b] = b < ln ? acc : 0;
            }
        }
        if (lane == 0) a.out_len[x - a.row_off] = ln;
        __builtin_amdgcn_wave_barrier();  // lc is rewritten by the next packet
    }
}

template __global__ void fec_recover_kernel_t<17>(RecArgs);
template __global__ void fec_recover_kernel_t<32>(RecArgs);

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
