// fec_kernels.hip -- see fec_kernels.h for the map from reference functions to kernels.
#include "fec_device.h"
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
        if (!a.cw_len) break;  // (the caller does not want them: fec::encode_batch_nolen)
        const uint8_t* row = xout + tl * a.CW;
        a.cw_len[t0 + tl] = row[a.CW - 1] ? a.CW : last_nonzero_end(row, a.CW - 1);
    }
}

// Decode, step 1 (resync points, episodes, shapes, erased outputs): fec_episode_kernel,
// fec_shapes.hip.

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
    const int64_t pairs = static_cast<int64_t>(a.counters[6]) * n;
    const int64_t items = pairs + a.counters[7];
    for (int64_t pr = blockIdx.x; pr < items; pr += gridDim.x) {
        if (pr >= pairs) {
            episode_dup_fill(a, static_cast<int>(pr - pairs), lane);
            continue;
        }
        const int64_t tr = a.work[pr / n];
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
// Erased output packets whose k symbols are all recovered (their plan rows -- or their shape
// representative's -- say so, Decoder_Basic.cpp:76-79) -> rec_list as (x, x + src_d[x]) pairs,
// counted in counters[2]; the others are lost (zero_lost: their rows and lengths zeroed here).
// Lane (j, i) = symbol i of entry j, J = 64 / k entries per wave and round, one append atomic
// per wave and round.
__global__ __launch_bounds__(256) void fec_compact_kernel(CompactArgs a) {
    const int lane = threadIdx.x & 63, k = a.k;
    const int ner = a.counters[1];
    const int J = 64 / k;
    const int jl = lane / k, il = lane - jl * k;
    const int waves = gridDim.x * (blockDim.x >> 6);
    for (int r0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * J; r0 < ner; r0 += waves * J) {
        const int r = r0 + jl;
        const bool valid = jl < J && r < ner;
        int x = 0, xr = 0;
        bool bad = false;
        if (valid) {
            x = a.erased[r];
            xr = x + a.src_d[x];
            bad = !a.sym_ok[static_cast<int64_t>(xr) * k + il];
        }
        const uint64_t badm = __builtin_amdgcn_ballot_w64(bad);
        // a group's verdict on its first lane: no bad lane in [l0, l0 + k)
        const bool lead = valid && il == 0;
        uint64_t gbad = 0;
        for (int s = 0; s < k; ++s) gbad |= badm >> s;
        const bool ok = lead && !((gbad >> lane) & 1u);
        const uint64_t okm = __builtin_amdgcn_ballot_w64(ok);
        if (okm) {
            int base = 0;
            if (lane == __builtin_ctzll(okm)) base = atomicAdd(&a.counters[2], __builtin_popcountll(okm));
            base = __shfl(base, __builtin_ctzll(okm));
            if (ok) {
                const int at = base + __builtin_popcountll(okm & ((1ull << lane) - 1ull));
                a.rec_list[2 * at] = x;
                a.rec_list[2 * at + 1] = xr;
            }
        }
        if (a.zero_lost) {
            uint64_t lost = __builtin_amdgcn_ballot_w64(lead && !ok);
            while (lost) {
                const int l0 = __builtin_ctzll(lost);
                lost &= lost - 1;
                const int xl = __builtin_amdgcn_readlane(x, l0);
                if (xl < a.row_off) continue;
                for (int b = lane; b < a.L; b += 64) a.out[static_cast<int64_t>(xl - a.row_off) * a.L + b] = 0;
                if (lane == 0) a.out_len[xl - a.row_off] = 0;
            }
        }
    }
}

constexpr int kRecMaxK = 16;      // = kMaxK (fec_host.h)
constexpr int kRecLogZero = 512;  // log of 0: any sum with it indexes the zero tail of ex[]
constexpr int kRecStageChunks = 12;  // 16-byte pieces per lane of a staged span (<= 12 KB)

// One wave per erased output packet entry, 4 waves per workgroup, a grid of resident size: the
// wave's entries r = w, w + waves, ... are checked J = 64 / k at a time (lane (j, i) = symbol i
// of entry j: the dependent loads erased -> src_d -> sym_ok of all of them overlap), then the
// recovered ones (their plan rows -- or their shape representative's -- say all k symbols are,
// Decoder_Basic.cpp:76-79) are rebuilt one after the other:
//   * the k x n coefficient rows go to LDS as logs (0 -> kRecLogZero);
//   * STAGED: the k+n-1 codeword rows x-k+1 .. x+n-1 the diagonals of packet x touch are one
//     contiguous span of the codeword buffer; it lands in the wave's LDS region with 16-byte
//     loads issued together with the coefficient loads (one memory round trip), and every source
//     byte is an LDS read; otherwise (large codewords) every source byte is a byte load;
//   * lane h computes bytes h, h+64, ... of [len_hi, len_lo, payload]: sub-stream s = h / k,
//     position i = h % k, XOR_q coef[i][q] * cw[x-i+q][s*n+q] over the received symbols q, as n
//     independent branch-free terms ex[log coef + log byte] (a zero either way lands in the zero
//     tail of ex).
template <int MAXN, bool STAGED>
__global__ __launch_bounds__(256) void fec_recover_kernel_t(RecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t rsm[];
    uint8_t* ex = rsm;                                        // 1040: 2^i, zero from 512
    uint16_t* lg = reinterpret_cast<uint16_t*>(rsm + 1040);   // 256: log2 v, lg[0] = kRecLogZero
    const int tid = threadIdx.x;
    const int lane = tid & 63, wl = tid >> 6;
    const int L = a.L, k = a.k, n = a.n, CW = a.CW;
    constexpr int kLcBytes = (2 * kRecMaxK * MAXN + 15) & ~15;
    uint16_t* lc = reinterpret_cast<uint16_t*>(rsm + 1552 + wl * (kLcBytes + a.stage_bytes));
    uint8_t* rows = rsm + 1552 + wl * (kLcBytes + a.stage_bytes) + kLcBytes;
    phase_stamp(a.stamps, blockIdx.x, 0);
    for (int i = tid; i < 1040; i += 256) ex[i] = i < 512 ? a.gf[i] : 0;
    for (int i = tid; i < 256; i += 256) lg[i] = i ? a.gf[512 + i] : static_cast<uint16_t>(kRecLogZero);
    __syncthreads();
    phase_stamp(a.stamps, blockIdx.x, 1);
    const int nrec = a.counters[2];
    const int waves = gridDim.x * 4;
    const int64_t cw_total = a.P * CW;
    {
        for (int r = blockIdx.x * 4 + wl; r < nrec; r += waves) {
            const int x = a.rec_list[2 * r], xr = a.rec_list[2 * r + 1];
            if (x < a.row_off) continue;  // before the caller's first output row (wave-uniform)
            uint8_t* orow = a.out + static_cast<int64_t>(x - a.row_off) * L;
            // rows x-k+1 .. x+n-1 inside [0, P): bytes [s0, s1) of the codeword buffer
            const int rlo = x - k + 1 > 0 ? x - k + 1 : 0;
            const int64_t s0 = static_cast<int64_t>(rlo) * CW;
            const int64_t s1 = static_cast<int64_t>(x + n < a.P ? x + n : a.P) * CW;
            const int64_t a0 = s0 & ~int64_t(15);
            uint4 piece[STAGED ? kRecStageChunks : 1];
            const int nb = STAGED ? static_cast<int>((s1 - a0 + 15) >> 4) : 0;
            if constexpr (STAGED) {
#pragma unroll
                for (int j = 0; j < kRecStageChunks; ++j) {
                    const int c = lane + 64 * j;
                    const int64_t o = a0 + 16 * c;
                    piece[j] = make_uint4(0u, 0u, 0u, 0u);
                    if (c < nb) {
                        if (o + 16 <= cw_total) {
                            piece[j] = *reinterpret_cast<const uint4*>(a.cw + o);
                        } else {  // the buffer's last piece
                            uint32_t t[4] = {0u, 0u, 0u, 0u};
                            for (int e = 0; e < 16; ++e)
                                if (o + e < cw_total) t[e >> 2] |= static_cast<uint32_t>(a.cw[o + e]) << (8 * (e & 3));
                            piece[j] = make_uint4(t[0], t[1], t[2], t[3]);
                        }
                    }
                }
            }
            constexpr int kCf = (kRecMaxK * MAXN + 63) / 64;
            uint32_t cf[kCf];
            const uint8_t* cfp = a.coef + static_cast<int64_t>(xr) * k * n;
#pragma unroll
            for (int j = 0; j < kCf; ++j) cf[j] = lane + 64 * j < k * n ? cfp[lane + 64 * j] : 0u;
            if constexpr (STAGED) {
#pragma unroll
                for (int j = 0; j < kRecStageChunks; ++j)
                    if (lane + 64 * j < nb) *reinterpret_cast<uint4*>(rows + 16 * (lane + 64 * j)) = piece[j];
            }
#pragma unroll
            for (int j = 0; j < kCf; ++j)
                if (lane + 64 * j < k * n) lc[lane + 64 * j] = lg[cf[j]];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int ln = 0;
            for (int h0 = 0; h0 < L + 2; h0 += 64) {
                const int h = h0 + lane;
                const int sidx = h / k, i = h - sidx * k;
                // term q is row x-i+q: inside [0, P) for q in [qlo, qhi)
                const int qlo = i - x > 0 ? i - x : 0;
                const int qhi = h < L + 2 ? min(n, static_cast<int>(a.P - x) + i) : 0;
                // staged: byte (row, s*n+q) sits at base + q*(CW+1) of the span
                const int base = (x - i - rlo) * CW + static_cast<int>(s0 - a0) + sidx * n;
                uint32_t lq[MAXN], v[MAXN];
#pragma unroll
                for (int q = 0; q < MAXN; ++q) {
                    const bool use = q >= qlo && q < qhi;
                    lq[q] = lc[i * n + (q < n ? q : 0)];
                    if constexpr (STAGED) {
                        v[q] = use ? rows[base + q * (CW + 1)] : 0u;
                    } else {
                        v[q] = use ? a.cw[static_cast<int64_t>(x - i + q) * CW + sidx * n + q] : 0u;
                    }
                }
                uint32_t acc = 0;
#pragma unroll
                for (int q = 0; q < MAXN; ++q) acc ^= ex[lq[q] + lg[v[q]]];
                if (h0 == 0) {  // recovered length (Decoder.cpp:141-149): bytes 0, 1, clamped to L
                    const int hi = __builtin_amdgcn_readlane(static_cast<int>(acc), 0);
                    const int lo = __builtin_amdgcn_readlane(static_cast<int>(acc), 1);
                    ln = min(hi * 256 + lo, L);
                }
                const int b = h - 2;
                if (b >= 0 && b < L) orow[b] = b < ln ? static_cast<uint8_t>(acc) : 0;
            }
            if (lane == 0) a.out_len[x - a.row_off] = ln;
            __builtin_amdgcn_wave_barrier();  // lc and rows are rewritten by the next packet
        }
    }
    phase_stamp(a.stamps, blockIdx.x, 2);  // wave 0 done
}

template __global__ void fec_recover_kernel_t<17, true>(RecArgs);
template __global__ void fec_recover_kernel_t<17, false>(RecArgs);
template __global__ void fec_recover_kernel_t<32, false>(RecArgs);

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
