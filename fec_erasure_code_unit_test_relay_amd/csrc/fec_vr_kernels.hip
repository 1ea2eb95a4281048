// fec_vr_kernels.hip -- the byte work of a variable-rate schedule (fec_vr.h) in three launches:
// encode = one launch over every encoder instance of every (T,B,N) tuple, straight from the
// payload rows into the frames' arrays; decode = one copy launch for every received packet (each
// in its decoder's geometry) + one recovery launch over the host plan's coefficient rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "fec_amd.h"
#include "fec_device.h"
#include "fec_vr.h"
#include "fec_vr_cf.h"

namespace fec {
namespace {

// One wave per packet row.
__global__ __launch_bounds__(256) void fec_vr_frame_kernel(VrFrameArgs a) {
    const int lane = threadIdx.x & 63;
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); r < a.rows;
         r += static_cast<int64_t>(gridDim.x) * 4) {
        const int lc = a.len_cur[r], lo = a.len_old[r];
        uint8_t* o = a.packets + r * a.stride;
        const uint8_t* c = a.cur + a.cur_off[r];
        const uint8_t* d = a.old + a.old_off[r];
        if (lane < 10) {
            const int32_t* h = a.hdr + 4 * r;
            uint8_t v;
            switch (lane) {
                case 0: v = static_cast<uint8_t>((r >> 24) & 0xff); break;
                case 1: v = static_cast<uint8_t>((r >> 16) & 0xff); break;
                case 2: v = static_cast<uint8_t>((r >> 8) & 0xff); break;
                case 3: v = static_cast<uint8_t>(r & 0xff); break;
                case 8: v = static_cast<uint8_t>((lc - lc % 256) / 256); break;
                case 9: v = static_cast<uint8_t>(lc % 256); break;
                default: v = static_cast<uint8_t>(h[lane - 4]); break;
            }
            o[lane] = v;
        }
        for (int b = lane; b < lc; b += 64) o[10 + b] = c[b];
        for (int b = lane; b < lo; b += 64) o[10 + lc + b] = d[b];
        if (lane == 0) a.packet_len[r] = 10 + lc + lo;
    }
}

__global__ __launch_bounds__(256) void fec_vr_parse_kernel(VrParseArgs a) {
    const int lane = threadIdx.x & 63;
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); r < a.rows;
         r += static_cast<int64_t>(gridDim.x) * 4) {
        const uint8_t* p = a.packets + r * a.stride;
        const int plen = a.packet_len[r];
        const int lc = plen >= 10 ? p[8] * 256 + p[9] : 0;
        const int64_t lo = plen - 10 - lc;
        uint8_t* c = a.cur + a.cur_off[r];
        uint8_t* d = a.old + a.old_off[r];
        const int64_t wc = a.cur_off[r + 1] - a.cur_off[r], wo = a.old_off[r + 1] - a.old_off[r];
        for (int64_t b = lane; b < wc; b += 64) c[b] = b < lc ? p[10 + b] : 0;
        for (int64_t b = lane; b < wo; b += 64) d[b] = b < lo ? p[10 + lc + b] : 0;
        if (a.hdr && lane == 0) {
            int32_t* h = a.hdr + 5 * r;
            h[0] = (p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3];
            h[1] = p[4];
            h[2] = p[5];
            h[3] = p[6];
            h[4] = p[7];
        }
    }
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Each wave encodes a contiguous run of the codeword list, closed form of the diagonal
// interleaving (as fec_encode_kernel) with the instance's geometry at run time:
//     cw_seq[s*n + j] = X_seq[s][j]                                  j <  k
//     cw_seq[s*n + j] = XOR_{i<k} G[i][j] * X_{seq-(j-i)}[s][i]      j >= k
// over the instance's own packets (X before its first call = 0), X_r[s][i] = byte s*k+i of
// [len_hi, len_lo, payload, zero pad].  The wave keeps the last n rows in an LDS ring (slot
// r % n), each transposed to k planes of ceil(S/4) words (word g of plane i = X_r[4g..4g+3][i]),
// and loads one new row per codeword while it stays in one instance.  One lane task = (position j,
// group g of 4 sub-streams): a plane word, or k packed gf_mul4 products with the instance's
// register tables (staged in LDS per instance); its 4 bytes go to the LDS output row, which
// leaves as dword stores (bytes at the row's two ends).  The trimmed size is the last non-zero
// byte + 1 (FEC_Encoder.cpp:55-60), a wave max.
__global__ __launch_bounds__(256) void fec_vr_encode_kernel(VrEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint8_t* base = smem + wv * a.wave_bytes;
    uint32_t* tabw = reinterpret_cast<uint32_t*>(base);              // [k*(n-k)][8]
    uint8_t* outb = base + a.tab_bytes;                               // output row at offset head
    uint8_t* ring = outb + a.out_bytes;                               // n_max slots
    const int L = a.L;
    const int64_t total = a.cum[a.nenc];
    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (blockDim.x >> 6);
    const int64_t chunk = (total + nwaves - 1) / nwaves;
    const int64_t c0 = (static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + wv) * chunk;
    const int64_t c1 = min(total, c0 + chunk);
    if (c0 >= c1) return;
    int lo = 0, hi = a.nenc - 1;  // last e with cum[e] <= c0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.cum[mid] <= c0) lo = mid; else hi = mid - 1;
    }
    int e = lo, k = 0, n = 0, CW = 0, S = 0, NSG = 0, PL = 0, SB = 0;
    float rk = 1.0f;
    int64_t first = 0, sw = 0, next_row = 0;  // next_row: first row not yet in the ring
    const bool words = (L & 3) == 0 && (reinterpret_cast<uintptr_t>(a.payload) & 3) == 0;
    auto put = [&](uint8_t* slot, int q, uint32_t v) {  // X byte q -> plane q % k, column q / k
        const int sidx = static_cast<int>((static_cast<float>(q) + 0.5f) * rk);
        slot[(q - sidx * k) * PL + sidx] = static_cast<uint8_t>(v);
    };
    // rows r0..r1 into their ring slots: zeroed, then the header and payload bytes of every row
    // with its loads in flight together (a fresh instance needs n rows: one dependent HBM round
    // trip for all of them, not one per row)
    auto load_rows = [&](int64_t r0, int64_t r1) {
        const int nr = static_cast<int>(r1 - r0 + 1);
        const int sw_ = k * NSG;
        for (int d = lane; d < nr * sw_; d += 64) {
            const int rr = d / sw_;
            reinterpret_cast<uint32_t*>(ring + static_cast<int>(((r0 + rr) % n + n) % n) * SB)[d - rr * sw_] = 0;
        }
        wave_sync();
        auto row_len = [&](int64_t r) {
            int ln = a.len ? a.len[r] : L;
            return ln < 0 ? 0 : (ln > L ? L : ln);
        };
        for (int rr = lane; rr < nr; rr += 64) {
            const int64_t r = r0 + rr;
            if (r < first) continue;  // all-zero row before the instance's first call
            const int ln = row_len(r);
            uint8_t* slot = ring + static_cast<int>((r % n + n) % n) * SB;
            put(slot, 0, static_cast<uint32_t>(ln >> 8));
            put(slot, 1, static_cast<uint32_t>(ln & 0xff));
        }
        const int nw = words ? (L + 3) >> 2 : L;  // loads per row
        constexpr int kU = 4;
        for (int i0 = lane; i0 < nr * nw; i0 += 64 * kU) {
            uint32_t v[kU];
            int lim[kU], q0[kU];
            uint8_t* sl[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int idx = i0 + 64 * u;
                const int rr = idx / nw, w = idx - rr * nw;
                const int64_t r = r0 + rr;
                lim[u] = 0;
                v[u] = 0;
                sl[u] = ring;
                q0[u] = 0;
                if (idx < nr * nw && r >= first) {
                    const int ln = row_len(r);
                    const int b0 = words ? 4 * w : w;
                    if (b0 < ln) {
                        const uint8_t* src = a.payload + r * L;
                        v[u] = words ? *reinterpret_cast<const uint32_t*>(src + b0) : src[b0];
                        lim[u] = min(words ? 4 : 1, ln - b0);
                        q0[u] = b0 + 2;
                        sl[u] = ring + static_cast<int>((r % n + n) % n) * SB;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < kU; ++u)
                for (int b = 0; b < lim[u]; ++b) put(sl[u], q0[u] + b, v[u] >> (8 * b));
        }
    };
    for (int64_t c = c0; c < c1; ++c) {
        bool fresh = c == c0;
        while (a.cum[e + 1] <= c) {
            ++e;
            fresh = true;
        }
        if (fresh) {
            k = a.inst[4 * e];
            n = a.inst[4 * e + 1];
            CW = a.inst[4 * e + 2];
            S = CW / n;
            NSG = (S + 3) >> 2;
            PL = 4 * NSG;
            SB = k * PL;
            rk = 1.0f / static_cast<float>(k);
            first = a.span[2 * e];
            sw = a.span[2 * e + 1];
        }
        const int64_t seq = first + (c - a.cum[e]);
        wave_sync();  // earlier reads of the ring, tables and output row are done
        if (fresh) {
            const uint32_t* gt = a.gtab + a.inst[4 * e + 3];
            for (int i = lane; i < k * (n - k) * 8; i += 64) tabw[i] = gt[i];
            load_rows(seq - (n - 1), seq);
        } else {
            load_rows(next_row, seq);
        }
        next_row = seq + 1;
        const bool to_old = seq >= sw;
        const int64_t CWp = (CW + 15) & ~15;
        uint8_t* row = to_old ? a.old + a.base[2 * e + 1] + (seq - sw) * CWp : a.cur + a.base[2 * e] + (seq - first) * CWp;
        const int head = static_cast<int>(reinterpret_cast<uintptr_t>(row) & 3);
        wave_sync();
        const int slot_seq = static_cast<int>(seq % n);
        const float rg = 1.0f / static_cast<float>(NSG);
        for (int task = lane; task < n * NSG; task += 64) {
            const int j = static_cast<int>((static_cast<float>(task) + 0.5f) * rg);
            const int g = task - j * NSG;
            uint32_t v;
            if (j < k) {
                v = reinterpret_cast<const uint32_t*>(ring + slot_seq * SB + j * PL)[g];
            } else {
                v = 0;
                for (int i = 0; i < k; ++i) {
                    const uint32_t* t = tabw + (i * (n - k) + (j - k)) * 8;
                    if (!t[5]) continue;
                    int sl = slot_seq - (j - i);
                    sl += sl < 0 ? n : 0;
                    v ^= gf_mul4x(t, reinterpret_cast<const uint32_t*>(ring + sl * SB + i * PL)[g]);
                }
            }
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (4 * g + b < S) outb[head + (4 * g + b) * n + j] = static_cast<uint8_t>(v >> (8 * b));
        }
        wave_sync();
        const int nw = (head + CW + 3) >> 2;
        int last_nz = -1;
        for (int w = lane; w < nw; w += 64) {
            const uint32_t v = reinterpret_cast<const uint32_t*>(outb)[w];
            uint8_t* dst = row - head + 4 * w;
            const int p0 = 4 * w - head;  // row byte of word byte 0
            if (p0 >= 0 && p0 + 4 <= CW) {
                *reinterpret_cast<uint32_t*>(dst) = v;
                if (v) last_nz = p0 + 3 - (__builtin_clz(v) >> 3);
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int p = p0 + b;
                    if (p < 0 || p >= CW) continue;
                    const uint8_t x = static_cast<uint8_t>(v >> (8 * b));
                    dst[b] = x;
                    if (x) last_nz = p;
                }
            }
        }
        for (int o = 32; o > 0; o >>= 1) last_nz = max(last_nz, __shfl_xor(last_nz, o));
        if (lane == 0) (to_old ? a.len_old : a.len_cur)[seq] = last_nz + 1;
    }
}

// Instances of tuples with n = k (VrNp0Args): the codeword is X = [len BE16, payload, zero pad],
// so a row is the payload shifted by the 2 header bytes.  A thread per 16-byte chunk c of a row at
// stride W (the segment's rows x chunks flattened over the workgroup, every lane busy): the chunk's
// payload dwords 4c-1 .. 4c+3 (the header stands in for dword -1), shifted by 2 bytes, bytes past
// the length zeroed, one 16-byte store; the trimmed size (FEC_Encoder.cpp:55-60) is each row's max
// of the last non-zero byte + 1 (an LDS max per row).  In config 4 this is (10,0,0): 181 437 of the
// 360 010 codewords, which the tile encoder walked with its parity machinery idle.
__global__ __launch_bounds__(256) void fec_vr_encode_np0_kernel(VrNp0Args a) {
    __shared__ int s_last[kVrNp0Rows];
    const int64_t* sg = a.seg + 8 * blockIdx.x;
    const int64_t sfirst = sg[0], ssw = sg[1], P = sg[2];
    const int t0 = static_cast<int>(sg[3] & 0xffffffff), cnt = static_cast<int>(sg[3] >> 32);
    const int64_t scur = sg[4], sold = sg[5];
    const int W = static_cast<int>(sg[6] >> 32), NCH = W >> 4;
    const int64_t nsw = min(ssw - sfirst, P);  // rows from nsw on go to the old rows
    const int tid = threadIdx.x, L = a.L;
    if (tid < kVrNp0Rows) s_last[tid] = -1;
    __syncthreads();
    const float rch = 1.0f / static_cast<float>(NCH);
    for (int i = tid; i < cnt * NCH; i += 256) {
        const int rr = static_cast<int>((static_cast<float>(i) + 0.5f) * rch), c = i - rr * NCH;
        const int64_t t = t0 + rr, seq = sfirst + t;
        int ln = a.len ? a.len[seq] : L;
        ln = ln < 0 ? 0 : (ln > L ? L : ln);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.payload + seq * L);
        uint32_t d[5];
        if (16 * c + 16 <= L) {
            const uint4 v = *reinterpret_cast<const uint4*>(src + 4 * c);
            d[1] = v.x;
            d[2] = v.y;
            d[3] = v.z;
            d[4] = v.w;
        } else {
#pragma unroll
            for (int m = 1; m < 5; ++m) d[m] = 4 * (4 * c + m - 1) < L ? src[4 * c + m - 1] : 0u;
        }
        d[0] = c == 0 ? (static_cast<uint32_t>((ln >> 8) & 0xff) << 16) | (static_cast<uint32_t>(ln & 0xff) << 24)
                      : src[4 * c - 1];
        uint32_t o[4];
        int last = -1;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int q = 16 * c + 4 * m;  // X byte of o[m]'s byte 0
            o[m] = __builtin_amdgcn_alignbyte(d[m + 1], d[m], 2) & keep_bytes(ln + 2 - q);
            if (o[m]) last = q + 3 - (__builtin_clz(o[m]) >> 3);
        }
        if (last >= 0) atomicMax(&s_last[rr], last);
        const bool to_old = t >= nsw;
        uint8_t* row = to_old ? a.old + sold + (t - nsw) * W : a.cur + scur + t * W;
        *reinterpret_cast<uint4*>(row + 16 * c) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
    if (tid < cnt) {
        const int64_t t = t0 + tid;
        (t >= nsw ? a.len_old : a.len_cur)[sfirst + t] = s_last[tid] + 1;
    }
}

// fec_vr_encode_cf_kernel: the closed-form leftovers alone (fec_vr_cf.h)
__global__ __launch_bounds__(256) void fec_vr_encode_cf_kernel(VrEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    vr_encode_cf_body(a, smem, static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x));
}

// The copy's per-packet word, one thread per packet: geo[x] = k | n << 8 | fate << 16 | slow << 24
// in the reporting decoder's geometry (fate != 1: fate << 16 only).  Paying the chain fate ->
// decoder -> geometry once here, with a thread per packet, leaves the copy one level of dependent
// loads (its word) in front of the row bytes.  With a.tdesc, the first lane of each half-wave (a
// tile of kVrFastTP = 32 packets) also writes the tile's descriptor for fec_vr_copy_fast_kernel:
// its first cur row's offset, the geometry and row width shared by all its packets when every one
// is received in one geometry at one row width (else 0), and its slow bits (ballots over the half).
constexpr int kVrFastTP = 32;
static_assert(256 % 64 == 0 && 2 * kVrFastTP == 64, "a tile descriptor is a half-wave's");
struct VrTileDesc {  // fec_vr_copy_fast_kernel's tile of kVrFastTP packets
    int64_t o0;      // byte offset of its first cur row
    uint32_t g1, g2; // runs 1 and 2: k | n << 8 | row width << 16 (the received packets' geometry)
    uint16_t split;  // run 2's first packet (>= the tile's packets: one run)
    uint16_t ok;     // at most two runs, every received packet's row width < 64 KB, something received
    uint32_t slow, recv, rec;  // bit t: packet t on the slow path / received (fate 1) / recovered (fate 2)
};
static_assert(sizeof(VrTileDesc) == 32, "descriptor size (fec_vr.cpp reserves 32 bytes per tile)");
__global__ __launch_bounds__(256) void fec_vr_geo_kernel(VrCopyArgs a) {
    const int64_t x = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    const bool in = x < a.P;
    uint32_t g = 0;
    int rw = 0;
    if (in) {
        const uint32_t f = a.fate[x];
        g = f << 16;
        if (f == 1) {
            const int j = a.pk_dec[x];
            g |= static_cast<uint32_t>(a.inst[4 * j]) | static_cast<uint32_t>(a.inst[4 * j + 1]) << 8 |
                 (a.slow[x] ? 1u << 24 : 0u);
        }
        a.geo[x] = g;
        rw = static_cast<int>(a.cur_off[x + 1] - a.cur_off[x]);
    }
    if (a.tdesc == nullptr) return;  // uniform over the grid
    // the tile's runs: run 1 = packets [0, split), run 2 = [split, np), each one row width over all
    // its packets and one geometry over its received ones (run 1's taken from the tile's first
    // received packet; a run without one takes the other's, its rows being zero or the recovery's)
    const int lane = static_cast<int>(threadIdx.x & 63), h = lane & 32, li = lane & 31;
    const bool recv = in && ((g >> 16) & 0xff) == 1, rec = in && ((g >> 16) & 0xff) == 2;
    const int kn = static_cast<int>(g & 0xffff);
    const uint32_t recv_h = static_cast<uint32_t>(__ballot(recv) >> h);
    const uint32_t rec_h = static_cast<uint32_t>(__ballot(rec) >> h);
    const uint32_t slow_h = static_cast<uint32_t>(__ballot(in && (g >> 24) != 0) >> h);
    const uint32_t wide_h = static_cast<uint32_t>(__ballot(in && rw > 0xffff) >> h);
    const int rw1 = __shfl(rw, h);
    const int kn_first = __shfl(kn, h + (recv_h ? __builtin_ctz(recv_h) : 0));
    const uint32_t diff_h = static_cast<uint32_t>(__ballot(in && (rw != rw1 || (recv && kn != kn_first))) >> h);
    const int split = diff_h ? __builtin_ctz(diff_h) : 32;
    const uint32_t recv2 = split < 32 ? recv_h & (~0u << split) : 0u;
    const int rw2 = __shfl(rw, h + (split < 32 ? split : 0));
    const int kn2 = recv2 ? __shfl(kn, h + __builtin_ctz(recv2)) : kn_first;
    const uint32_t bad_h =
        static_cast<uint32_t>(__ballot(in && li >= split && (rw != rw2 || (recv && kn != kn2))) >> h);
    const uint32_t key1 = static_cast<uint32_t>(kn_first) | static_cast<uint32_t>(rw1 & 0xffff) << 16;
    const uint32_t key2 = static_cast<uint32_t>(kn2) | static_cast<uint32_t>(rw2 & 0xffff) << 16;
    if (li == 0 && in) {
        VrTileDesc d;
        d.o0 = a.cur_off[x];
        d.g1 = key1;
        d.g2 = split < 32 ? key2 : 0u;
        d.split = static_cast<uint16_t>(min<int64_t>(split, a.P - x));
        d.ok = (recv_h != 0 && bad_h == 0 && wide_h == 0) ? 1 : 0;  // (rows at one stride per run)
        d.slow = slow_h;
        d.recv = recv_h;
        d.rec = rec_h;
        reinterpret_cast<VrTileDesc*>(a.tdesc)[x / kVrFastTP] = d;
    }
}

// The received packets' systematic copies for L % 4 != 0 (or rows too long for the output tile
// below): a tile of kVrCopyTP consecutive packets per workgroup:
// their cur rows are one contiguous span of the compact layout, read with 16-byte loads into LDS
// next to a per-packet record (row offset and width, geometry, copied length); then each thread
// makes output dwords (payload byte b = codeword byte (h / k) * n + h % k of the reporting
// decoder's geometry, fec_vr_geo_kernel's word, h = b + 2; the header at symbols 0 and 1 of
// sub-stream 0, k = 1: position 0 of sub-streams 0 and 1, Decoder.cpp:89-96; the slow path clamps
// the length, :148-149), and the tile's payload rows leave as one contiguous run.  A tile wider
// than the stage (rows of k <= 3) gathers from HBM.  Lost packets get a zero row and length 0;
// recovered ones are left to fec_vr_recover_kernel.  Bytes past a row read as zero.
constexpr int kVrCopyTP = 16;
constexpr int kVrCopyStage = 16384;
__global__ __launch_bounds__(256) void fec_vr_copy_gather_kernel(VrCopyArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kVrCopyStage];
    __shared__ int s_ro[kVrCopyTP], s_rw[kVrCopyTP], s_kn[kVrCopyTP], s_cp[kVrCopyTP];
    __shared__ float s_rk[kVrCopyTP];
    const int tid = threadIdx.x;
    const int L = a.L, L4 = (L + 3) >> 2;
    const float rl4 = 1.0f / static_cast<float>(L4);
    const int64_t ntiles = (a.P + kVrCopyTP - 1) / kVrCopyTP;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t x0 = tile * kVrCopyTP;
        const int np = static_cast<int>(min<int64_t>(kVrCopyTP, a.P - x0));
        const int64_t o0 = a.cur_off[x0];
        const int64_t span = a.cur_off[x0 + np] - o0;
        const bool staged = span <= kVrCopyStage;  // uniform over the workgroup
        if (staged) {
            const uint4* src = reinterpret_cast<const uint4*>(a.cur + o0);
            for (int c = tid; 16 * c < span; c += 256) reinterpret_cast<uint4*>(stage)[c] = src[c];
        }
        int ln = 0;
        if (tid < np) {
            const int64_t x = x0 + tid;
            const uint32_t g = a.geo[x];
            const int64_t ro = a.cur_off[x];
            s_ro[tid] = static_cast<int>(ro - o0);
            s_rw[tid] = static_cast<int>(a.cur_off[x + 1] - ro);
            const int f = static_cast<int>(g >> 16 & 0xff);
            const int k = f == 1 ? static_cast<int>(g & 0xff) : 1;
            s_kn[tid] = f == 1 ? static_cast<int>(g & 0xffff) : (f == 2 ? -1 : 0);  // -1: recovered, 0: lost
            s_rk[tid] = 1.0f / static_cast<float>(k);
        }
        __syncthreads();
        if (tid < np) {  // the header of a received packet: its length, clamped on the slow path
            const int64_t x = x0 + tid;
            const int kn = s_kn[tid];
            if (kn > 0) {
                const int k = kn & 0xff, n = kn >> 8, rw = s_rw[tid];
                const uint8_t* lrow = stage + s_ro[tid];
                const uint8_t* grow = a.cur + o0 + s_ro[tid];
                const int p1 = k > 1 ? 1 : n;
                const int h0 = rw > 0 ? (staged ? lrow[0] : grow[0]) : 0;
                const int h1 = p1 < rw ? (staged ? lrow[p1] : grow[p1]) : 0;
                const int hdr = h0 * 256 + h1;
                ln = (a.geo[x] >> 24) ? min(hdr, L) : hdr;
            }
            if (kn >= 0) a.out_len[x] = ln;
            s_cp[tid] = min(ln, L);
        }
        __syncthreads();
        for (int d = tid; d < np * L4; d += 256) {
            const int p = static_cast<int>((static_cast<float>(d) + 0.5f) * rl4);
            const int w = d - p * L4;
            const int kn = s_kn[p];
            if (kn < 0) continue;  // recovered: fec_vr_recover_kernel's row
            const int cp = s_cp[p], b0 = 4 * w;
            uint32_t val = 0;
            if (b0 < cp) {
                const int k = kn & 0xff, n = kn >> 8, rw = s_rw[p];
                const uint8_t* lrow = stage + s_ro[p];
                const uint8_t* grow = a.cur + o0 + s_ro[p];
                const int h = b0 + 2;
                int sidx = static_cast<int>((static_cast<float>(h) + 0.5f) * s_rk[p]);
                int i = h - sidx * k;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int pos = sidx * n + i;
                    if (b0 + e < cp && pos < rw) val |= static_cast<uint32_t>(staged ? lrow[pos] : grow[pos]) << (8 * e);
                    if (++i == k) {
                        i = 0;
                        ++sidx;
                    }
                }
            }
            uint8_t* o = a.out + (x0 + p) * L;
            if ((L & 3) == 0) {
                *reinterpret_cast<uint32_t*>(o + b0) = val;
            } else {
                for (int e = 0; e < 4 && b0 + e < L; ++e) o[b0 + e] = static_cast<uint8_t>(val >> (8 * e));
            }
        }
        __syncthreads();  // the stage and records are read before the next tile's
    }
}

// The received packets' systematic copies, a tile of kVrCopyTP consecutive packets per workgroup:
// their cur rows are one contiguous span of the compact layout, read with 16-byte loads into LDS
// next to a per-packet record (row offset and width, geometry, copied length).  Then a half-wave
// per packet and a lane per sub-stream s: the sub-stream's k systematic bytes (row bytes
// [s*n, s*n+k), three dword shifts) go to bytes [s*k, s*k+k) of the packet's [header, payload]
// image in an LDS output tile, as 12 byte writes in reverse order -- the writes past k land in
// the next sub-stream's bytes first and that lane's own writes come later, so no lane needs k at
// compile time or a per-byte test (a thread per output dword instead spent a division and four
// dependent byte positions per dword: 88.9 vs 81.4 us on the schedule of bin/erasure.bin,
// tools/ubench/vr_copy_real.hip).  The header (symbols 0 and 1 of sub-stream 0, k = 1: position 0
// of sub-streams 0 and 1, Decoder.cpp:89-96) gives the length, clamped on the slow path
// (:148-149); the tile's payload rows leave as one contiguous run of 16-byte stores, bytes past a
// packet's copied length zero.  A tile wider than the stage (rows of k <= 3) gathers from HBM into
// the output tile.  Lost packets get a zero row and length 0; recovered ones are left to
// fec_vr_recover_kernel.  Needs L % 4 == 0 (output dwords inside one row).
constexpr int kVrCopyOrs = 32;  // output tile row = L + 32 bytes: [6 guard][header 2][payload][spill]
// One tile of at most kVrCopyTP packets from x0 (stage: kVrCopyStage + 16 bytes, otile: kVrCopyTP
// rows of L + kVrCopyOrs bytes; every thread of the workgroup calls it).
__device__ void vr_copy_tile_generic(const VrCopyArgs& a, int64_t x0, int np, uint8_t* stage, uint8_t* otile) {
    __shared__ int s_ro[kVrCopyTP], s_rw[kVrCopyTP], s_kn[kVrCopyTP], s_cp[kVrCopyTP], s_S[kVrCopyTP];
    const int tid = threadIdx.x, l32 = tid & 31, hw = tid >> 5;
    const int L = a.L, ors = L + kVrCopyOrs;
    {
        const int64_t o0 = a.cur_off[x0];
        const int64_t span = a.cur_off[x0 + np] - o0;
        const bool staged = span <= kVrCopyStage;  // uniform over the workgroup
        if (staged) {
            const uint4* src = reinterpret_cast<const uint4*>(a.cur + o0);
            for (int c = tid; 16 * c < span; c += 256) reinterpret_cast<uint4*>(stage)[c] = src[c];
        }
        if (tid < np) {
            const int64_t x = x0 + tid;
            const uint32_t g = a.geo[x];
            const int64_t ro = a.cur_off[x];
            s_ro[tid] = static_cast<int>(ro - o0);
            s_rw[tid] = static_cast<int>(a.cur_off[x + 1] - ro);
            const int f = static_cast<int>(g >> 16 & 0xff);
            const int k = f == 1 ? static_cast<int>(g & 0xff) : 1;
            s_kn[tid] = f == 1 ? static_cast<int>(g & 0xffff) : (f == 2 ? -1 : 0);  // -1: recovered, 0: lost
            s_S[tid] = (L + 2 + k - 1) / k;
        }
        __syncthreads();
        if (tid < np) {  // the header of a received packet: its length, clamped on the slow path
            const int64_t x = x0 + tid;
            const int kn = s_kn[tid];
            int ln = 0;
            if (kn > 0) {
                const int k = kn & 0xff, n = kn >> 8, rw = s_rw[tid];
                const uint8_t* lrow = stage + s_ro[tid];
                const uint8_t* grow = a.cur + o0 + s_ro[tid];
                const int p1 = k > 1 ? 1 : n;
                const int h0 = rw > 0 ? (staged ? lrow[0] : grow[0]) : 0;
                const int h1 = p1 < rw ? (staged ? lrow[p1] : grow[p1]) : 0;
                const int hdr = h0 * 256 + h1;
                ln = (a.geo[x] >> 24) ? min(hdr, L) : hdr;
            }
            if (kn >= 0) a.out_len[x] = ln;
            s_cp[tid] = min(ln, L);
        }
        if (staged) {
            for (int pp = hw; pp < np; pp += 8) {
                const int kn = s_kn[pp];
                if (kn <= 0) continue;
                const int k = kn & 0xff, n = kn >> 8, S = s_S[pp];
                const int ro = s_ro[pp];
                uint8_t* img = otile + pp * ors + 6;  // byte q of the packet's [header, payload]
                for (int sb = l32; sb < S; sb += 32) {
                    const int aa = ro + sb * n;  // rows start 16-byte aligned in the stage
                    const uint32_t* src = reinterpret_cast<const uint32_t*>(stage + (aa & ~3));
                    const uint32_t d0 = src[0], d1 = src[1], d2 = src[2], d3 = src[3];
                    const int sh = aa & 3;
                    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
                    const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
                    const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
                    uint8_t* dst = img + sb * k;
                    dst[11] = static_cast<uint8_t>(w2 >> 24);
                    dst[10] = static_cast<uint8_t>(w2 >> 16);
                    dst[9] = static_cast<uint8_t>(w2 >> 8);
                    dst[8] = static_cast<uint8_t>(w2);
                    dst[7] = static_cast<uint8_t>(w1 >> 24);
                    dst[6] = static_cast<uint8_t>(w1 >> 16);
                    dst[5] = static_cast<uint8_t>(w1 >> 8);
                    dst[4] = static_cast<uint8_t>(w1);
                    dst[3] = static_cast<uint8_t>(w0 >> 24);
                    dst[2] = static_cast<uint8_t>(w0 >> 16);
                    dst[1] = static_cast<uint8_t>(w0 >> 8);
                    dst[0] = static_cast<uint8_t>(w0);
                }
            }
        } else {
            const int L4 = L >> 2;
            for (int d = tid; d < np * L4; d += 256) {
                const int p = d / L4, w = d - p * L4;
                const int kn = s_kn[p];
                if (kn <= 0) continue;
                const int k = kn & 0xff, n = kn >> 8, rw = s_rw[p];
                const uint8_t* grow = a.cur + o0 + s_ro[p];
                const int h = 4 * w + 2;
                int sidx = h / k, i = h - sidx * k;
                uint32_t val = 0;
                for (int e = 0; e < 4; ++e) {
                    const int pos = sidx * n + i;
                    if (pos < rw) val |= static_cast<uint32_t>(grow[pos]) << (8 * e);
                    if (++i == k) {
                        i = 0;
                        ++sidx;
                    }
                }
                *reinterpret_cast<uint32_t*>(otile + p * ors + 8 + 4 * w) = val;
            }
        }
        __syncthreads();
        const int ob = np * L;
        uint8_t* dst = a.out + x0 * L;
        const bool al16 = ((reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
        // chunk o = bytes [o, o+16) of the tile's rows: row p, byte off; both advance without a
        // division (L % 4 == 0: a dword never straddles two rows)
        const int step_p = 4096 / L, step_off = 4096 - step_p * L;
        int p0 = (16 * tid) / L, off0 = 16 * tid - p0 * L;
        for (int o = 16 * tid; o < ob; o += 16 * 256) {
            uint32_t v[4];
            bool skip[4], any_skip = false;
            int p = p0, off = off0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (off >= L) {
                    off -= L;
                    ++p;
                }
                const int oq = o + 4 * q;
                skip[q] = oq >= ob || s_kn[p < np ? p : 0] < 0;
                any_skip |= skip[q];
                v[q] = skip[q] ? 0u : *reinterpret_cast<const uint32_t*>(otile + p * ors + 8 + off) & keep_bytes(s_cp[p] - off);
                off += 4;
            }
            p0 += step_p;
            off0 += step_off;
            if (off0 >= L) {
                off0 -= L;
                ++p0;
            }
            if (!any_skip && al16) {
                *reinterpret_cast<uint4*>(dst + o) = make_uint4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (!skip[q]) *reinterpret_cast<uint32_t*>(dst + o + 4 * q) = v[q];
            }
        }
        __syncthreads();  // the stage, records and output tile are read before the next tile's
    }
}

__global__ __launch_bounds__(256) void fec_vr_copy_kernel(VrCopyArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kVrCopyStage + 16];
    extern __shared__ __attribute__((aligned(16))) uint8_t otile[];
    const int64_t ntiles = (a.P + kVrCopyTP - 1) / kVrCopyTP;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t x0 = tile * kVrCopyTP;
        vr_copy_tile_generic(a, x0, static_cast<int>(min<int64_t>(kVrCopyTP, a.P - x0)), stage, otile);
    }
}


// The received packets' copies specialised on the reporting decoders' (k, n-k): a workgroup per tile
// of kVrFastTP consecutive packets, described by fec_vr_geo_kernel (VrTileDesc).  A tile whose
// received packets form at most two runs of one geometry each (a decoder switch inside the tile)
// with a specialisation below (the adaptive tuples (10, b, b) with k >= 4) is the headline copy
// (fec_copy_fast.hip) at the compact layout's row stride, without a stage: a lane per (packet,
// group of 4 sub-streams), 64 / NS4 packets per wave, the group's 4n codeword bytes loaded straight
// into registers (buffer loads at dword alignment; reads past cur return zero), the 4k systematic
// bytes picked with constant-selector v_perm_b32 and written, shifted by the 2 header bytes, to the
// LDS output tile; the length (header at symbols 0 and 1 of sub-stream 0, from the packet's first
// lane by a lane shuffle) clamped on the slow path (Decoder.cpp:148-149).  A lost packet gets a zero
// row and length 0; a recovered one is left alone (fec_vr_recover_kernel writes it meanwhile: the
// tile's rows leave as 16-byte stores, dword stores around such a row).  Every other tile (three
// or more runs, k <= 3, nothing received) takes the per-packet path above, as two tiles of
// kVrCopyTP.  (Staging the rows in LDS first, as the headline copy does, measured slower here:
// 82.5 vs 65.4 us, profiles/r05/vr/r05zb_*: at the compact layout's 16-byte row stride the
// gather's dword reads conflict 4- to 16-way.)
constexpr int kVrFastStage = kVrCopyStage + 16;  // the per-packet path's stage

template <int NW>
__device__ __forceinline__ void load_dwords(__amdgpu_buffer_rsrc_t r, int off, uint32_t (&D)[NW]) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int c = 0; c + 4 <= NW; c += 4) {
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off + 4 * c, 0, 0);
        D[c] = v.x;
        D[c + 1] = v.y;
        D[c + 2] = v.z;
        D[c + 3] = v.w;
    }
    constexpr int c0 = NW & ~3, rem = NW & 3;
    if constexpr (rem >= 2) {
        const v2u v = __builtin_amdgcn_raw_buffer_load_b64(r, off + 4 * c0, 0, 0);
        D[c0] = v.x;
        D[c0 + 1] = v.y;
    }
    if constexpr (rem == 1 || rem == 3) D[NW - 1] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * (NW - 1), 0, 0);
}

// Packets [lo, hi) of the tile (one geometry, rows from byte ob of cur at stride rw) into the
// output tile xo (row t at t * L) and their lengths.
template <int K, int NP>
__device__ __forceinline__ void vr_copy_run_direct(const VrCopyArgs& a, const VrTileDesc& d, int64_t x0, int lo, int hi,
                                                   int64_t ob, int rw, uint8_t* xo) {
    constexpr int n = K + NP;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, L = a.L;
    const int S = (L + 2 + K - 1) / K, NS4 = (S + 3) >> 2;
    const int ppw = 64 / NS4;  // NS4 <= 64 (the caller's condition)
    const int pl = lane / NS4, g = lane - pl * NS4;
    const int64_t left = a.cur_bytes - ob;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(a.cur + ob), 0, static_cast<int>(left < fec::kRsrcMax ? left : fec::kRsrcMax), 0x00020000);
    for (int p0 = lo + wv * ppw; p0 < hi; p0 += 4 * ppw) {
        const int t = p0 + pl;
        const bool on = pl < ppw && t < hi;
        const bool recv = on && ((d.recv >> t) & 1u), rec = on && ((d.rec >> t) & 1u);
        uint32_t D[n];
        load_dwords<n>(r, recv ? (t - lo) * rw + 4 * n * g : 0x7ffffff0, D);
        // header (symbols 0 and 1 of sub-stream 0: bytes 0 and 1 for k > 1) on the packet's first lane
        const int hdr = static_cast<int>(((D[0] & 0xff) << 8) | ((D[0] >> 8) & 0xff));
        const int ln0 = !recv ? 0 : (((d.slow >> t) & 1u) ? min(hdr, L) : hdr);
        const int ln = __shfl(ln0, pl * NS4);
        if (on && !rec && g == 0) a.out_len[x0 + t] = ln;
        const int cl = min(ln, L);
        if (!on || rec) continue;
        uint32_t W[K + 1];
#pragma unroll
        for (int m = 0; m < K; ++m) {
            const int i0 = 4 * m, i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3;
            W[m] = gather4(D, (i0 / K) * n + i0 % K, (i1 / K) * n + i1 % K, (i2 / K) * n + i2 % K,
                           (i3 / K) * n + i3 % K);
        }
        W[K] = 0;
        uint8_t* orow = xo + t * L;  // payload bytes [4gK-2, 4gK+4K-2): head 2, K-1 dwords, tail 2
        const int bh = 4 * g * K - 2;
        if (bh >= 0 && bh < L) *reinterpret_cast<uint16_t*>(orow + bh) = static_cast<uint16_t>(W[0] & keep_bytes(cl - bh));
#pragma unroll
        for (int m = 0; m < K - 1; ++m) {
            const int b = 4 * g * K + 4 * m;
            if (b < L)
                *reinterpret_cast<uint32_t*>(orow + b) = __builtin_amdgcn_alignbyte(W[m + 1], W[m], 2) & keep_bytes(cl - b);
        }
        const int bt = 4 * g * K + 4 * K - 4;
        if (bt < L) *reinterpret_cast<uint16_t*>(orow + bt) = static_cast<uint16_t>((W[K - 1] >> 16) & keep_bytes(cl - bt));
    }
}

#define FEC_VR_FAST_LIST(X) X(11, 0) X(10, 1) X(9, 2) X(8, 3) X(7, 4) X(6, 5) X(5, 6) X(4, 7)

// Is (k | n << 8) one of the specialisations, with a packet's groups inside one wave (NS4 <= 64)?
__device__ __forceinline__ bool vr_direct_ok(int kn, int L) {
    switch (kn) {
#define FEC_VR_DIRECT_OK(K, NP) \
    case K | ((K + NP) << 8): return (L + 2 + K - 1) / K <= 256;
        FEC_VR_FAST_LIST(FEC_VR_DIRECT_OK)
#undef FEC_VR_DIRECT_OK
        default: return false;
    }
}

// One tile of fec_vr_copy_fast_kernel.
__device__ __forceinline__ void vr_copy_fast_tile(const VrCopyArgs& a, int64_t tile, const VrTileDesc& d, uint8_t* stage,
                                                  uint8_t* xo) {
    const int64_t x0 = tile * kVrFastTP;
    const int np = static_cast<int>(min<int64_t>(kVrFastTP, a.P - x0));
    const int L = a.L;
    const int kn1 = static_cast<int>(d.g1 & 0xffff), rw1 = static_cast<int>(d.g1 >> 16);
    const int kn2 = static_cast<int>(d.g2 & 0xffff), rw2 = static_cast<int>(d.g2 >> 16);
    const int split = static_cast<int>(d.split);  // np: one run
    if (d.ok && vr_direct_ok(kn1, L) && (split >= np || vr_direct_ok(kn2, L))) {
        // the two runs as straight-line code (in a loop, the cases' loop invariants were hoisted
        // in front of it all together: 145 VGPRs against 42 for one case)
        auto run = [&](int lo, int hi, int kn, int rw, int64_t ob) __attribute__((always_inline)) {
            switch (kn) {
#define FEC_VR_DIRECT_CASE(K, NP) \
    case K | ((K + NP) << 8): vr_copy_run_direct<K, NP>(a, d, x0, lo, hi, ob, rw, xo); break;
                FEC_VR_FAST_LIST(FEC_VR_DIRECT_CASE)
#undef FEC_VR_DIRECT_CASE
                default: break;
            }
        };
        run(0, min(split, np), kn1, rw1, d.o0);
        if (split < np) run(split, np, kn2, rw2, d.o0 + static_cast<int64_t>(split) * rw1);
        __syncthreads();
        const int tid = threadIdx.x;
        const int ob = np * L;
        uint8_t* dst = a.out + x0 * L;
        if ((ob & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            for (int o = 16 * tid; o < ob; o += 16 * 256) {
                const uint4 v = *reinterpret_cast<const uint4*>(xo + o);
                if (d.rec == 0) {
                    nt_store16(dst + o, v);
                } else {  // rows of recovered packets are the recovery's (L % 4 == 0: dwords in one row)
                    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (!((d.rec >> ((o + 4 * q) / L)) & 1u)) *reinterpret_cast<uint32_t*>(dst + o + 4 * q) = w4[q];
                }
            }
        } else {
            for (int o = 4 * tid; o < ob; o += 4 * 256)
                if (!((d.rec >> (o / L)) & 1u)) *reinterpret_cast<uint32_t*>(dst + o) = *reinterpret_cast<const uint32_t*>(xo + o);
        }
        return;
    }
    for (int h = 0; h < kVrFastTP && h < np; h += kVrCopyTP)
        vr_copy_tile_generic(a, x0 + h, min(kVrCopyTP, np - h), stage, xo);
}

// A workgroup per tile (resident workgroups walking several tiles, the next descriptor loaded
// ahead, measured slower: 88.0 vs 83.7 us, and they held the recovery's waves off the CUs until
// the copy's end, 90 vs 61 us; profiles/r05/vr/r05z_*).
__global__ __launch_bounds__(256) void fec_vr_copy_fast_kernel(VrCopyArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* stage = smem;                    // kVrFastStage (the per-packet path)
    uint8_t* xo = smem + kVrFastStage;        // output tile: kVrFastTP rows of L (per-packet path: kVrCopyTP of L + 32)
    const int64_t tile = blockIdx.x;
    const VrTileDesc* dp = reinterpret_cast<const VrTileDesc*>(a.tdesc) + tile;
    VrTileDesc d;  // one scalar load of the descriptor in front of the row bytes
    d.o0 = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->o0 & 0xffffffff)) & 0xffffffffu) |
           static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->o0 >> 32))) << 32;
    d.g1 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->g1)));
    d.g2 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->g2)));
    d.split = static_cast<uint16_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->split)));
    d.ok = static_cast<uint16_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->ok)));
    d.slow = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->slow)));
    d.recv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->recv)));
    d.rec = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->rec)));
    vr_copy_fast_tile(a, tile, d, stage, xo);
}

// Per-row offsets of the compact layout, one thread per row s: e = the last instance with
// first_e <= s (binary search); cur row at base_cur_e + (s - first_e) * CWp_e; the same seq's old
// row belongs to instance e-1 while s < end_{e-1} (double coding), else it is empty (offset = where
// e's old block begins, base_old_e).
__global__ __launch_bounds__(256) void fec_vr_offsets_kernel(VrOffsetsArgs a) {
    const int64_t s = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (s == 0) {
        a.cur_off[a.rows] = a.cur_total;
        a.old_off[a.rows] = a.old_total;
    }
    if (s >= a.rows) return;
    int lo = 0, hi = a.nenc - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.inst[6 * mid] <= s) lo = mid; else hi = mid - 1;
    }
    const int64_t* me = a.inst + 6 * lo;
    a.cur_off[s] = me[4] + (s - me[0]) * me[3];
    const int64_t* pv = lo > 0 ? me - 6 : nullptr;
    a.old_off[s] = (pv && s >= pv[1] && s < pv[2]) ? pv[5] + (s - pv[1]) * pv[3] : me[5];
}

// One wave per recovered packet (as fec_recover_kernel): byte h = (sub-stream h/k, position i =
// h%k) = XOR_q coef[i][q] * symbol q of packet x-i+q, read from the reporting decoder's input.
// The k+n-1 input rows' addresses (cur before the decoder's role switch, old after; none outside
// the frames) are resolved once per packet into LDS, so each symbol is one dependent load.
__device__ __forceinline__ void vr_recover_body(const VrRecArgs& a, int bid, int nblk) {
    __shared__ uint8_t gexp[512];
    __shared__ uint8_t glog[256];
    __shared__ uint8_t lcf[4][kVrCoefStride];
    __shared__ const uint8_t* rowp[4][kMaxK + kMaxRuleN];
    __shared__ int32_t roww[4][kMaxK + kMaxRuleN];  // the row's width in the compact layout
    const int tid = threadIdx.x;
    for (int i = tid; i < 512; i += 256) gexp[i] = a.gf[i];
    for (int i = tid; i < 256; i += 256) glog[i] = a.gf[512 + i];
    __syncthreads();
    const int lane = tid & 63, wl = tid >> 6;
    const int L = a.L;
    uint8_t* lc = lcf[wl];
    const uint8_t** rp = rowp[wl];
    int32_t* rw = roww[wl];
    for (int r = bid * 4 + wl; r < a.nrec; r += nblk * 4) {
        const int64_t x = a.rec_x[r];
        const int j = a.rec_dec[r];
        const int k = a.inst[4 * j], n = a.inst[4 * j + 1];
        const int64_t sw = a.inst_switch[j];
        for (int i = lane; i < k * n; i += 64) {
            const uint8_t c = a.rec_coef[static_cast<int64_t>(r) * kVrCoefStride + i];
            lc[i] = c ? glog[c] : 255;
        }
        if (lane < k + n - 1) {  // row x-k+1+lane
            const int64_t row = x - k + 1 + lane;
            // a row spans [off[row], off[row+1]) (offsets [rows+1]); an empty old row has width 0,
            // and a symbol past a row's width reads 0 (as the zero-padded rows of the reference)
            const bool in = row >= 0 && row < a.rows;
            const int64_t* off = row < sw ? a.cur_off : a.old_off;
            rp[lane] = !in ? nullptr : (row < sw ? a.cur : a.old) + off[row];
            rw[lane] = !in ? 0 : static_cast<int32_t>(off[row + 1] - off[row]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // (the symbol loads of all five 64-byte steps of a packet issued together -- one round trip
        // instead of five -- measured slower beside the copy: 95 vs 61 us, 133 VGPRs,
        // profiles/r05/vr/r05za_*)
        int ln = 0;
        for (int h0 = 0; h0 < L + 2; h0 += 64) {
            const int h = h0 + lane;
            uint8_t acc = 0;
            if (h < L + 2) {
                const int s = h / k, i = h - s * k;
                const uint8_t* const* rpi = rp + (k - 1 - i);  // row of symbol q: x-i+q
                const int32_t* rwi = rw + (k - 1 - i);
                const uint8_t* lci = lc + i * n;
                // every symbol's load first (rows outside the frames read a harmless byte that is
                // then dropped), so the n loads of a lane are in flight together
                uint8_t sym[kMaxRuleN];
#pragma unroll
                for (int q = 0; q < kMaxRuleN; ++q) {
                    if (q < n) {
                        const uint8_t* row = rpi[q];
                        sym[q] = *(row && s * n + q < rwi[q] ? row + s * n + q : a.cur);
                    }
                }
#pragma unroll
                for (int q = 0; q < kMaxRuleN; ++q) {
                    if (q < n) {
                        const int lq = lci[q];
                        const uint8_t v = (lq == 255 || !rpi[q] || s * n + q >= rwi[q]) ? 0 : sym[q];
                        if (v) acc ^= gexp[lq + glog[v]];
                    }
                }
            }
            if (h0 == 0) {
                const int hi = __builtin_amdgcn_readlane(static_cast<int>(acc), 0);
                const int lo = __builtin_amdgcn_readlane(static_cast<int>(acc), 1);
                ln = min(hi * 256 + lo, L);
            }
            const int b = h - 2;
            if (b >= 0 && b < L) a.out[x * L + b] = b < ln ? acc : 0;
        }
        if (lane == 0) a.out_len[x] = ln;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

__global__ __launch_bounds__(256) void fec_vr_recover_kernel(VrRecArgs a) {
    vr_recover_body(a, static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x));
}

// The decode in one launch: workgroups [0, nrb) are the recovery's (fec_vr_recover_kernel's grid,
// dispatched first so that its latency-bound waves start beside the copy), the others one copy
// tile each (fec_vr_copy_fast_kernel).  The two write disjoint rows, so no order between them is
// needed; one launch instead of a fork to a side stream and a join back saves their event waits.
__global__ __launch_bounds__(256) void fec_vr_decode_kernel(VrCopyArgs a, VrRecArgs ra, int nrb) {
    if (static_cast<int>(blockIdx.x) < nrb) {
        vr_recover_body(ra, static_cast<int>(blockIdx.x), nrb);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* stage = smem;
    uint8_t* xo = smem + kVrFastStage;
    const int64_t tile = static_cast<int64_t>(blockIdx.x) - nrb;
    const VrTileDesc* dp = reinterpret_cast<const VrTileDesc*>(a.tdesc) + tile;
    VrTileDesc d;
    d.o0 = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->o0 & 0xffffffff)) & 0xffffffffu) |
           static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->o0 >> 32))) << 32;
    d.g1 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->g1)));
    d.g2 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->g2)));
    d.split = static_cast<uint16_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->split)));
    d.ok = static_cast<uint16_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->ok)));
    d.slow = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->slow)));
    d.recv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->recv)));
    d.rec = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(dp->rec)));
    vr_copy_fast_tile(a, tile, d, stage, xo);
}


}  // namespace

int vr_launch_frames(const VrFrameArgs& a, void* s) {
    if (a.rows <= 0) return FEC_OK;
    const int64_t blocks = std::min<int64_t>((a.rows + 3) / 4, 16384);
    hipLaunchKernelGGL(fec_vr_frame_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int vr_launch_parse(const VrParseArgs& a, void* s) {
    if (a.rows <= 0) return FEC_OK;
    const int64_t blocks = std::min<int64_t>((a.rows + 3) / 4, 16384);
    hipLaunchKernelGGL(fec_vr_parse_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int vr_launch_encode(const VrEncodeArgs& a, void* s) {
    if (a.nenc <= 0) return FEC_OK;
    const int wpb = std::min(4, 65536 / std::max(1, a.wave_bytes));
    if (wpb < 1) return FEC_ERR_ARG;
    // A wave walks its codewords one after another (a chain of dependent loads per codeword):
    // as many waves as the chip holds before the walks get longer than 2 codewords.
    const int64_t waves = std::max<int64_t>(1, std::min<int64_t>((a.cum_host_total + 1) / 2, 16384));
    const unsigned grid = static_cast<unsigned>((waves + wpb - 1) / wpb);
    hipLaunchKernelGGL(fec_vr_encode_kernel, dim3(grid), dim3(64 * wpb), static_cast<size_t>(wpb) * a.wave_bytes,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_encode_np0(const VrNp0Args& a, void* s) {
    if (a.nseg <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_encode_np0_kernel, dim3(static_cast<unsigned>(a.nseg)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
size_t vr_encode_cf_lds(const VrEncodeArgs& a) {
    return static_cast<size_t>(a.tab_bytes) + static_cast<size_t>(a.n_max) * ((a.L + 2 + kMaxK + 3) & ~3);
}
int vr_launch_encode_cf(const VrEncodeArgs& a, void* s) {
    if (a.nenc <= 0 || a.cum_host_total <= 0) return FEC_OK;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(a.cum_host_total, 16384));
    const size_t lds = vr_encode_cf_lds(a);
    if (lds > 65536) return vr_launch_encode(a, s);  // (the ring walk)
    hipLaunchKernelGGL(fec_vr_encode_cf_kernel, dim3(grid), dim3(256), lds, static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_geo(const VrCopyArgs& a, void* s) {
    if (a.P <= 0) return FEC_OK;
    hipLaunchKernelGGL(fec_vr_geo_kernel, dim3(static_cast<unsigned>((a.P + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_copy(const VrCopyArgs& a, void* s) {
    if (a.P <= 0) return FEC_OK;
    const int64_t grid = (a.P + kVrCopyTP - 1) / kVrCopyTP;
    const size_t otile = static_cast<size_t>(kVrCopyTP) * (a.L + kVrCopyOrs);
    const char* fv = std::getenv("FEC_VR_COPY_FAST");  // (an A/B switch, read per launch)
    const bool fast_on = !(fv && fv[0] == '0');
    const size_t ofast = std::max(static_cast<size_t>(kVrFastTP) * a.L, otile);
    if (fast_on && a.tdesc && (a.L & 3) == 0 && ofast <= 32768) {  // the specialised tiles (the generic ones inside)
        const int64_t g2 = (a.P + kVrFastTP - 1) / kVrFastTP;
        const size_t lds = kVrFastStage + ofast;
        hipLaunchKernelGGL(fec_vr_copy_fast_kernel, dim3(static_cast<unsigned>(g2)), dim3(256), lds,
                           static_cast<hipStream_t>(s), a);
        return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
    }
    if ((a.L & 3) == 0 && otile <= 32768)
        hipLaunchKernelGGL(fec_vr_copy_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), otile,
                           static_cast<hipStream_t>(s), a);
    else
        hipLaunchKernelGGL(fec_vr_copy_gather_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0,
                           static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_decode(const VrCopyArgs& a, const VrRecArgs& ra, void* s) {
    const size_t otile = static_cast<size_t>(kVrCopyTP) * (a.L + kVrCopyOrs);
    const size_t ofast = std::max(static_cast<size_t>(kVrFastTP) * a.L, otile);
    const char* fv = std::getenv("FEC_VR_COPY_FAST");
    if ((fv && fv[0] == '0') || !a.tdesc || (a.L & 3) != 0 || ofast > 32768 || a.P <= 0 || ra.nrec <= 0)
        return 1;  // not this form: vr_launch_copy + vr_launch_recover
    int nrb = 1024;  // the recovery's grid (as vr_launch_recover)
    if (const char* e = std::getenv("FEC_VR_REC_BLOCKS")) nrb = std::max(1, std::atoi(e));
    const int64_t g2 = (a.P + kVrFastTP - 1) / kVrFastTP;
    hipLaunchKernelGGL(fec_vr_decode_kernel, dim3(static_cast<unsigned>(nrb + g2)), dim3(256), kVrFastStage + ofast,
                       static_cast<hipStream_t>(s), a, ra, nrb);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_offsets(const VrOffsetsArgs& a, void* s) {
    hipLaunchKernelGGL(fec_vr_offsets_kernel, dim3(static_cast<unsigned>((std::max<int64_t>(1, a.rows) + 255) / 256)),
                       dim3(256), 0, static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}
int vr_launch_recover(const VrRecArgs& a, void* s) {
    if (a.nrec <= 0) return FEC_OK;
    // one wave per recovered packet, beside the copy (fewer workgroups, each wave walking several
    // packets, measured slower: 0.140 / 0.197 / 0.301 ms per decode at 256 / 128 / 64 against
    // 0.128 at 1024, profiles/r04/vr/r04u_rec_grid.txt)
    hipLaunchKernelGGL(fec_vr_recover_kernel, dim3(1024), dim3(256), 0,
                       static_cast<hipStream_t>(s), a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // namespace fec
