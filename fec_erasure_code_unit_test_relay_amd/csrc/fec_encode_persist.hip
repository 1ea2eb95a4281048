// fec_encode_persist.hip -- streaming encode kernel: persistent workgroups, specialised on k, n-k.
//
// Same closed form and the same dword/v_perm data path as fec_encode_fast_kernel
// (fec_encode_fast.hip); differs in how a workgroup walks the stream:
//   * each workgroup owns a contiguous range of tiles (TP packets) and walks it in order;
//   * the payload rows of tile j+1 are loaded into registers (16-byte loads) while tile j is
//     transposed, encoded and stored, and written to LDS when tile j is done -- the HBM latency
//     of the input is behind the previous tile's work;
//   * the position planes of the last n-1 rows of a tile are carried to the next tile (the
//     parity of packet t reads rows t-n+1 .. t-1): no halo row is loaded or transposed twice,
//     except the n-1 rows in front of the range, once;
//   * the parity step gives each lane two consecutive packets of one group of 4 sub-streams:
//     plane i supplies the words of rows [2p+i, 2p+i+NP] to both, so each word is read from LDS
//     and split into its three table selectors once for up to 2*(n-k) products.
// Per tile:  regs -> LDS rows | prefetch next | B: transpose rows into planes | C: parity and
// codeword interleave into the LDS output tile | D: 16-byte stores, trimmed sizes, halo carry.
#include "fec_device.h"
#include "fec_kernels.h"

namespace fec {
namespace {

constexpr int kPersistThreads = 320;
constexpr int kPrefetchMax = 6;  // 16-byte chunks per thread (host keeps TP*L/16 <= 6*threads)

// Transpose rows [0, nrows) of the row-major LDS payload tile into position planes at plane
// rows dst0 + r.  rowlen[r] < 0: the row does not exist (zero words).
template <int K>
__device__ __forceinline__ void transpose_rows(const uint32_t* raw32, const int32_t* rowlen, uint32_t* xin,
                                               int nrows, int dst0, int L, int NS4, int ROWS, int tid,
                                               int nth) {
    const int planes = NS4 * ROWS;
    for (int it = tid; it < nrows * NS4; it += nth) {
        const int g = it / nrows;
        const int r = it - g * nrows;
        const int ln = rowlen[r];
        uint32_t PW[K];
        if (ln < 0) {
#pragma unroll
            for (int i = 0; i < K; ++i) PW[i] = 0;
        } else {
            const int rowbase = r * L;
            const int b0 = 4 * g * K - 4;  // payload offset of dword D[0]
            uint32_t D[K + 1];
#pragma unroll
            for (int m = 0; m <= K; ++m) {
                const int b = b0 + 4 * m;
                D[m] = (b >= 0 && b < L) ? raw32[(rowbase + b) >> 2] : 0u;
            }
            uint32_t W[K];
#pragma unroll
            for (int m = 0; m < K; ++m) W[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], 2);
            if (g == 0) W[0] = (W[0] & 0xffff0000u) | ((ln & 0xff) << 8) | ((ln >> 8) & 0xff);
            if (b0 + 2 + 4 * K > ln) {  // bytes at payload offsets >= ln are zero
#pragma unroll
                for (int m = 0; m < K; ++m) W[m] &= keep_bytes(ln - (b0 + 2 + 4 * m));
            }
#pragma unroll
            for (int i = 0; i < K; ++i) PW[i] = gather4(W, i, K + i, 2 * K + i, 3 * K + i);
        }
#pragma unroll
        for (int i = 0; i < K; ++i) xin[i * planes + g * ROWS + dst0 + r] = PW[i];
    }
}

// native 16-byte vector (HIP's uint4 class keeps arrays of it in scratch memory)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte chunks q*nth + tid (q < kPrefetchMax, chunk < nch) of a tile into registers.
__device__ __forceinline__ void prefetch_tile(u32x4 (&pf)[kPrefetchMax], const uint8_t* tile, int nch,
                                              int tid, int nth) {
    const u32x4* g = reinterpret_cast<const u32x4*>(tile);
#pragma clang loop unroll(full)
    for (int q = 0; q < kPrefetchMax; ++q) {
        const int c = q * nth + tid;
        pf[q] = g[c < nch ? c : nch - 1];  // unconditional: keeps pf[] in registers
    }
}

// Selectors of v_perm_b32 for the three tables of gf_mul4x.
struct Sel3 {
    uint32_t s0, s1, s2;
};
__device__ __forceinline__ Sel3 split_sel(uint32_t x) {
    return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}
__device__ __forceinline__ uint32_t mul_sel(const uint4& t, uint32_t t4, const Sel3& s) {
    return __builtin_amdgcn_perm(t.y, t.x, s.s0) ^ __builtin_amdgcn_perm(t.w, t.z, s.s1) ^
           __builtin_amdgcn_perm(t4, t4, s.s2);
}

// Interleave the n words of one packet's group (k systematic, n-k parity) into the codeword
// layout [sub-stream][k | n-k] and write its vb valid bytes at xout + off.  A full group is
// written with straight-line code for its start alignment (head bytes, n-1 dwords, tail bytes);
// only the last group of a packet can be partial.
template <int K, int NP>
__device__ __forceinline__ void write_group(uint8_t* xout, const uint32_t (&src)[K + NP + 1], int off, int vb) {
    constexpr int n = K + NP;
    uint32_t O[n];
#pragma unroll
    for (int m = 0; m < n; ++m) {
        const int o0 = 4 * m, o1 = o0 + 1, o2 = o0 + 2, o3 = o0 + 3;
        O[m] = gather4(src, (o0 % n) * 4 + o0 / n, (o1 % n) * 4 + o1 / n, (o2 % n) * 4 + o2 / n,
                       (o3 % n) * 4 + o3 / n);
    }
    uint8_t* p = xout + off;
    const int h = off & 3;
    if (vb == 4 * n) {
        if (h == 0) {
#pragma unroll
            for (int m = 0; m < n; ++m) reinterpret_cast<uint32_t*>(p)[m] = O[m];
            return;
        }
        const int s = 4 - h;  // head bytes
        uint32_t* d = reinterpret_cast<uint32_t*>(p + s);
#pragma unroll
        for (int m = 0; m < n - 1; ++m) d[m] = __builtin_amdgcn_alignbyte(O[m + 1], O[m], s);
        uint8_t* tl = p + s + 4 * (n - 1);
        const uint32_t last = O[n - 1];
        if (h == 2) {
            *reinterpret_cast<uint16_t*>(p) = static_cast<uint16_t>(O[0]);
            *reinterpret_cast<uint16_t*>(tl) = static_cast<uint16_t>(last >> 16);
        } else if (h == 1) {
            p[0] = static_cast<uint8_t>(O[0]);
            *reinterpret_cast<uint16_t*>(p + 1) = static_cast<uint16_t>(O[0] >> 8);
            tl[0] = static_cast<uint8_t>(last >> 24);
        } else {
            p[0] = static_cast<uint8_t>(O[0]);
            tl[0] = static_cast<uint8_t>(last >> 8);
            *reinterpret_cast<uint16_t*>(tl + 1) = static_cast<uint16_t>(last >> 16);
        }
        return;
    }
#pragma unroll
    for (int b = 0; b < 4 * n; ++b)
        if (b < vb) p[b] = static_cast<uint8_t>(O[b >> 2] >> (8 * (b & 3)));
}

}  // namespace

template <int K, int NP>
__global__ __launch_bounds__(kPersistThreads) void fec_encode_persist_kernel(EncFastArgs a) {
    constexpr int n = K + NP;
    constexpr int H = n - 1;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // coefficient tables (8 dwords per (i, jj): gf_mul4x tables 0-4), read as wave-wide broadcasts
    __shared__ uint4 tabs[(K * NP > 0 ? K * NP : 1) * 2];
    uint8_t* raw = smem;  // payload rows of the tile, then its output tile
    uint8_t* xout = smem;
    uint32_t* raw32 = reinterpret_cast<uint32_t*>(smem);
    uint32_t* xin = reinterpret_cast<uint32_t*>(smem + a.raw_bytes);
    int32_t* rowlen = reinterpret_cast<int32_t*>(smem + a.raw_bytes + a.xin_bytes);
    uint32_t* par = reinterpret_cast<uint32_t*>(rowlen + a.TP);  // [NP][NS4][TP + 1] parity words

    const int tid = threadIdx.x, nth = blockDim.x;
    const int L = a.L, NS4 = a.NS4, ROWS = a.ROWS, CW = a.CW, TP = a.TP;
    const int planes = NS4 * ROWS;
    const int64_t ntiles = (a.P + TP - 1) / TP;
    const int64_t tb = static_cast<int64_t>(blockIdx.x) * a.tiles_per_wg;
    const int64_t te = min<int64_t>(ntiles, tb + a.tiles_per_wg);
    if (tb >= te) return;
    // diagnostics: cycles per phase summed over the workgroup's tiles (thread 0, s_memtime)
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tprev = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t tstart = tprev;
    auto mark = [&](int k) {
        if (a.stamps) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            ph[k] += now - tprev;
            tprev = now;
        }
    };
    for (int q = tid; q < K * NP * 2; q += nth) tabs[q] = reinterpret_cast<const uint4*>(a.ptab)[q];

    // ---- prologue: the n-1 rows in front of the range -> plane rows [0, H)
    {
        const int64_t t0 = tb * TP;
        const int L4 = L >> 2;
        for (int r = tid; r < H; r += nth) {
            const int64_t pk = t0 - H + r;
            int ln = -1;
            if (pk >= -a.history) {
                ln = a.len ? a.len[pk] : L;
                ln = ln < 0 ? 0 : (ln > L ? L : ln);
            }
            rowlen[r] = ln;
        }
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.payload);
        for (int idx = tid; idx < H * L4; idx += nth) {
            const int r = idx / L4;
            const int64_t pk = t0 - H + r;
            raw32[idx] = (pk >= -a.history) ? src[pk * L4 + (idx - r * L4)] : 0u;
        }
        __syncthreads();
        transpose_rows<K>(raw32, rowlen, xin, H, 0, L, NS4, ROWS, tid, nth);
    }
    mark(0);

    // prefetch registers (full tiles only, TP*L % 16 == 0): 16-byte chunk q*nth + tid of the tile
    const int64_t full_end = a.P / TP;  // tiles [0, full_end) are full
    const int nch = (TP * L) >> 4;
    u32x4 pf[kPrefetchMax];
    if (tb < full_end) prefetch_tile(pf, a.payload + tb * TP * L, nch, tid, nth);

    for (int64_t tile = tb; tile < te; ++tile) {
        const int64_t t0 = tile * TP;
        const int ntile = static_cast<int>(min<int64_t>(TP, a.P - t0));
        __syncthreads();  // the previous tile's output (aliasing raw) has left LDS; halo copied
        if (tile < full_end) {
            u32x4* raw4 = reinterpret_cast<u32x4*>(raw);
#pragma clang loop unroll(full)
            for (int q = 0; q < kPrefetchMax; ++q) {
                const int c = q * nth + tid;
                if (c < nch) raw4[c] = pf[q];
            }
        } else {  // the stream's last, partial tile: direct dword loads (L % 4 == 0)
            const uint32_t* g4 = reinterpret_cast<const uint32_t*>(a.payload + t0 * L);
            for (int o = tid; o < (ntile * L) >> 2; o += nth) raw32[o] = g4[o];
        }
        for (int r = tid; r < ntile; r += nth) {
            int ln = a.len ? a.len[t0 + r] : L;
            rowlen[r] = ln < 0 ? 0 : (ln > L ? L : ln);
        }
        if (tile + 1 < te && tile + 1 < full_end)
            prefetch_tile(pf, a.payload + (tile + 1) * TP * L, nch, tid, nth);
        __syncthreads();
        mark(1);

        // B. new rows -> plane rows [H, H + ntile)
        transpose_rows<K>(raw32, rowlen, xin, ntile, H, L, NS4, ROWS, tid, nth);
        __syncthreads();
        mark(2);

        // C1. parity words of two consecutive packets (2p, 2p+1) of group g per item.  Packet t
        // reads plane i at rows t + H - (K + jj - i) = t + i + NP - 1 - jj: for the pair, rows
        // 2p+i .. 2p+i+NP, each read and split into table selectors once.
        const int npair = (ntile + 1) >> 1;
        if (NP > 0) {
            for (int it = tid; it < NS4 * npair; it += nth) {
                const int g = it / npair;
                const int p = it - g * npair;
                const int r0 = 2 * p;
                const uint32_t* pg = xin + g * ROWS;
                uint32_t acc0[NP > 0 ? NP : 1], acc1[NP > 0 ? NP : 1];
#pragma unroll
                for (int jj = 0; jj < NP; ++jj) acc0[jj] = acc1[jj] = 0;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const uint32_t* pl = pg + i * planes;
                    // the tables are loop invariant: an opaque zero in their index keeps the
                    // reads here (hoisted, all (i, jj) tables would stay live in registers)
                    int z;
                    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
                    const uint4* tp = tabs + z + i * NP * 2;
                    Sel3 sl[NP + 1];
#pragma unroll
                    for (int m = 0; m <= NP; ++m) sl[m] = split_sel(pl[r0 + i + m]);
#pragma unroll
                    for (int jj = 0; jj < NP; ++jj) {
                        const uint4 t = tp[jj * 2];
                        const uint32_t t4 = tp[jj * 2 + 1].x;
                        acc0[jj] ^= mul_sel(t, t4, sl[NP - 1 - jj]);
                        acc1[jj] ^= mul_sel(t, t4, sl[NP - jj]);
                    }
                    __builtin_amdgcn_sched_barrier(0);  // one plane's words and tables at a time
                }
                uint32_t* pw = par + g * TP + r0;  // parity plane jj: par[(jj*NS4 + g)*TP + t]
#pragma unroll
                for (int jj = 0; jj < NP; ++jj) {
                    pw[jj * NS4 * TP] = acc0[jj];
                    pw[jj * NS4 * TP + 1] = acc1[jj];  // row TP of a tile with odd ntile: slack
                }
            }
            __syncthreads();
        }
        mark(3);

        // C2. codeword interleave of each (packet, group) into the LDS output tile
        for (int it = tid; it < NS4 * ntile; it += nth) {
            const int g = it / ntile;
            const int t = it - g * ntile;
            uint32_t src[n + 1];
#pragma unroll
            for (int i = 0; i < K; ++i) src[i] = xin[i * planes + g * ROWS + t + H];
#pragma unroll
            for (int jj = 0; jj < NP; ++jj) src[K + jj] = par[(jj * NS4 + g) * TP + t];
            src[n] = 0;
            write_group<K, NP>(xout, src, t * CW + 4 * n * g, min(4 * n, CW - 4 * n * g));
        }
        __syncthreads();
        mark(4);

        // D. tile out + trimmed wire sizes (FEC_Encoder.cpp:55-60); halo planes for the next tile
        const int bytes = ntile * CW;
        uint8_t* dstg = a.cw + t0 * CW;
        if ((bytes & 15) == 0 && (reinterpret_cast<uintptr_t>(dstg) & 15) == 0) {
            for (int o = tid * 16; o < bytes; o += nth * 16)
                *reinterpret_cast<uint4*>(dstg + o) = *reinterpret_cast<const uint4*>(xout + o);
        } else {
            for (int o = tid; o < bytes; o += nth) dstg[o] = xout[o];
        }
        for (int tl = tid; tl < ntile; tl += nth) {
            const uint8_t* row = xout + tl * CW;
            int z = CW - 1;
            while (z >= 0 && row[z] == 0) --z;
            a.cw_len[t0 + tl] = z + 1;
        }
        if (tile + 1 < te) {  // full tile: rows [TP, TP + H) -> [0, H)  (TP >= H)
            for (int idx = tid; idx < K * NS4 * H; idx += nth) {
                const int pl = idx / H;
                const int r = idx - pl * H;
                xin[pl * ROWS + r] = xin[pl * ROWS + TP + r];
            }
        }
        mark(5);
    }
    if (a.stamps && tid == 0) {
        uint64_t* st = a.stamps + static_cast<int64_t>(blockIdx.x) * 8;
        for (int k = 0; k < 6; ++k) st[k] = ph[k];
        st[6] = __builtin_amdgcn_s_memtime() - tstart;
        st[7] = static_cast<uint64_t>(te - tb);
    }
}

#define FEC_ENC_PERSIST_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(1, 10) X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)

#define FEC_ENC_PERSIST_INST(K, NP) \
    template __global__ void fec_encode_persist_kernel<K, NP>(EncFastArgs);
FEC_ENC_PERSIST_LIST(FEC_ENC_PERSIST_INST)

const void* fec_encode_persist_kernel_for(int k, int np) {
#define FEC_ENC_PERSIST_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_encode_persist_kernel<K, NP>);
    FEC_ENC_PERSIST_LIST(FEC_ENC_PERSIST_CASE)
#undef FEC_ENC_PERSIST_CASE
    return nullptr;
}

}  // namespace fec
