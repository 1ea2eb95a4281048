// fec_encode_fast.hip -- encode kernel specialised at compile time on k and n-k.
//
// Same closed form as fec_encode_kernel (fec_kernels.hip), organised so that every byte moves in
// dwords and every GF product is a packed 4-sub-stream operation:
//   A. the tile's payload rows (TP packets + an (n-1)-packet halo) are copied from HBM into LDS
//      with 16-byte loads, as one contiguous block (rows stay 300 bytes apart);
//   B. one lane per (row, group of 4 sub-streams): the 4k-byte window [len_hi, len_lo, payload]
//      of the group is read as k+1 dwords, shifted into place (v_alignbyte), masked past the
//      payload length, and transposed in registers into k "position words" (byte e of word i =
//      position i of sub-stream 4g+e) with constant-selector v_perm_b32; the words go to LDS
//      position planes [i][group][row] (conflict-free: lanes walk rows);
//   C. one lane per (packet, group): parity word j = XOR_i G[i][j] * plane_i[row - (j-i)] with
//      gf_mul4 (three v_perm_b32 table lookups per packed product); the n words of the group are
//      re-interleaved into the codeword layout [s][k systematic | n-k parity] with constant
//      selectors and written to the LDS output tile;
//   D. the tile leaves in 16-byte stores; trimmed wire sizes are taken from the tile.
#include "fec_device.h"
#include "fec_kernels.h"

namespace fec {


template <int K, int NP>
__global__ __launch_bounds__(256) void fec_encode_fast_kernel(EncFastArgs a) {
    constexpr int n = K + NP;
    constexpr int H = n - 1;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* raw = smem;   // phases A-B: payload rows; phases C-D: the output tile
    uint8_t* xout = smem;
    uint32_t* raw32 = reinterpret_cast<uint32_t*>(smem);
    uint32_t* xin = reinterpret_cast<uint32_t*>(smem + a.raw_bytes);
    int32_t* rowlen = reinterpret_cast<int32_t*>(smem + a.raw_bytes + a.xin_bytes);

    const int tid = threadIdx.x;
    phase_stamp(a.stamps, blockIdx.x, 0);
    const int L = a.L, NS4 = a.NS4, ROWS = a.ROWS, CW = a.CW;
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * a.TP;
    const int ntile = static_cast<int>(min<int64_t>(a.TP, a.P - t0));
    const int rows = ntile + H;
    const int64_t pa = max<int64_t>(t0 - H, -a.history);  // first packet that exists
    const int r_lo = static_cast<int>(pa - (t0 - H));
    const int64_t pb = t0 + ntile;

    for (int r = tid; r < rows; r += 256) {
        const int64_t pk = t0 - H + r;
        int ln = -1;
        if (pk >= pa) {
            ln = a.len ? a.len[pk] : L;
            ln = ln < 0 ? 0 : (ln > L ? L : ln);
        }
        rowlen[r] = ln;
    }

    // A. contiguous payload rows [pa, pb) -> raw[delta + (pk-pa)*L + b]
    const uint8_t* gA = a.payload + pa * L;
    const int delta = static_cast<int>(reinterpret_cast<uintptr_t>(gA) & 15);
    const uint8_t* gbase = gA - delta;
    const int total = delta + static_cast<int>(pb - pa) * L;
    stage_to_lds<8>(raw, gbase, delta, total, tid, 256);
    __syncthreads();
    phase_stamp(a.stamps, blockIdx.x, 1);

    // B. transpose windows into position planes xin[(i*NS4 + g)*ROWS + r]
    const int planes = NS4 * ROWS;
    for (int it = tid; it < rows * NS4; it += 256) {
        const int g = it / rows;
        const int r = it - g * rows;
        const int ln = rowlen[r];
        uint32_t PW[K];
        if (ln < 0) {
#pragma unroll
            for (int i = 0; i < K; ++i) PW[i] = 0;
        } else {
            const int rowbase = delta + (r - r_lo) * L;
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
            // window byte e*K + i  ->  position word i, byte e
#pragma unroll
            for (int i = 0; i < K; ++i) PW[i] = gather4(W, i, K + i, 2 * K + i, 3 * K + i);
        }
#pragma unroll
        for (int i = 0; i < K; ++i) xin[i * planes + g * ROWS + r] = PW[i];
    }
    __syncthreads();
    phase_stamp(a.stamps, blockIdx.x, 2);

    // C. parity + interleave into the codeword layout.  Each thread holds up to IPT items so that
    // every coefficient table is fetched once and applied to all of them (the tables are
    // wave-uniform scalar loads), and their LDS reads are in flight together.
    constexpr int IPT = 3;
    const int nitems = ntile * NS4;
    for (int base = 0; base < nitems; base += 256 * IPT) {
        int rowoff[IPT];  // dword index of the item's row in plane 0
        bool valid[IPT];
#pragma unroll
        for (int q = 0; q < IPT; ++q) {
            const int it = base + q * 256 + tid;
            valid[q] = it < nitems;
            const int itc = valid[q] ? it : 0;
            const int g = itc / ntile;
            const int t = itc - g * ntile;
            rowoff[q] = g * ROWS + t + H;
        }
        uint32_t acc[IPT][NP > 0 ? NP : 1];
#pragma unroll
        for (int q = 0; q < IPT; ++q)
#pragma unroll
            for (int jj = 0; jj < NP; ++jj) acc[q][jj] = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const uint32_t* pl = xin + i * planes;
#pragma unroll
            for (int jj = 0; jj < NP; ++jj) {
                const uint32_t* tab = a.ptab + (i * NP + jj) * 8;  // zero coefficient: zero tables
                const int d = K + jj - i;
#pragma unroll
                for (int q = 0; q < IPT; ++q) acc[q][jj] ^= gf_mul4x(tab, pl[rowoff[q] - d]);
            }
        }
#pragma unroll
        for (int q = 0; q < IPT; ++q) {
            if (!valid[q]) continue;
            const int it = base + q * 256 + tid;
            const int g = it / ntile;
            const int t = it - g * ntile;
            uint32_t src[n + 1];  // words 0..k-1: systematic positions, k..n-1: parity
#pragma unroll
            for (int i = 0; i < K; ++i) src[i] = xin[i * planes + rowoff[q]];
#pragma unroll
            for (int jj = 0; jj < NP; ++jj) src[K + jj] = acc[q][jj];
            src[n] = 0;
            // output byte o = e*n + j (e = sub-stream in the group) = word j, byte e
            uint32_t O[n + 1];
#pragma unroll
            for (int m = 0; m < n; ++m) {
                const int o0 = 4 * m, o1 = o0 + 1, o2 = o0 + 2, o3 = o0 + 3;
                O[m] = gather4(src, (o0 % n) * 4 + o0 / n, (o1 % n) * 4 + o1 / n,
                               (o2 % n) * 4 + o2 / n, (o3 % n) * 4 + o3 / n);
            }
            O[n] = 0;
            // write bytes [off, off + valid) of the tile; off may be unaligned (CW odd/even)
            const int off = t * CW + 4 * n * g;
            const int vb = min(4 * n, CW - 4 * n * g);
            const int head = (4 - (off & 3)) & 3;
            const int hv = min(head, vb);
            for (int e = 0; e < hv; ++e) xout[off + e] = static_cast<uint8_t>(O[0] >> (8 * e));
            const int body = vb - hv;
            const int nfull = body >> 2;
            uint32_t* dst = reinterpret_cast<uint32_t*>(xout + off + hv);
            uint32_t tailw = 0;
#pragma unroll
            for (int m = 0; m < n; ++m) {
                const uint32_t w = __builtin_amdgcn_alignbyte(O[m + 1], O[m], head);
                if (m < nfull) dst[m] = w;
                if (m == nfull) tailw = w;
            }
            const int tail = body & 3;
            uint8_t* tb = xout + off + hv + 4 * nfull;
            for (int e = 0; e < tail; ++e) tb[e] = static_cast<uint8_t>(tailw >> (8 * e));
        }
    }
    __syncthreads();
    phase_stamp(a.stamps, blockIdx.x, 3);

    // D. tile out + trimmed wire sizes (FEC_Encoder.cpp:55-60)
    const int bytes = ntile * CW;
    uint8_t* dstg = a.cw + t0 * CW;
    if ((bytes & 15) == 0 && (reinterpret_cast<uintptr_t>(dstg) & 15) == 0) {
        for (int o = tid * 16; o < bytes; o += 256 * 16)
            *reinterpret_cast<uint4*>(dstg + o) = *reinterpret_cast<const uint4*>(xout + o);
    } else {
        for (int o = tid; o < bytes; o += 256) dstg[o] = xout[o];
    }
    for (int tl = tid; tl < ntile; tl += 256) {
        const uint8_t* row = xout + tl * CW;
        int z = CW - 1;
        while (z >= 0 && row[z] == 0) --z;
        a.cw_len[t0 + tl] = z + 1;
    }
    phase_stamp(a.stamps, blockIdx.x, 4);
}

// Instantiated (k, n-k): the adaptive estimator's (10,b,b) family (k = 11-b, n = 11), the BASELINE
// fixed configurations and the published fixed-rate logs' configurations.
#define FEC_ENC_FAST_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(1, 10) X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)

#define FEC_ENC_FAST_INST(K, NP) template __global__ void fec_encode_fast_kernel<K, NP>(EncFastArgs);
FEC_ENC_FAST_LIST(FEC_ENC_FAST_INST)

const void* fec_encode_fast_kernel_for(int k, int np) {
#define FEC_ENC_FAST_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_encode_fast_kernel<K, NP>);
    FEC_ENC_FAST_LIST(FEC_ENC_FAST_CASE)
#undef FEC_ENC_FAST_CASE
    return nullptr;
}

}  // namespace fec
