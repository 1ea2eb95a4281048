// fec_encode_tile.hip -- encode kernel over contiguous packet chunks, staged through LDS tiles.
//
// Same closed form as every encode kernel here (fec_kernels.hip): for packet t, sub-stream s,
//     cw_t[s*n + j] = X_t[s][j]                                   j <  k
//     cw_t[s*n + j] = XOR_i G[i][j] * X_{t-(j-i)}[s][i]           j >= k
// with X_t[s] = bytes [s*k, s*k+k) of [len_hi, len_lo, payload, zero pad] (Encoder.cpp:65-98,
// Encoder_Basic.cpp:48-74, codingOperations.cpp:131-147).
//
// Organisation: a workgroup (4 waves) owns a contiguous run of tiles of R = 4*PPW packets and walks
// it; only the tile in front of its first one is read twice (the n-1 packets of parity history), so
// HBM reads are L bytes per packet plus ~1/tiles_per_wg.  Per tile:
//   * the tile's payload rows (one contiguous R*L-byte slab) arrive in LDS by LDS-DMA
//     (buffer_load ... lds), issued two tiles ahead: no registers hold loads in flight, and rows
//     outside [-history, P) come back as zero (buffer range check) -- the X_{t'<t0} = 0 semantics;
//   * A: item (p, g) = packet p of the tile, group g of 4 sub-streams; its thread builds the K
//     window words H (header, zero pad) and the K position words (byte e of word i = position i of
//     sub-stream 4g+e) and writes the position words to LDS;
//   * B: parity forward: position word i of packet p contributes G[i][K+jj] * word to parity jj of
//     packet p + (K+jj-i).  The K*NP (i, jj) products are split over the 4 waves at compile time, so
//     a wave's coefficient tables stay in its registers for the whole kernel; each wave sweeps every
//     item of the tile and XORs its products into the tile's parity rows in LDS (ds_xor, rows
//     [0, R+n-1); the rows past R are the next tile's first n-1 packets);
//   * C: item (p, g) reads its finished parity, interleaves the n codeword words of its 4
//     sub-streams, shifts them to the packet's byte alignment (the bytes in front come from the lane
//     to its left: every wave holds whole packets) and writes them into the LDS output tile; the
//     parity rows move down by R;
//   * D: the output tile (R*CW bytes, a multiple of 16 at a 16-byte aligned offset) goes to HBM in
//     16-byte stores, 1 KB contiguous per wave instruction; one lane per packet computes the
//     trimmed wire size (FEC_Encoder.cpp:55-60) from the LDS tile.
// Four workgroup barriers per tile (tile in LDS; position words written, when the DMA two tiles
// ahead is issued into the freed input buffer; parity complete; output tile complete); several
// workgroups per CU overlap one another's phases.
#include "fec_device.h"
#include "fec_kernels.h"
#include "fec_vr_cf.h"

#include <cstdlib>
#include <utility>

namespace fec {
namespace {

constexpr int kTileThreads = 256;
#ifndef FEC_TILE_MINWG
#define FEC_TILE_MINWG 5  // workgroups per CU the register budget is sized for
#endif

template <typename F, int... Is>
__device__ __forceinline__ void tfor_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void tfor(F&& f) {
    tfor_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ uint32_t txor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct TSel {
    uint32_t s0, s1, s2;
};
__device__ __forceinline__ TSel tsplit(uint32_t x) {
    return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}
struct TTab {
    uint32_t x, y, z, w, t4;  // c*{0..7} (x: 0..3, y: 4..7), c*({0..7}<<3) (z, w), c*({0..3}<<6)
};
__device__ __forceinline__ uint32_t tprod(const TTab& t, const TSel& s) {
    return txor3(__builtin_amdgcn_perm(t.y, t.x, s.s0), __builtin_amdgcn_perm(t.w, t.z, s.s1),
                 __builtin_amdgcn_perm(t.t4, t.t4, s.s2));
}

__device__ __forceinline__ uint32_t tbperm(int src_lane, uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src_lane << 2, static_cast<int>(v)));
}

// s_waitcnt vmcnt(n) (expcnt, lgkmcnt: no wait); n is a run-time value, the immediate is not
__device__ __forceinline__ void wait_vm(int n) {
#define FEC_VM_CASE(N) \
    case N: __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14)); break;
    switch (n < 0 ? 0 : n) {
        FEC_VM_CASE(0) FEC_VM_CASE(1) FEC_VM_CASE(2) FEC_VM_CASE(3) FEC_VM_CASE(4) FEC_VM_CASE(5)
        FEC_VM_CASE(6) FEC_VM_CASE(7) FEC_VM_CASE(8) FEC_VM_CASE(9) FEC_VM_CASE(10) FEC_VM_CASE(11)
        FEC_VM_CASE(12) FEC_VM_CASE(13) FEC_VM_CASE(14) FEC_VM_CASE(15) FEC_VM_CASE(16) FEC_VM_CASE(17)
        FEC_VM_CASE(18) FEC_VM_CASE(19) FEC_VM_CASE(20) FEC_VM_CASE(21) FEC_VM_CASE(22) FEC_VM_CASE(23)
        default: FEC_VM_CASE(24)
    }
#undef FEC_VM_CASE
}

__device__ __forceinline__ void wait_lds_barrier() {
    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0) only
    __builtin_amdgcn_s_barrier();
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef uint32_t tv4u __attribute__((ext_vector_type(4)));

// Buffer descriptor as four SGPRs (raw buffer, stride 0, num_records bytes; gfx950 dword 3 flags).
__device__ __forceinline__ tv4u raw_rsrc(const void* base, int num_records) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    return tv4u{static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(b & 0xffffffffu))),
                static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>((b >> 32) & 0xffffu))),
                static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(num_records)), 0x00020000u};
}

// LDS-DMA (buffer_load ... lds): lane i's SIZE bytes at byte voff of the buffer land at LDS byte
// lds + SIZE*i.  Issued from asm so that hipcc does not treat every later LDS access as possibly
// reading the DMA's destination (it would wait vmcnt(0) in front of each, draining the prefetch);
// completion is counted here with wait_vm.  M0 is written and restored inside the statement.
__device__ __forceinline__ void dma16(tv4u rsrc, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma16_nt(tv4u rsrc, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(tv4u rsrc, uint32_t voff, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_ptr)(p)));
}

// The dword whose byte q is byte I_q of the concatenated words src[] (compile-time indices): a
// plain copy when the four bytes are one word in place, one v_perm_b32 when they come from at most
// two words, else two v_perm_b32 and an OR.
template <int NW, int I0, int I1, int I2, int I3>
__device__ __forceinline__ uint32_t tgather4(const uint32_t (&src)[NW]) {
    constexpr int w0 = I0 >> 2, w1 = I1 >> 2, w2 = I2 >> 2, w3 = I3 >> 2;
    if constexpr (w0 == w1 && w1 == w2 && w2 == w3 && (I0 & 3) == 0 && (I1 & 3) == 1 && (I2 & 3) == 2 &&
                  (I3 & 3) == 3) {
        return src[w0];
    } else {
        constexpr int a = w0;  // first source word; the other one, if any
        constexpr int b = (w1 != a) ? w1 : (w2 != a) ? w2 : w3;
        if constexpr ((w1 == a || w1 == b) && (w2 == a || w2 == b) && (w3 == a || w3 == b)) {
            constexpr auto code = [](int w, int i) constexpr { return w == a ? (i & 3) : 4 + (i & 3); };
            constexpr uint32_t sel = sel4(code(w0, I0), code(w1, I1), code(w2, I2), code(w3, I3));
            return __builtin_amdgcn_perm(src[b], src[a], sel);
        } else {
            return gather4(src, I0, I1, I2, I3);
        }
    }
}

// Codeword words of the group: bytes [e*n, e*n+n) = sub-stream 4g+e: K systematic bytes, NP parity.
template <int K, int NP>
__device__ __forceinline__ void tgroup_words(const uint32_t (&H)[K], const uint32_t (&Q)[NP > 0 ? NP : 1],
                                             uint32_t (&X)[K + NP]) {
    constexpr int n = K + NP;
    uint32_t src[n];
#pragma unroll
    for (int m = 0; m < K; ++m) src[m] = H[m];
#pragma unroll
    for (int jj = 0; jj < NP; ++jj) src[K + jj] = Q[jj];
    constexpr auto idx = [](int b) constexpr {
        const int e = b / n, j = b % n;
        return j < K ? (e * K + j) : (4 * (K + j - K) + e);
    };
    tfor<n>([&](auto qc) __attribute__((always_inline)) {
        constexpr int qq = decltype(qc)::value;
        X[qq] = tgather4<n, idx(4 * qq), idx(4 * qq + 1), idx(4 * qq + 2), idx(4 * qq + 3)>(src);
    });
}

// Last 4 valid bytes of the group's words (bytes [vb-4, vb)), vb = n * REM for the last group.
template <int n, int REM>
__device__ __forceinline__ uint32_t ttail_rem(const uint32_t (&X)[n]) {
    constexpr int b = n * REM - 4;
    if constexpr (b < 0) {
        return X[0] << (8 * (4 - n * REM));
    } else if constexpr (b % 4 == 0) {
        return X[b / 4];
    } else {
        return __builtin_amdgcn_alignbyte(X[b / 4 + 1], X[b / 4], b % 4);
    }
}

// LC > 0: L (and every size derived from it) fixed at compile time; LC = 0: from the arguments.
// SEG: segment mode (the variable-rate schedule's instances, a.seg) compiled in; the one-stream
// kernels are built without it (its branches cost the headline encoder 10 %: 158 vs 144 us).
template <int K, int NP, int W, int LC, bool SEG>
__device__ __forceinline__ void tile_walk(const EncTileArgs& a, uint8_t* smem) {
    constexpr int n = K + NP;
    constexpr TileGeom CG = tile_geometry(K, NP, LC > 0 ? LC : 300, SEG);
    constexpr bool CL = LC > 0;
    static_assert(!CL || CG.ok, "no tile geometry for this (k, n-k, L)");
    constexpr int NPA = NP > 0 ? NP : 1;
    constexpr int KNP = K * NP;
    constexpr int k0 = W * KNP / 4, k1 = (W + 1) * KNP / 4;  // this wave's (i, jj) products
    constexpr int NPW = k1 - k0;
    constexpr int NPWA = NPW > 0 ? NPW : 1;
    constexpr int i_lo = NPW > 0 ? k0 / NPA : 0;
    constexpr int i_hi = NPW > 0 ? (k1 - 1) / NPA : -1;
    constexpr int PWS = K | 1;  // position words per item in LDS (odd: conflict-free item strides)

    const int lane = threadIdx.x & 63;
    const int tid = threadIdx.x;
    const int L = CL ? LC : a.L, CW = CL ? CG.CW : a.CW, NS4 = CL ? CG.NS4 : a.NS4;
    const int PPW = CL ? CG.PPW : a.PPW, R = 4 * PPW;
    // Segment mode (a.seg, the variable-rate schedule): this workgroup encodes tiles [t0, t0+cnt)
    // of one encoder instance -- a fresh encoder over the payload rows [sfirst, sfirst+P) -- and
    // writes row t to the frames' array of its role (cur before the role switch, old after) in the
    // compact layout (fec_vr.h): the instance's cur rows from byte scur, its old rows from sold,
    // stride a.W (its CW rounded to 16).
    constexpr bool segm = SEG;
    int P = a.P;
    int64_t sfirst = 0, ssw = 0, scur = 0, sold = 0;
    int seg_t0 = 0, seg_cnt = 0;
    if (segm) {
        const int64_t* sg = a.seg + 6 * blockIdx.x;
        sfirst = sg[0];
        ssw = sg[1];
        P = static_cast<int>(sg[2]);
        seg_t0 = static_cast<int>(sg[3] & 0xffffffff);
        seg_cnt = static_cast<int>(sg[3] >> 32);
        scur = sg[4];
        sold = sg[5];
    }
    const uint8_t* pay_base = segm ? a.payload_base + sfirst * (CL ? LC : a.L) : a.payload_base;
    const int pay_bytes = segm ? P * (CL ? LC : a.L) : a.payload_bytes;
    const int32_t* len_base = segm ? (a.len_base ? a.len_base + sfirst : nullptr) : a.len_base;
    const int len_bytes = segm ? 4 * P : a.len_bytes;
    const int dbg = CL ? 0 : a.dbg;  // timing experiments: the runtime-L kernel only
    const int nvl = CL ? CG.nvl : a.nvl, rem = CL ? CG.rem : a.rem;
    const int off_in = CL ? CG.off_in : a.off_in, in_bytes = CL ? CG.in_bytes : a.in_bytes;
    const int off_pw = CL ? CG.off_pw : a.off_pw, off_q = CL ? CG.off_q : a.off_q;
    const int off_out = CL ? CG.off_out : a.off_out, off_len = CL ? CG.off_len : a.off_len;
    const int off_scratch = CL ? CG.off_scratch : a.off_scratch;
    const int last_g = NS4 - 1;
    const int ipw = PPW * NS4;                 // items per wave slice
    const bool active = lane < ipw;
    const int pl = active ? lane / NS4 : 0;    // packet of the lane inside its wave slice
    const int g = active ? lane - pl * NS4 : 0;
    const int p = W * PPW + pl;                // own packet in the tile
    const int item = p * NS4 + g;
    const bool is_last = g == last_g;
    const int ROWS = R + n - 1;
    const int QJ = ROWS * NS4;                 // dwords per parity plane

    // LDS carve-up (byte offsets from the launcher)
    uint32_t* pw = reinterpret_cast<uint32_t*>(smem + off_pw);
    uint32_t* q = reinterpret_cast<uint32_t*>(smem + off_q);
    uint8_t* out = smem + off_out;
    uint32_t* scratch = reinterpret_cast<uint32_t*>(smem + off_scratch);  // one dword per thread
    const uint32_t* lensl = reinterpret_cast<const uint32_t*>(smem + off_len);

    // coefficient tables of this wave's products, in registers for the whole walk
    TTab tab[NPWA];
    tfor<NPW>([&](auto kc) __attribute__((always_inline)) {
        constexpr int kk = k0 + decltype(kc)::value;
        constexpr int I = kk / NPA, JJ = kk % NPA;
        const uint32_t* t = a.ptab + (I * NP + JJ) * 8;
        TTab& d = tab[decltype(kc)::value];
        d = {t[0], t[1], t[2], t[3], t[4]};
        // in VGPRs: scalar copies of 5 dwords per product would crowd out the SGPRs
        asm volatile("" : "+v"(d.x), "+v"(d.y), "+v"(d.z), "+v"(d.w), "+v"(d.t4));
    });

    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(pay_base), 0, pay_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(a.cw, 0, a.cw_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(a.cw_len, 0, 4 * P, 0x00020000);
    const bool has_len = len_base != nullptr;

    const int first = segm ? seg_t0 : static_cast<int>(blockIdx.x) * a.tiles_per_wg;
    const int cnt = segm ? seg_cnt : min(a.tiles_per_wg, a.ntiles - first);  // real tiles of this workgroup (>= 1)
    const int ngl = CL ? CG.ngl : a.ngl;                     // payload LDS-DMA instructions per wave per tile
    const int nso = CL ? CG.nso : a.nso;                     // 16-byte stores per thread per tile
    // segment mode's row-chunk iterations (two stores each: the cur and old resources)
    const int nch_seg = (CW + 15) >> 4;
    const int nit_seg = (R * nch_seg + kTileThreads - 1) / kTileThreads;
    // VMEM bookkeeping instead of hand-counted waits: vm_issued counts the VMEM instructions this
    // wave has issued (the same in every wave: each counted instruction sits in uniform control
    // flow and is issued even when no lane's offset is in range), incremented right where they are
    // issued; vm_mark[it & 1] is vm_issued just after tile it's LDS-DMA.  Waiting for that DMA is
    // wait_vm(vm_issued - vm_mark[it & 1]): every instruction issued after it may stay in flight.
    // Instructions left uncounted (the tail tile's extra dword/byte stores) only make a wait
    // stricter, never weaker; moving a DMA or a store moves its count with it.
    uint32_t vm_issued = 0;
    uint32_t vm_mark[2] = {0u, 0u};

    // tile it (0 = the tile in front of the first one) -> LDS input buffer (it & 1)
    const tv4u rs4 = raw_rsrc(pay_base, pay_bytes);
    const tv4u rl4 = raw_rsrc(len_base, len_bytes);
    const uint32_t lds_in = lds_addr(smem + off_in), lds_len = lds_addr(smem + off_len);
    // LDS image of a tile: row p at p*RS (RS = L rounded up to 16 bytes), so that every row starts
    // 16-byte aligned; the DMA's destination is lane-linear, its per-lane source picks the row
    // piece (tile-invariant offsets, computed once).  A row's last piece also brings the first
    // bytes of the next row (never read as payload: past L they are the zero pad's business).
    const int CPR = (L + 15) >> 4;  // 16-byte pieces per row
    const int RS = CPR * 16;
    int srel[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = (j * 4 + (tid >> 6)) * 64 + lane;
        const int row = c / CPR;
        srel[j] = row * L + (c - row * CPR) * 16;
    }
    auto issue = [&](int it) __attribute__((always_inline)) {
        const int row0 = (first - 1 + it) * R;
        const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
        const uint32_t dst = lds_in + (it & 1) * in_bytes;
        const int base = (row0 + a.history) * L;  // may be negative: those pieces read as zero
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j < ngl) {
                const int o = base + srel[j];
                if (a.nt & 2)
                    dma16_nt(rs4, static_cast<uint32_t>(o < 0 ? 0x7fffffff : o), dst + (j * 4 + wv) * 1024);
                else
                    dma16(rs4, static_cast<uint32_t>(o < 0 ? 0x7fffffff : o), dst + (j * 4 + wv) * 1024);
                ++vm_issued;
            }
        }
        if (has_len) {
            const int r = row0 + a.history + lane;
            const bool ok = wv == 0 && lane < R && r >= 0;
            dma4(rl4, static_cast<uint32_t>(ok ? r * 4 : 0x7fffffff), lds_len + (it & 1) * 1024 + wv * 256);
            ++vm_issued;
        }
        vm_mark[it & 1] = vm_issued;
    };

    // parity rows start zeroed
    for (int x = tid; x < NPA * QJ; x += kTileThreads) q[x] = 0;

    // tile 0 (in front of the first one) only feeds parity history: none to feed without parity,
    // nor in front of an instance's first tile (its rows read as zero: the parity rows' zeros)
    // (a.nt bit 2, FEC_VR_HIST0=1: computed anyway, as before)
    const int it0 = (NP == 0 || (SEG && seg_t0 == 0 && !(a.nt & 4))) ? 1 : 0;
    issue(it0);
    if (cnt >= it0 + 1) issue(it0 + 1);

    uint32_t H[K];
    for (int it = it0; it <= cnt; ++it) {
        // tile it's input: every VMEM instruction issued after it may still be in flight
        wait_vm(static_cast<int>(vm_issued - vm_mark[it & 1]));
        wait_lds_barrier();  // B1: the tile is in LDS everywhere; last tile's output stored
        const int row0 = (first - 1 + it) * R;
        const uint8_t* in = smem + off_in + (it & 1) * in_bytes;
        if (L & 15) {
            // the batch's last row: its last piece runs past the end of the payload rows, and an
            // LDS-DMA out of range as a whole reads zeros: its valid dwords again, one by one
            const int pl_last = P - 1 - row0;
            if (pl_last >= 0 && pl_last < R) {
                if (tid < 4) {
                    const int b = (CPR - 1) * 16 + 4 * tid;
                    if (b < L)
                        reinterpret_cast<uint32_t*>(smem + off_in + (it & 1) * in_bytes)[(pl_last * RS + b) >> 2] =
                            __builtin_amdgcn_raw_buffer_load_b32(rs, (P - 1 + a.history) * L + b, 0, 0);
                }
                wait_vm(0);  // (wave 0's loads only: not counted, drained here)
                wait_lds_barrier();
            }
        }

        // ---- A: window words and position words of the own item
        if (active) {
            const int t = row0 + p;
            int lv = L;
            if (has_len) {
                lv = static_cast<int>(lensl[(it & 1) * 256 + p]);
                lv = lv < 0 ? 0 : (lv > L ? L : lv);
            }
            const int ln = (t < -a.history || t >= P) ? 0 : lv;
            const int rb = p * RS + 4 * K * g;  // byte of row dword K*g
            uint32_t D[K + 1];
            D[0] = *reinterpret_cast<const uint32_t*>(in + rb - 4);
            if constexpr (K == 8) {
                // 16-byte reads from asm: left to the compiler, the L = 300 instance's loads are
                // re-paired with D[0] into ds_read2_b32 (32-bank groups: 4-way conflicts here,
                // SQ_LDS_BANK_CONFLICT 19.3 M per launch vs 8.3 M with ds_read_b128)
                tv4u v0, v1;
                asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                             : "=&v"(v0), "=&v"(v1)
                             : "v"(lds_addr(in + rb))
                             : "memory");
                D[1] = v0.x;
                D[2] = v0.y;
                D[3] = v0.z;
                D[4] = v0.w;
                D[5] = v1.x;
                D[6] = v1.y;
                D[7] = v1.z;
                D[8] = v1.w;
            } else if constexpr (K % 4 == 0) {
#pragma unroll
                for (int m = 0; m < K; m += 4) {
                    const uint4 v = *reinterpret_cast<const uint4*>(in + rb + 4 * m);
                    D[m + 1] = v.x;
                    D[m + 2] = v.y;
                    D[m + 3] = v.z;
                    D[m + 4] = v.w;
                }
            } else {
#pragma unroll
                for (int m = 0; m < K; ++m) D[m + 1] = *reinterpret_cast<const uint32_t*>(in + rb + 4 * m);
            }
            const uint32_t hdr =
                (static_cast<uint32_t>(ln & 0xff) << 24) | (static_cast<uint32_t>((ln >> 8) & 0xff) << 16);
            D[0] = g == 0 ? hdr : D[0];
#pragma unroll
            for (int m = 0; m < K; ++m)  // the last group's dwords past the row end: zero pad
                if (m >= nvl) D[m + 1] = is_last ? 0u : D[m + 1];
#pragma unroll
            for (int m = 0; m < K; ++m) H[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], 2);
            if (ln != L) {
                const int lim = ln > 0 ? ln + 2 - 4 * K * g : 0;  // empty / missing packet: no header
#pragma unroll
                for (int m = 0; m < K; ++m) H[m] &= keep_bytes(lim - 4 * m);
            }
            tfor<K>([&](auto ic) __attribute__((always_inline)) {
                constexpr int i = decltype(ic)::value;
                pw[item * PWS + i] = tgather4<K, i, K + i, 2 * K + i, 3 * K + i>(H);
            });
        }
        wait_lds_barrier();  // position words of the whole tile written; the input buffer is free
        // the DMA two tiles ahead starts here, before phase B (no VMEM instruction between here and
        // phase D, so the hand-counted waits are unchanged): step 0.3161 vs 0.3170 ms with it after
        // B2, encoder alone 166.4 vs 167.4 us (same process, profiles/r03/r03v_tile_early_issue_ab.txt)
        if (it + 2 <= cnt) issue(it + 2);

        // ---- B: this wave's products over every item of the tile, XORed into the parity rows
        if constexpr (NPW > 0) {
            if (active && !(dbg & 1)) {
#ifdef FEC_TILE_BUNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
                for (int sl = 0; sl < 4; ++sl) {
                    const int it_item = (sl * PPW + pl) * NS4 + g;
                    const int pp = sl * PPW + pl;
                    const uint32_t* src = pw + it_item * PWS;
                    uint32_t* qb = q + pp * NS4 + g;
                    tfor<i_hi - i_lo + 1>([&](auto ic) __attribute__((always_inline)) {
                        constexpr int I = i_lo + decltype(ic)::value;
                        const TSel s = tsplit(src[I]);
                        tfor<NPA>([&](auto jc) __attribute__((always_inline)) {
                            constexpr int JJ = decltype(jc)::value;
                            constexpr int kk = I * NPA + JJ;
                            if constexpr (kk >= k0 && kk < k1) {
                                const uint32_t v = tprod(tab[kk - k0], s);
                                __hip_atomic_fetch_xor(qb + JJ * QJ + (K + JJ - I) * NS4, v, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                        });
                    });
                }
            }
        }
        wait_lds_barrier();  // B2: parity of rows [0, R) complete

        // ---- C: codeword words of the own item into the output tile; parity rows move down by R
        {
            uint32_t Qv[NPA];
#pragma unroll
            for (int jj = 0; jj < NPA; ++jj) Qv[jj] = 0;
            if (active) {
                // rows [0, n-1) take over rows [R, R+n-1) (zeroed); the other rows are zeroed
                const bool mv = p < n - 1;
                uint32_t* zdst = scratch + tid;  // writes that must not land anywhere
#pragma unroll
                for (int jj = 0; jj < NP; ++jj) {
                    uint32_t* r0p = q + jj * QJ + p * NS4 + g;
                    uint32_t* r1p = q + jj * QJ + (R + (mv ? p : 0)) * NS4 + g;
                    const uint32_t v0 = *r0p, v1 = *r1p;
                    Qv[jj] = v0;
                    *r0p = mv ? v1 : 0u;
                    *(mv ? r1p : zdst) = 0u;
                }
            }
            const int t = row0 + p;
            uint32_t X[n];
            tgroup_words<K, NP>(H, Qv, X);
            if constexpr (SEG) {
                // rows at the compact layout's stride W (16-byte aligned, dword-aligned groups): the
                // group's n words in place; the last group's lane also zeroes the row's pad dwords past
                // its words (its words past the codeword's end are zero: zero pad, zero parity)
                const int Wb = CL ? ((CG.CW + 15) & ~15) : static_cast<int>(a.W);
                const int d0 = (p * Wb + 4 * n * g) >> 2;
                const int cntw = !(it > 0 && active && t < P) ? 0 : (is_last ? min(n + 3, (Wb >> 2) - n * g) : n);
                uint32_t* outw = reinterpret_cast<uint32_t*>(out) + d0;
                uint32_t* zdst = scratch + tid;
#pragma unroll
                for (int qq = 0; qq < n + 3; ++qq) *(qq < cntw ? outw + qq : zdst) = qq < n ? X[qq] : 0u;
            } else {
            // the batch's last codeword may end inside a dword: the packet after it (not emitted)
            // still writes its first dword, which carries that codeword's last bytes
            const bool emit = it > 0 && active && (t < P || (t == P && g == 0));
            uint32_t tw = X[n - 1];
            if (is_last) {
                switch (rem) {
                    case 1: tw = ttail_rem<n, 1>(X); break;
                    case 2: tw = ttail_rem<n, 2>(X); break;
                    case 3: tw = ttail_rem<n, 3>(X); break;
                    default: break;
                }
            }
            const uint32_t prev = tbperm(lane - 1 < 0 ? 0 : lane - 1, tw);
            const int o = p * CW + 4 * n * g;  // byte offset of the item in the output tile
            const int al = o & 3;
            // word qq of the shifted image = bytes [4 - al, 8 - al) of {X[qq-1] (or prev), X[qq]}
            const uint32_t shsel = 0x03020100u + static_cast<uint32_t>(4 - al) * 0x01010101u;
            const int d0 = (o - al) >> 2;
            // dwords written: n, except the last group of a packet: up to the packet end (the dword
            // shared with the next packet is that packet's first lane's)
            const int cntw = !emit ? 0 : (t >= P ? 1 : (is_last ? ((p + 1) * CW >> 2) - d0 : n));
            if (!(dbg & 2)) {
                uint32_t* outw = reinterpret_cast<uint32_t*>(out) + d0;
                uint32_t* zdst = scratch + tid;
#pragma unroll
                for (int qq = 0; qq < n; ++qq) {
                    const uint32_t lo = qq == 0 ? prev : X[qq - 1];
                    *(qq < cntw ? outw + qq : zdst) = __builtin_amdgcn_perm(X[qq], lo, shsel);
                }
            }
            }
        }
        wait_lds_barrier();  // B3: output tile complete
        if (it == 0) continue;

        // ---- D: output tile -> HBM (16-byte chunks); trimmed sizes
        if (segm) {
            // row by row into the frames' arrays (stride W, a multiple of 16): chunk c of row p is
            // LDS bytes [p*CW + 16c, +16), the bytes past the codeword zeroed.  Every wave issues
            // the same stores (counted in vm_issued): one into the cur rows and one into the old rows per
            // chunk, a lane's other one out of range (buffer stores drop it).
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            const int64_t W64 = a.W;
            const int nsw = static_cast<int>(min<int64_t>(ssw - sfirst, P));  // rows from nsw on go to old
            const __amdgpu_buffer_rsrc_t rcur =
                __builtin_amdgcn_make_buffer_rsrc(a.cur_rows + scur, 0, static_cast<int>(nsw * W64), 0x00020000);
            const __amdgpu_buffer_rsrc_t rold =
                __builtin_amdgcn_make_buffer_rsrc(a.old_rows + sold, 0, static_cast<int>((P - nsw) * W64), 0x00020000);
            for (int j = 0; j < nit_seg; ++j) {
                const int qq = tid + j * kTileThreads;
                const int pq = qq / nch_seg, c = qq - pq * nch_seg;
                const int t = row0 + pq;
                const bool ok = qq < R * nch_seg && t < P;
                // row pq of the output tile at stride W (phase C wrote its pad dwords as zero)
                const v4u vv = *reinterpret_cast<const v4u*>(out + (ok ? pq * static_cast<int>(W64) + 16 * c : 0));
                const int off = t * static_cast<int>(W64) + 16 * c;
                const int off_old = (t - nsw) * static_cast<int>(W64) + 16 * c;
                __builtin_amdgcn_raw_buffer_store_b128(vv, rcur, ok && t < nsw ? off : 0x7ffffff0, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(vv, rold, ok && t >= nsw ? off_old : 0x7ffffff0, 0, 0);
                vm_issued += 2;
            }
            const bool own = tid < R && row0 + tid < P;
            const uint8_t* cwp = out + (own ? tid : 0) * static_cast<int>(W64);
            int sz = CW;
            if (__builtin_amdgcn_ballot_w64(own && cwp[CW - 1] == 0)) {  // rare: a codeword ending in zero bytes
                if (own && cwp[CW - 1] == 0) {
                    sz = 0;
                    for (int b = CW - 2; b >= 0; --b)
                        if (cwp[b] != 0) {
                            sz = b + 1;
                            break;
                        }
                }
            }
            const __amdgpu_buffer_rsrc_t rlc = __builtin_amdgcn_make_buffer_rsrc(a.cur_len + sfirst, 0, 4 * P, 0x00020000);
            const __amdgpu_buffer_rsrc_t rlo = __builtin_amdgcn_make_buffer_rsrc(a.old_len + sfirst, 0, 4 * P, 0x00020000);
            const int tl = row0 + tid;
            __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(sz), rlc, own && tl < nsw ? 4 * tl : 0x7ffffff0, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(sz), rlo, own && tl >= nsw ? 4 * tl : 0x7ffffff0, 0, 0);
            vm_issued += 2;
        } else {
            const int gbase = row0 * CW;  // 16-byte aligned
            const int lim = P * CW - gbase;
            const int tb = R * CW;
            const bool tail_tile = lim < tb;  // the batch ends inside this tile (uniform)
            for (int j = 0; j < nso; ++j) {
                const int c = (tid + j * kTileThreads) * 16;
                const bool inb = c < tb;
                const uint4 v = *reinterpret_cast<const uint4*>(out + (inb ? c : 0));
                if (tail_tile && inb && c + 16 > lim && c < lim) {  // the batch end inside this chunk: dwords, bytes
                    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
                    for (int b = 0; b < lim - c; b += 4) {
                        if (b + 4 <= lim - c) {
                            __builtin_amdgcn_raw_buffer_store_b32(w4[b >> 2], rc, gbase + c + b, 0, 0);
                        } else {
                            for (int y = b; y < lim - c; ++y)
                                __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(w4[b >> 2] >> (8 * (y - b))),
                                                                     rc, gbase + c + y, 0, 0);
                        }
                    }
                }
                const bool full = inb && c + 16 <= lim;
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                const v4u vv = {v.x, v.y, v.z, v.w};
                const int so = full && !(dbg & 4) ? gbase + c : 0x7ffffff0;
                if (a.nt & 1)
                    __builtin_amdgcn_raw_buffer_store_b128(vv, rc, so, 0, 2);  // nt
                else
                    __builtin_amdgcn_raw_buffer_store_b128(vv, rc, so, 0, 0);
                ++vm_issued;
            }
            // trimmed wire size of packet tid (FEC_Encoder.cpp:55-60): 1 + last non-zero byte; a
            // runtime-L kernel's caller may not want them (cw_len null: the adaptive relay's batches)
            if (LC == 0 && a.cw_len == nullptr) continue;
            const bool own = tid < R && row0 + tid < P;
            const uint8_t* cwp = out + (own ? tid : 0) * CW;
            const bool zlast = cwp[CW - 1] == 0;
            int sz = CW;
            if (__builtin_amdgcn_ballot_w64(own && zlast)) {  // a codeword ending in zero bytes
                if (own && zlast) {
                    if constexpr (LC == 0) {
                        // the runtime-L kernels (the adaptive relay's codes, whose zero-length gap
                        // rows are all-zero codewords): 16 bytes a step
                        sz = last_nonzero_end(cwp, CW - 1);
                    } else {
                        // byte by byte: the scan above inlined here made the L = 300 headline
                        // kernel 137 -> 230 us (registers; profiles/r06/r06z_encoder_scan.txt)
                        sz = 0;
                        for (int b = CW - 2; b >= 0; --b)
                            if (cwp[b] != 0) {
                                sz = b + 1;
                                break;
                            }
                    }
                }
            }
            __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(sz), rw, own ? 4 * (row0 + tid) : 0x7ffffff0,
                                                  0, 0);
            ++vm_issued;
        }
    }
    wait_vm(0);
}

}  // namespace

// Workgroups per CU the register budget is sized for: five (96 VGPRs), or four / three when a
// wave's share of the K*NP coefficient tables would not fit beside the rest (it spilled to scratch).
template <int K, int NP>
constexpr int tile_min_wg() {
    return K * NP > 36 ? 3 : (K * NP >= 27 ? 4 : FEC_TILE_MINWG);
}

template <int K, int NP, int LC, bool SEG>
__global__ __launch_bounds__(kTileThreads, (tile_min_wg<K, NP>())) void fec_encode_tile_kernel(EncTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tsmem[];
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
        case 0: tile_walk<K, NP, 0, LC, SEG>(a, tsmem); break;
        case 1: tile_walk<K, NP, 1, LC, SEG>(a, tsmem); break;
        case 2: tile_walk<K, NP, 2, LC, SEG>(a, tsmem); break;
        default: tile_walk<K, NP, 3, LC, SEG>(a, tsmem); break;
    }
}

#ifdef FEC_WAVE_ONLY
#define FEC_ENC_TILE_LIST(X) X(8, 3)
#define FEC_ENC_TILE_L300_LIST(X) X(8, 3)
#define FEC_ENC_TILE_SEG300_LIST(X) X(8, 3)
#else
#define FEC_ENC_TILE_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(3, 8) X(2, 9)  \
    X(10, 3) X(9, 3) X(10, 4) X(8, 4) X(10, 5) X(7, 5) X(3, 9)
// L = 300 specialisations: the (T,B,N) of BASELINE configs 1-3 and 5
#define FEC_ENC_TILE_L300_LIST(X) X(8, 3) X(9, 5)
// segment mode at L = 300 (config 4's tuples): the list's entries with an L = 300 tile geometry
#define FEC_ENC_TILE_SEG300_LIST(X) \
    X(8, 3) X(9, 5) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(10, 3) X(9, 3) X(10, 4) \
    X(8, 4) X(10, 5) X(7, 5) X(10, 0) X(9, 1) X(6, 0) X(9, 0) X(8, 2) X(8, 1) X(5, 0)
#endif

#define FEC_ENC_TILE_INST(K, NP) \
    template __global__ void fec_encode_tile_kernel<K, NP, 0, false>(EncTileArgs); \
    template __global__ void fec_encode_tile_kernel<K, NP, 0, true>(EncTileArgs);
#define FEC_ENC_TILE_INST300(K, NP) template __global__ void fec_encode_tile_kernel<K, NP, 300, false>(EncTileArgs);
#define FEC_ENC_TILE_SEG_INST300(K, NP) template __global__ void fec_encode_tile_kernel<K, NP, 300, true>(EncTileArgs);
FEC_ENC_TILE_LIST(FEC_ENC_TILE_INST)
FEC_ENC_TILE_L300_LIST(FEC_ENC_TILE_INST300)
FEC_ENC_TILE_SEG300_LIST(FEC_ENC_TILE_SEG_INST300)

const void* fec_encode_tile_kernel_for(int k, int np, int L) {
    if (!std::getenv("FEC_TILE_RUNTIME_L") && L == 300) {
#define FEC_ENC_TILE_CASE300(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_encode_tile_kernel<K, NP, 300, false>);
        FEC_ENC_TILE_L300_LIST(FEC_ENC_TILE_CASE300)
#undef FEC_ENC_TILE_CASE300
    }
#define FEC_ENC_TILE_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_encode_tile_kernel<K, NP, 0, false>);
    FEC_ENC_TILE_LIST(FEC_ENC_TILE_CASE)
#undef FEC_ENC_TILE_CASE
    return nullptr;
}

// Several tuples' segment walks in one launch (EncMultiArgs).  The register budget is that of 4
// workgroups per CU (128 VGPRs), which every listed tuple's walk fits; LDS is the largest listed
// tuple's (the launcher sizes it).
// (the second line: the hop-1 tuples of the two-hop relay session, whose sender splits T_TOT --
// T = T_TOT - N2 -- so T < 10 codes with B = N appear: (9,0,0), (9,1,1), (5,0,0), (8,0,0), (9,2,2),
// (8,1,1), (4,0,0) are 48 % of its packets on bin/erasure.bin)
#define FEC_ENC_TILE_MULTI_LIST(X) \
    X(8, 3) X(11, 0) X(10, 1) X(9, 2) X(7, 4) X(6, 5) X(5, 6) X(4, 7) X(10, 3) X(9, 3) X(8, 4) X(7, 5) \
    X(10, 0) X(9, 1) X(6, 0) X(9, 0) X(8, 2) X(8, 1) X(5, 0)

template <int K, int NP>
__device__ __forceinline__ void tile_multi_case(const EncMultiArgs& m, int ti, uint8_t* smem) {
    constexpr TileGeom CG = tile_geometry(K, NP, 300, true);
    EncTileArgs a{};
    a.payload_base = m.payload;
    a.len_base = m.len;
    a.ptab = m.gtab + m.toff[ti];
    a.L = 300;
    // the walk reads segment blockIdx.x: with the leftovers' workgroups first, that is m.ncf past
    // its segment in m.seg
    a.seg = m.cf_first ? m.seg - 6 * static_cast<int64_t>(m.ncf) : m.seg;
    a.cur_rows = m.cur_rows;
    a.old_rows = m.old_rows;
    a.cur_len = m.cur_len;
    a.old_len = m.old_len;
    a.W = (CG.CW + 15) & ~15;
    a.nt = m.nt;
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
        case 0: tile_walk<K, NP, 0, 300, true>(a, smem); break;
        case 1: tile_walk<K, NP, 1, 300, true>(a, smem); break;
        case 2: tile_walk<K, NP, 2, 300, true>(a, smem); break;
        default: tile_walk<K, NP, 3, 300, true>(a, smem); break;
    }
}

// Workgroups past the segments' (m.ncf of them) encode the schedule's leftover codewords in closed
// form (fec_vr_cf.h): they start as the segment walks drain and fill the launch's tail.
__global__ __launch_bounds__(kTileThreads, 4) void fec_encode_tile_multi_kernel(EncMultiArgs m, VrEncodeArgs cf) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tsmem[];
    int bid = static_cast<int>(blockIdx.x);
    if (m.cf_first) {  // (the leftovers' workgroups first instead)
        if (bid < m.ncf) {
            vr_encode_cf_body(cf, tsmem, bid, m.ncf);
            return;
        }
        bid -= m.ncf;
    } else if (bid >= m.tfirst[m.ntuple]) {
        vr_encode_cf_body(cf, tsmem, bid - m.tfirst[m.ntuple], m.ncf);
        return;
    }
    int ti = 0;
    while (ti + 1 < m.ntuple && bid >= m.tfirst[ti + 1]) ++ti;
    switch (m.tkey[ti]) {
#define FEC_ENC_TILE_MULTI_CASE(K, NP) \
    case K * 32 + NP: tile_multi_case<K, NP>(m, ti, tsmem); break;
        FEC_ENC_TILE_MULTI_LIST(FEC_ENC_TILE_MULTI_CASE)
#undef FEC_ENC_TILE_MULTI_CASE
        default: break;
    }
}

bool fec_encode_tile_multi_supports(int k, int np, int L) {
    if (L != 300) return false;
#define FEC_ENC_TILE_MULTI_HAS(K, NP) \
    if (k == K && np == NP) return true;
    FEC_ENC_TILE_MULTI_LIST(FEC_ENC_TILE_MULTI_HAS)
#undef FEC_ENC_TILE_MULTI_HAS
    return false;
}
const void* fec_encode_tile_multi_kernel_ptr() { return reinterpret_cast<const void*>(&fec_encode_tile_multi_kernel); }

// The segment-mode instance for the variable-rate schedule (L = 300 fixed at compile time, else
// from the arguments), or nullptr.
const void* fec_encode_tile_seg_kernel_for(int k, int np, int L) {
    if (L == 300) {
#define FEC_ENC_TILE_SEG_CASE300(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_encode_tile_kernel<K, NP, 300, true>);
        FEC_ENC_TILE_SEG300_LIST(FEC_ENC_TILE_SEG_CASE300)
#undef FEC_ENC_TILE_SEG_CASE300
    }
#define FEC_ENC_TILE_SEG_CASE(K, NP) \
    if (k == K && np == NP) return reinterpret_cast<const void*>(&fec_encode_tile_kernel<K, NP, 0, true>);
    FEC_ENC_TILE_LIST(FEC_ENC_TILE_SEG_CASE)
#undef FEC_ENC_TILE_SEG_CASE
    return nullptr;
}

}  // namespace fec
