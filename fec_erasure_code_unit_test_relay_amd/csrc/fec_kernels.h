// fec_kernels.h -- device kernels of the MI355X streaming-erasure codec (gfx950 / CDNA4).
//
// Byte-wise GF(2^8) work, HBM-bound: no MFMA.  The kernels (launchers in fec_codec.hip):
//   fec_encode_kernel      closed-form diagonal-interleaved encode of a tile of packets
//                          (replaces Encoder::encodeStream -> Encoder_Basic -> encodeBlock,
//                          src/Encoder.cpp:65-98, src/Encoder_Basic.cpp:48-74,
//                          src/codingOperations.cpp:131-147);
//   fec_episode_kernel     finds the packets where the reference decoder leaves its fast path
//                          and resynchronises (src/Decoder.cpp:80-83, 109-133), the loss
//                          episodes they start and their shapes (fec_shapes.hip);
//   fec_plan_kernel        one wavefront per (erasure episode, diagonal block): symbolic replay of
//                          the reference's per-symbol decode (decodeBlock / gf256_rref_matrix
//                          through the precomputed decode rules), emitting for every erased
//                          symbol whether it is recovered and its n GF coefficients over the
//                          received symbols of its diagonal codeword;
//   fec_copy_kernel        systematic gather + length parse for every received packet (the
//                          decoder's fast path, src/Decoder.cpp:77-108, and the slow path's
//                          received packets);
//   fec_recover_kernel     applies the coefficients to the bytes of every recovered packet.
// The per-packet coders run on fec_streams.hip's kernels (stream_encode_one / stream_decode_one).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <stdint.h>

namespace fec {

struct EncArgs {
    const uint8_t* payload;     // row 0 = first packet of the batch
    const int32_t* len;         // may be null (all L)
    int64_t history;            // valid rows before row 0
    int64_t P;
    uint8_t* cw;
    int32_t* cw_len;
    const uint32_t* ptab;       // [k][n-k][8] perm tables per parity coefficient
    int L, k, n, S, CW;
    int SP;                     // S rounded up to a multiple of 4
    int TP;                     // packets per workgroup tile
    int ROWS;                   // TP + n - 1
    int plane;                  // ROWS * SP  (bytes of one position plane)
    int xin_bytes, xout_bytes;  // 16-aligned LDS carve sizes
};

struct EncTileArgs {
    const uint8_t* payload_base;  // row -history (4-byte aligned, L % 4 == 0)
    const int32_t* len_base;      // lengths of rows -history.. (null: all L)
    int payload_bytes;            // (history + P) * L < 2^31 (the launcher splits larger batches)
    int len_bytes;                // (history + P) * 4
    int history;                  // valid rows before row 0 (<= n-1)
    int P;
    uint8_t* cw;                  // 16-byte aligned
    int cw_bytes;                 // P * CW < 2^31
    int32_t* cw_len;
    const uint32_t* ptab;         // [k][n-k][8] register tables of G's parity coefficients
    int L, CW, NS4;
    int PPW;                      // packets per wave slice (tile R = 4 * PPW packets, PPW*CW % 4 == 0)
    int rem;                      // sub-streams in the last group (1..4)
    int nvl;                      // payload dwords of a row from dword K*(NS4-1) on (last group)
    int tiles_per_wg, ntiles;     // consecutive tiles per workgroup; ceil(P / R)
    int ngl;                      // 1 KB LDS-DMA pieces per wave per tile (4 * ngl KB >= R*L + 4K + 8)
    int nso;                      // 16-byte output stores per thread per tile (ceil(R*CW / 4096))
    int off_in, in_bytes, off_pw, off_q, off_out, off_len;  // dynamic LDS carve-up (bytes)
    int off_scratch;              // 1 KB: a dword per thread for writes that must land nowhere
    int dbg;                      // timing experiments only (FEC_TILE_DBG): 1 no parity products,
                                  // 2 no codeword words, 4 no output stores
    int nt;                       // 1: codeword stores non-temporal (FEC_TILE_NT); 2: payload loads non-temporal;
                                  // 4: segment mode computes the zero history tile of an instance start
    // segment mode (variable-rate schedule, fec_vr.cpp): null for one stream.  Per workgroup 6
    // int64: first seq of the encoder instance (its row 0), its role-switch seq, its rows P,
    // t0 | cnt << 32 (tiles [t0, t0+cnt) of the instance), and the byte offsets of the instance's
    // first cur row and first old row in cur_rows / old_rows (the compact layout, fec_vr.h).
    // history = 0; rows before / from the role switch go to cur_rows / old_rows at stride W (the
    // instance's CW rounded to 16).
    const int64_t* seg;
    uint8_t* cur_rows;
    uint8_t* old_rows;
    int32_t* cur_len;
    int32_t* old_len;
    int64_t W;
};

// Geometry of the tile encoder for (k, n-k, L): one definition for the host launcher and the
// kernels specialised on L at compile time.  ok = 0: the tile form does not apply.
struct TileGeom {
    int ok;
    int S, CW, NS4, PPW, R, rem, nvl, ngl, nso;
    int off_in, in_bytes, off_pw, off_q, off_out, off_len, off_scratch;
    int lds, lds_len;  // dynamic LDS without / with the length rows
};
// seg: the segment-mode layout, whose output tile holds rows at the compact layout's stride W
// (CW rounded to 16: rows leave as aligned 16-byte LDS reads) instead of packed at CW.
constexpr TileGeom tile_geometry(int k, int np, int L, bool seg = false) {
    TileGeom t{};
    const int n = k + np;
    t.S = (L + 2 + k - 1) / k;
    t.CW = t.S * n;
    t.NS4 = (t.S + 3) / 4;
    // a wave slice holds whole packets (PPW * NS4 <= 64) whose codewords end on a dword
    // (PPW * CW % 4 == 0), and a tile (4 * PPW packets) covers the n-1 packets of parity history
    const int unit = (t.CW & 3) == 0 ? 1 : ((t.CW & 1) == 0 ? 2 : 4);
    const int ppw = t.NS4 > 0 && t.NS4 <= 64 ? (64 / t.NS4) / unit * unit : 0;
    if ((L & 3) != 0 || np < 0 || ppw <= 0 || 4 * ppw < n - 1) return t;
    t.PPW = ppw;
    t.R = 4 * ppw;
    const int rs = (L + 15) & ~15;  // LDS row stride of the input tile
    t.ngl = (t.R * rs + 16 + 4095) / 4096;
    const int pws = k | 1;
    const int rows = t.R + n - 1;
    const int npa = np > 0 ? np : 1;
    int off = 64;  // guard in front of the input buffers (the first row's dword -1)
    t.in_bytes = t.ngl * 4096;
    t.off_in = off;
    off += 2 * t.in_bytes;
    // the position words (read before the second barrier of a tile) and the output tile (written
    // after it) share one region
    t.off_pw = off;
    t.off_out = off;
    const int pwb = 4 * t.R * t.NS4 * pws, outb = t.R * (seg ? (t.CW + 15) & ~15 : t.CW);
    off = (off + (pwb > outb ? pwb : outb) + 15) & ~15;
    t.off_q = off;
    off = (off + 4 * npa * rows * t.NS4 + 15) & ~15;
    t.off_scratch = off;
    off += 1024;
    t.lds = off;
    t.off_len = off;  // lengths (only with a length array)
    t.lds_len = off + 2048;
    t.nso = (t.R * t.CW / 16 + 255) / 256;
    t.rem = t.S - 4 * (t.NS4 - 1);
    t.nvl = L / 4 - k * (t.NS4 - 1);
    t.ok = t.ngl <= 4 && t.lds_len <= 160 * 1024;
    return t;
}

// fec_encode_tile_kernel<k, n-k, L> for L = 300 (the reference's payload size, L fixed at compile
// time) or <k, n-k, 0> (L from the arguments) (fec_encode_tile.hip), else nullptr.  256 threads.
const void* fec_encode_tile_kernel_for(int k, int np, int L);
// fec_encode_tile_kernel<k, n-k, 300 or 0> with segment mode (EncTileArgs::seg) compiled in, else nullptr.
const void* fec_encode_tile_seg_kernel_for(int k, int np, int L);

// Segment mode for several (k, n-k) tuples in one launch (the variable-rate schedule at L = 300):
// workgroup b serves segment b of the concatenated segment table; the segments of tuple t are
// [tfirst[t], tfirst[t+1]) and it is encoded by fec_encode_tile_kernel<k_t, n_t-k_t, 300, true>'s
// walk.  Only tuples for which fec_encode_tile_multi_supports() holds (their walk fits the shared
// register budget of 4 workgroups per CU).
constexpr int kEncMultiMax = 24;
struct EncMultiArgs {
    const uint8_t* payload;       // [sent][L] payload rows
    const int32_t* len;           // lengths (null: all L)
    const uint32_t* gtab;         // gf_mul4 tables of every tuple
    const int64_t* seg;           // [nseg][6] segment table, grouped by tuple
    uint8_t* cur_rows;
    uint8_t* old_rows;
    int32_t* cur_len;
    int32_t* old_len;
    int L;                        // 300
    int ntuple;
    int tkey[kEncMultiMax];       // k * 32 + (n - k)
    int tfirst[kEncMultiMax + 1];
    int toff[kEncMultiMax];       // dword offset of the tuple's tables in gtab
    int nt;                       // EncTileArgs::nt for every walk (bit 1: non-temporal payload loads)
    int ncf;                      // workgroups after the segments' running the closed-form leftovers
                                  // (the kernel's second argument, VrEncodeArgs; 0: none)
    int cf_first;                 // 1: those workgroups come first (FEC_VR_CF_FIRST=1)
};
bool fec_encode_tile_multi_supports(int k, int np, int L);
const void* fec_encode_tile_multi_kernel_ptr();

struct CopyFastArgs {
    const uint8_t* cw;
    const uint8_t* er;
    int64_t P, Pout;
    uint8_t* out;               // 4-byte aligned, L % 4 == 0
    int32_t* out_len;
    int L, CW, NS4, T, TP;
    int raw_bytes;              // codeword tile + slack (16-aligned)
    int out_bytes;              // payload tile (16-aligned)
    uint64_t* stamps;           // diagnostics: per-workgroup phase timestamps (null = off)
    int skip_erased;            // 1: leave erased packets' rows and lengths to fec_recover_kernel
    int nt;                     // 1: non-temporal codeword loads and payload stores
};

// fec_copy_fast_kernel<k, n-k> for the instantiated pairs (fec_copy_fast.hip), else nullptr.
const void* fec_copy_fast_kernel_for(int k, int np);
// Two consecutive tiles per workgroup, the second one's loads in flight while the first is
// converted (same arguments and LDS as fec_copy_fast_kernel; stage <= kPairQ * 4 KB), or nullptr.
const void* fec_copy_pair_kernel_for(int k, int np);
// Specialised planner for (k, n-k), or nullptr (then fec_plan_kernel runs); its rule table is
// the log-form copy (coefficient bytes log2, 0 -> 0xff).
const void* fec_plan_fast_kernel_for(int k, int np);

struct CopyArgs {
    const uint8_t* cw;
    const uint8_t* er;
    int64_t P, Pout;
    uint8_t* out;
    int32_t* out_len;
    int L, k, n, S, CW, T, TP;
    int cwt_bytes;              // 16-aligned
};

constexpr int kPlanMaxN = 31;  // windows w <= n <= 31 (n > 17: no rule table, rules computed in the wave)

struct PlanArgs {
    const uint8_t* er;
    int64_t P, Pout;
    const uint8_t* rules;
    const uint8_t* G;              // k x n generator (rules computed in the wave when wbase[w] < 0)
    int64_t wbase[kPlanMaxN + 1];  // byte offset of window w's rule table (-1: unused)
    const uint8_t* gf;             // exp[512] then log[256]
    int ES;                        // decode-rule entry stride (bytes, multiple of 4)
    int k, n, T;
    const int32_t* counters;       // [6] episodes to replay, [7] duplicate episodes
    const int32_t* work;           // start packets of the episodes to replay
    const int32_t* dups;           // duplicate episodes: (start packet, shape slot) pairs
    const uint64_t* keys;          // shape of each slot
    const int32_t* reps_tr;        // start packet of each slot's representative
    int32_t* src_d;                // [P] erased output x uses the plan rows of x + src_d[x]
    const uint8_t* rstate;         // post-resync block state per phase (build_resync_states)
    int rs_bytes;
    uint8_t* sym_ok;               // [P][k]: symbol i of erased packet x recovered
    uint8_t* coef;                 // [P][k][n]: coefficients of symbol i over its diagonal
};

// Plan item d >= replay pairs: duplicate episode d's erased outputs point at the representative's
// plan rows (one wave; a keyed shape spans < 64 packets).
__device__ __forceinline__ void episode_dup_fill(const PlanArgs& a, int d, int lane) {
    const int64_t tr = a.dups[2 * d];
    const int slot = a.dups[2 * d + 1];
    const uint64_t m = a.keys[slot];
    const int64_t x = tr + lane;
    if (((m >> lane) & 1u) && x < a.Pout) a.src_d[x] = a.reps_tr[slot] - static_cast<int32_t>(tr);
}

// Resync points, episodes and shapes in one pass (fec_shapes.hip).
struct EpisodeArgs {
    const uint8_t* er;
    int64_t P, Pout;
    int T;
    int tbits;                     // log2 of the hash-table size
    int dedup;                     // 0: every episode is replayed
    int32_t* counters;             // [1] erased outputs, [6] replay count, [7] duplicates (one 64-bit word)
    int32_t* erased;               // erased output packets
    int32_t* src_d;                // [P]: 0 for every erased output (duplicates: set by the plan)
    int32_t* work;                 // replay list (episode start packets)
    int32_t* dups;                 // duplicate list ((start packet, slot) pairs)
    uint64_t* keys;                // [2^tbits], zero = empty
    int32_t* reps_tr;              // [2^tbits] start packet of the slot's representative
    uint64_t* stamps;              // diagnostics: per-workgroup phase timestamps (null = off)
};
__global__ void fec_episode_kernel(EpisodeArgs a);

// Recovered packets -> rec_list (fec_compact_kernel).
struct CompactArgs {
    int32_t* counters;             // [1] erased outputs (in), [2] recovered packets (out)
    const int32_t* erased;         // erased output packets (fec_episode_kernel)
    const int32_t* src_d;          // plan rows of erased output x: those of x + src_d[x]
    const uint8_t* sym_ok;         // [P][k] from the planner
    int k;
    int32_t* rec_list;             // (x, x + src_d[x]) pairs
    int zero_lost;                 // 1: lost packets' rows (zeros) and lengths (0) written here
    uint8_t* out;
    int32_t* out_len;
    int L;
    int64_t row_off;               // packet x goes to output row x - row_off (x < row_off: skipped)
};
__global__ void fec_compact_kernel(CompactArgs a);

struct RecArgs {
    const uint8_t* cw;
    int64_t P, Pout;
    const int32_t* counters;       // [2] recovered packets
    const int32_t* rec_list;       // (x, plan-row packet) pairs (fec_compact_kernel)
    const uint8_t* coef;
    const uint8_t* gf;
    uint8_t* out;
    int32_t* out_len;
    int L, k, n, S, CW;
    int64_t row_off;               // packet x goes to output row x - row_off (x < row_off: skipped)
    int stage_bytes;               // per-wave LDS for the k+n-1 codeword rows of a packet (0: none)
    uint64_t* stamps;              // diagnostics: per-workgroup phase timestamps (null = off)
};
// dynamic LDS of fec_recover_kernel_t<MAXN, .>: tables + 4 waves x (coefficient logs + staged rows)
inline int recover_lds_bytes(int maxn, int stage_bytes) {
    return 1552 + 4 * (((2 * 16 * maxn + 15) & ~15) + stage_bytes);
}
template <int MAXN, bool STAGED>
__global__ void fec_recover_kernel_t(RecArgs a);


// Block mode (fec_block.hip): many independent code blocks of n symbols.
struct BlockArgs {
    const uint8_t* in;          // encode: nblk x k data; decode: nblk x n codewords
    const uint8_t* er;          // decode: nblk x n erasure flags (1 = erased)
    uint8_t* out;               // nblk x n
    uint8_t* er_out;            // decode: updated flags (may be null)
    int64_t nblk;
    int k, n;
    const uint8_t* G;           // k x n generator
    const uint8_t* gf;          // exp[512], log[256]
    const uint8_t* rules;       // decode rule table
    int64_t wbase_n;            // byte offset of window n's table
    int ES;                     // rule entry bytes
};
__global__ void fec_block_encode_kernel(BlockArgs a);

// Host view of a codec's device-resident constants (fec_codec.hip), for other launchers.
struct CodecView {
    int L, T, B, N, k, n, S, CW;
    const uint8_t* G;           // k x n generator (device)
    const uint8_t* gf;          // exp[512], log[256] (device)
    const uint8_t* rules;       // decode rule table, raw coefficients (device)
    int64_t wbase_n;            // byte offset of window n's rules
    int ES;                     // rule entry bytes
};
__global__ void fec_block_decode_kernel(BlockArgs a);

__global__ void fec_encode_kernel(EncArgs a);
__global__ void fec_plan_kernel(PlanArgs a);
__global__ void fec_copy_kernel(CopyArgs a);

__global__ void fec_fill_kernel(uint8_t* out, int64_t t0, int64_t count, int L, uint64_t seed);

}  // namespace fec

struct fec_codec;
namespace fec {
int codec_view(const ::fec_codec* c, CodecView* v);
// ---- resident per-packet servers (fec_server.hip) ----------------------------------------
// Mailbox shared by a per-packet coder (host) and its server workgroup (device), in pinned,
// coherent, mapped host memory.  The host writes the sealed request, then `req`; the server writes
// the result row, then `done`; `stop` ends the server; `alive` / `exited` are its exit handshake.
struct ServerBox {
    uint32_t req;     // ticket of the latest request (host, written last)
    uint32_t stop;    // host: 1 = exit now
    uint32_t alive;   // 1 while a server polls (host sets it before a launch; the server clears it
                      // when it starts to exit, and sets it again if a request arrived meanwhile)
    uint32_t done;    // ticket of the latest finished request (server, written last)
    uint32_t exited;  // server: 1 once its exit is final (after its last look at req); host clears
                      // it before a launch
    uint32_t reserved[7];
};
static_assert(offsetof(ServerBox, exited) == 16 && sizeof(ServerBox) == 48, "mailbox layout");
// A server's sealed request block (pinned, coherent, mapped): unit i = request dword i | ticket << 32,
// each written by the host as one 8-byte store, the units in decreasing index order and the mailbox's
// req word after them.  The server's poll reads the first kServerHeadUnits units and the stop word in
// one round trip and takes the request when every unit it read carries the new ticket; the units past
// the head were written before it and are read afterwards.  Encoder request: [len, seq lo, seq hi,
// payload words]; decoder request (a recovered packet only; the host outputs the systematic copies,
// DESIGN.md §4): [fate, clamp, 5 reserved, the k+n-1 zero-padded codewords of packets x-k+1 .. x+n-1
// (zero rows for missing ones), the k x n coefficients].
constexpr int kServerHeadUnits = 192;
constexpr int kEncReqFields = 3;
constexpr int kDecReqFields = 7;
struct EncServerArgs {
    ServerBox* box;
    const uint64_t* req;        // sealed request block: kEncReqFields + ceil(L / 4) units
    int nunits;
    const uint8_t* stage;       // mapped payload row (dword padded)
    uint8_t* res;               // mapped result row: codeword (dword padded) | trimmed size at res_len_off
    int res_len_off;
    uint8_t* win_home;          // HBM home of the W x SK window ring between launches
    const uint8_t* G;
    const uint8_t* gf;
    int L, k, n, S, CW, SK, W;
    uint32_t last;              // ticket served before this launch
    int64_t idle_ticks;         // exit after this long without a request (100 MHz real-time counter)
};
struct DecServerArgs {
    ServerBox* box;
    const uint64_t* req;        // sealed request block: kDecReqFields + win_units + ceil(k n / 4) units
    int nunits;
    int win_units;              // ceil(Wn * CW / 4)
    uint8_t* res;               // mapped result row: payload (dword padded) | length at res_len_off
    int res_len_off;
    const uint8_t* gf;
    int L, k, n, CW, Wn;        // Wn = k + n - 1 window rows
    uint32_t last;
    int64_t idle_ticks;
};
int server_encode_launch(const EncServerArgs& a, hipStream_t s);
int server_decode_launch(const DecServerArgs& a, hipStream_t s);

// The per-packet FEC_Encoder's call (fec_codec.hip): packet `seq` (relative to the encoder's first)
// of one stream whose window ring `win` ([n-1][S*k], fec_streams.hip's layout) lives on the device,
// through fec_streams_encode_kernel in one launch.  payload / cw / cw_len may be host-visible
// (mapped) rows; after them the kernel stores `ticket` into `done`.
int stream_encode_one(const CodecView& v, uint8_t* win, const uint8_t* payload, int payload_len, int64_t seq,
                      uint8_t* cw, int32_t* cw_len, uint32_t* done, uint32_t ticket, hipStream_t s);
// The per-packet FEC_Decoder's call: store packet `seq`'s codeword `cw` (a host-visible row padded to
// whole dwords; not read when erased) in the 64-row device ring `ring`, output packet x with the
// planner's fate (coef: k x n device block when recovered) into out / out_len, then `ticket` into `done`.
int stream_decode_one(const CodecView& v, uint8_t* ring, const uint8_t* cw, int64_t seq, int erased, int fate,
                      int clamp, int64_t x, const uint8_t* coef, uint8_t* out, int32_t* out_len, uint32_t* done,
                      uint32_t ticket, hipStream_t s);
}  // namespace fec
