/*
 * fec_amd.h -- C ABI of the MI355X-native GF(2^8) streaming-erasure codec.
 *
 * Drop-in boundary for the hot path of domanovi/FEC_Erasure_Code_Unit_Test_Relay.  Every entry
 * point takes plain pointers and sizes (no torch, no C++ types) and returns an int status
 * (FEC_OK = 0, negative = error, see fec_strerror); nothing throws across the ABI.
 *
 * Two layers:
 *   1. Streaming per-packet API (host buffers), one call per sequence number in increasing order
 *      starting at 0 -- exactly the reference's FEC_Encoder::onTransmit / FEC_Decoder::onReceive
 *      contract.  The C++ classes in fec_amd_dropin.h wrap it with the reference's names.
 *   2. Batched device-resident API: many packets of one stream per call, inputs and outputs in
 *      HBM, asynchronous on a caller-supplied hipStream_t (passed as void*; NULL = null stream).
 *
 * Wire formats are the reference's: codeword = S sub-streams of n bytes (k systematic bytes of
 * [len_hi, len_lo, payload, zero pad] then n-k parity bytes); the wire form is that codeword with
 * trailing zero bytes trimmed; a received wire codeword is zero-padded back to CW bytes.
 */
#ifndef FEC_AMD_H
#define FEC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FEC_OK 0
#define FEC_ERR_ARG (-1)          /* bad argument / unsupported (T,B,N) */
#define FEC_ERR_HIP (-2)          /* HIP runtime error (no device, launch failure, ...) */
#define FEC_ERR_NOMEM (-3)        /* allocation failed */
#define FEC_ERR_WORKSPACE (-4)    /* decode workspace too small */
#define FEC_ERR_SEQUENCE (-5)     /* streaming call out of sequence order */
#define FEC_ERR_HISTORY (-6)      /* continuing decode: not enough earlier packets in memory */

typedef struct fec_codec fec_codec;        /* one (max_payload,T,B,N) configuration on a device */
typedef struct fec_encoder fec_encoder;    /* one streaming encoder (per stream) */
typedef struct fec_decoder fec_decoder;    /* one streaming decoder (per stream) */

/* ABI version of this header, returned by fec_version().  2: fec_vr_parse_batch takes the plan
 * first and writes the compact cur/old layout (the d_cw_cur / d_cw_old of the fec_vr_* calls are
 * compact arrays since then, fec_vr.h); a caller built against version 1 must be rebuilt. */
#define FEC_AMD_ABI_VERSION 2

const char *fec_strerror(int status);
/* The last failed HIP runtime call behind an FEC_ERR_HIP (its error name and source line), as a
 * NUL-terminated string written to buf (truncated to size); returns its length, 0 when none. */
int fec_last_error(char *buf, size_t size);
int fec_version(void);

/* ---- configuration -------------------------------------------------------------------------
 * Replaces the constructors Encoder::Encoder / Decoder::Decoder (src/Encoder.cpp:26-50,
 * src/Decoder.cpp:24-53) and init_at_sender/gen_G_cauchy (src/codingOperations.cpp:48-116):
 * derives k=T-N+1, n=k+B, S=ceil((max_payload+2)/k), CW=S*n, builds G and the decode rules and
 * uploads them to the current HIP device.  Requires N <= B (as every reference configuration). */
int fec_codec_create(int max_payload, int T, int B, int N, fec_codec **out);
int fec_codec_destroy(fec_codec *codec);
int fec_codec_geometry(const fec_codec *codec, int *k, int *n, int *S, int *CW);
/* Kernel configuration chosen for this codec and device (tiles, resident workgroups), as a JSON
 * object written to buf (NUL-terminated, truncated to size). */
int fec_codec_info(const fec_codec *codec, char *buf, size_t size);
/* Encode kernel selection: 0 = automatic (the tile kernel -- contiguous runs of LDS-staged packet
 * tiles per workgroup -- when one is compiled for (k, n-k), max_payload % 4 == 0, the payload is
 * 4-byte and the codeword buffer 16-byte aligned; else the generic one), 1 = generic kernel,
 * 5 = tile kernel (FEC_ERR_ARG if unavailable).  Ids 2-4 (round 2's per-tile, streaming and
 * wave-sequence kernels, all slower) are retired and return FEC_ERR_ARG.  Every path produces
 * identical bytes; the switch exists for tests and A/B timing. */
int fec_codec_set_encode_path(fec_codec *codec, int path);
/* The same switch for the decoder's received-packet copy kernel: 0 automatic (the LDS-tile
 * specialised kernel when one is compiled for (k, n-k) and max_payload % 4 == 0, else the generic
 * one), 1 generic, 2 LDS-tile specialised.  Ids 3-6 (barrier-free wave, persistent tile, chunk and
 * per-wave LDS-DMA pipeline copies, all measured slower in the step) are retired. */
int fec_codec_set_copy_path(fec_codec *codec, int path);
/* The same switch for the decoder's planner (per-episode block replay). */
int fec_codec_set_plan_path(fec_codec *codec, int path);
/* Planner: replay one episode per distinct loss shape and copy its results to the other episodes
 * of that shape (default 1), or replay every episode (0).  Outputs are identical either way. */
int fec_codec_set_episode_dedup(fec_codec *codec, int on);
/* Encoder::getG / Decoder::getG (src/Encoder.cpp:61, src/Decoder.cpp:68): k*n bytes row-major. */
int fec_codec_generator(const fec_codec *codec, uint8_t *G);

/* ---- batched device-resident encode --------------------------------------------------------
 * Batched FEC_Encoder::onTransmit (src/FEC_Encoder.cpp:42-68) for P consecutive packets of one
 * stream.  d_payload: P rows of max_payload bytes (row p = packet seq0+p); d_payload_len: P
 * payload lengths (<= max_payload) or NULL = all max_payload.  `history` rows BEFORE d_payload
 * (d_payload - history*max_payload, and d_payload_len - history) are earlier packets of the same
 * stream; packets before those count as zero (encoder created there).  Writes d_codeword (P rows
 * of CW bytes, untrimmed, zero padded exactly as the decoder re-pads) and d_codeword_len (P
 * trimmed wire sizes). */
int fec_encode_batch(fec_codec *codec, const uint8_t *d_payload, const int32_t *d_payload_len,
                     int64_t history, int64_t P, uint8_t *d_codeword, int32_t *d_codeword_len,
                     void *hip_stream);

/* ---- batched device-resident decode --------------------------------------------------------
 * A fresh FEC_Decoder (src/FEC_Decoder.cpp:26-72) fed packets seq 0..P-1 of one stream:
 * d_codeword: P rows of CW bytes (zero padded; rows of erased packets are never read);
 * d_erasure: P bytes, 1 = packet missing.  Produces the reference's output for packets
 * 0..P-T-1: d_payload_out ((P-T) rows of max_payload bytes, zero beyond the payload) and
 * d_payload_len ((P-T) ints, 0 = lost).  d_workspace: fec_decode_workspace_bytes(P) bytes. */
size_t fec_decode_workspace_bytes(const fec_codec *codec, int64_t P);
int fec_decode_batch(fec_codec *codec, const uint8_t *d_codeword, const uint8_t *d_erasure,
                     int64_t P, uint8_t *d_payload_out, int32_t *d_payload_len, void *d_workspace,
                     size_t workspace_bytes, void *hip_stream);
/* ---- continuing batched decode --------------------------------------------------------------
 * One stream decoded in consecutive batches, each call continuing where the previous one ended
 * (the state of src/Decoder.cpp:72-175 -- latest erasure, stored codewords, open episode -- carried
 * across calls): equal, row for row, to fec_decode_batch over the concatenated stream.
 * fec_decode_stream_push takes the next P packets (d_codeword, d_erasure on the device; h_erasure
 * the same P flags on the host -- the receiver knows which packets arrived); `history` rows
 * BEFORE each of the three pointers are the stream's preceding packets (at least T of them after
 * the first call).  It writes *n_out rows (the packets whose output became available: from the
 * first packet not yet output up to the T-th last packet pushed) to d_payload_out / d_payload_len.
 * Internally the decode restarts at the latest packet where the reference decoder is on its fast
 * path for T+1 packets on both sides; FEC_ERR_HISTORY if no such packet lies within `history`
 * (keep more earlier packets: an erasure episode never exceeds the burst length + 2T + 2).
 * Workspace: fec_decode_workspace_bytes(P + history). */
typedef struct fec_decode_stream fec_decode_stream;
int fec_decode_stream_create(fec_decode_stream **out);
int fec_decode_stream_destroy(fec_decode_stream *st);
int fec_decode_stream_push(fec_codec *codec, fec_decode_stream *st, const uint8_t *d_codeword,
                           const uint8_t *d_erasure, const uint8_t *h_erasure, int64_t P, int64_t history,
                           uint8_t *d_payload_out, int32_t *d_payload_len, int64_t *n_out,
                           void *d_workspace, size_t workspace_bytes, void *hip_stream);
/* Packets pushed so far and the packet the last push restarted the decode at. */
int fec_decode_stream_state(const fec_decode_stream *st, int64_t *consumed, int64_t *last_cut);
/* The same decode in two halves.  fec_decode_plan needs only the erasure pattern (it can run
 * while the codewords are still being produced or transferred); fec_decode_apply needs the
 * codewords and must be ordered after the plan (same stream, or an event).  fec_decode_batch =
 * plan on an internal side stream concurrently with the systematic copy, joined before the
 * recovery pass. */
int fec_decode_plan(fec_codec *codec, const uint8_t *d_erasure, int64_t P, void *d_workspace,
                    size_t workspace_bytes, void *hip_stream);
int fec_decode_apply(fec_codec *codec, const uint8_t *d_codeword, const uint8_t *d_erasure,
                     int64_t P, uint8_t *d_payload_out, int32_t *d_payload_len, void *d_workspace,
                     size_t workspace_bytes, void *hip_stream);
/* fec_decode_apply = fec_decode_copy (received packets' rows and lengths; independent of the plan,
 * may run concurrently with it) followed by fec_decode_recover (erased packets' rows and lengths:
 * recovered bytes, or zeros and length 0 when lost; after the plan). */
int fec_decode_copy(fec_codec *codec, const uint8_t *d_codeword, const uint8_t *d_erasure,
                    int64_t P, uint8_t *d_payload_out, int32_t *d_payload_len, void *hip_stream);
int fec_decode_recover(fec_codec *codec, const uint8_t *d_codeword, int64_t P,
                       uint8_t *d_payload_out, int32_t *d_payload_len, void *d_workspace,
                       size_t workspace_bytes, void *hip_stream);
/* After the stream has finished the decode: erasure episodes, recovered and lost packets. */
int fec_decode_counters(const void *d_workspace, int64_t *episodes, int64_t *recovered,
                        int64_t *lost);
/* Planner statistics of the last plan in d_ws: episodes replayed and episodes filled from a
 * replayed episode of the same loss shape (fec_codec_set_episode_dedup). */
int fec_decode_plan_stats(const void *d_ws, int64_t *replayed, int64_t *filled);

/* ---- many independent streams, one packet of each per call ---------------------------------
 * A group of `nstreams` independent streams of one (max_payload,T,B,N): the state of one
 * FEC_Encoder and one FEC_Decoder per stream (include/FEC_Encoder.h:26-48, FEC_Decoder.h:27-46)
 * held in HBM (encoder windows, decoder codeword rings) plus the decoders' symbolic state on the
 * host.  One call hands over the next packet of each of M distinct streams (ids[m], host array)
 * and codes all of them in one launch -- the relay / receiver load of many 300-byte streams.
 *   fec_streams_encode  = FEC_Encoder::onTransmit per stream: d_payload M rows of max_payload
 *                         bytes, d_payload_len M sizes (NULL = all max_payload) -> d_codeword M rows
 *                         of CW bytes (untrimmed) + d_codeword_len M trimmed wire sizes.
 *   fec_streams_decode  = FEC_Decoder::onReceive per stream: erasure M host flags (1 = packet
 *                         missing), d_codeword M rows of CW bytes (zero padded; rows of missing
 *                         packets are not read) -> d_payload_out row m = the stream's packet seq-T
 *                         (seq = packets that stream had received before), d_payload_len m
 *                         (0 = lost or not available yet).
 * Asynchronous on hip_stream; ids must be distinct within a call (FEC_ERR_ARG otherwise). */
typedef struct fec_streams fec_streams;
int fec_streams_create(int max_payload, int T, int B, int N, int nstreams, fec_streams **out);
int fec_streams_destroy(fec_streams *group);
int fec_streams_encode(fec_streams *group, const int32_t *ids, int M, const uint8_t *d_payload,
                       const int32_t *d_payload_len, uint8_t *d_codeword, int32_t *d_codeword_len,
                       void *hip_stream);
int fec_streams_decode(fec_streams *group, const int32_t *ids, int M, const uint8_t *erasure,
                       const uint8_t *d_codeword, uint8_t *d_payload_out, int32_t *d_payload_len,
                       void *hip_stream);
/* Packets stream `id` has sent (encoded) and received (decoded) so far. */
int fec_streams_state(const fec_streams *group, int id, int64_t *sent, int64_t *received);

/* ---- per-kernel timing (HIP events recorded on the launch stream) --------------------------- */
#define FEC_KERNEL_ENCODE 0
#define FEC_KERNEL_DEC_SCAN 1
#define FEC_KERNEL_DEC_PLAN 2
#define FEC_KERNEL_DEC_COPY 3
#define FEC_KERNEL_DEC_RECOVER 4
#define FEC_KERNEL_COUNT 5
int fec_timing_enable(fec_codec *codec, int enable);
/* Synchronises the recorded events; total_ms[FEC_KERNEL_COUNT], launches[FEC_KERNEL_COUNT]. */
int fec_timing_collect(fec_codec *codec, double *total_ms, int64_t *launches);

/* Diagnostics: the next launches of `kernel` (FEC_KERNEL_ENCODE or FEC_KERNEL_DEC_COPY, the
 * specialised kernels) write s_memtime phase stamps, 8 uint64 per workgroup, to d_stamps
 * (NULL switches it off).  Timing-only; no output depends on it. */
int fec_debug_stamps(fec_codec *codec, int kernel, void *d_stamps);

/* ---- streaming per-packet API (host buffers) -----------------------------------------------
 * fec_encoder_transmit = FEC_Encoder::onTransmit: data (payload bytes), payload (<= max_payload),
 * seq (0,1,2,... consecutive); writes the wire codeword (cw_out must hold CW bytes; the trimmed
 * length goes to *codeword_size, bytes past it are zero).
 * fec_decoder_receive = FEC_Decoder::onReceive: codeword/codeword_size = wire bytes (ignored when
 * erasure != 0), seq consecutive from 0; writes packet seq-T's payload to payload_out
 * (max_payload bytes, zero beyond) and its length to *payload (0 = lost / not yet available).
 * Each call is one kernel launch (the stream-group kernels of fec_streams.hip on a one-stream
 * window / ring) reading and writing pinned, mapped host rows, and a poll of a completion word
 * (FEC_STREAM_SPIN=0: hipStreamSynchronize instead).  The encoder needs k = T-N+1 <= 16. */
int fec_encoder_create(int max_payload, int T, int B, int N, fec_encoder **out);
int fec_encoder_destroy(fec_encoder *enc);
int fec_encoder_transmit(fec_encoder *enc, const uint8_t *data, int payload, int seq,
                         uint8_t *cw_out, int *codeword_size);
int fec_decoder_create(int max_payload, int T, int B, int N, fec_decoder **out);
int fec_decoder_destroy(fec_decoder *dec);
int fec_decoder_receive(fec_decoder *dec, const uint8_t *codeword, int codeword_size, int seq,
                        int erasure, uint8_t *payload_out, int *payload);

/* ---- host-side planner probe (control plane only, no device needed) -------------------------
 * Runs the symbolic decoder over an erasure pattern of P packets and reports, for packets
 * 0..P-T-1, fate[x] (1 copy, 2 recovered, 3 lost).  Used by tests and by the streaming decoder. */
int fec_plan_host(int max_payload, int T, int B, int N, const uint8_t *erasure, int64_t P,
                  uint8_t *fate);

/* ---- block mode: many independent code blocks ------------------------------------------------
 * Batched forms of the reference's free functions as the relay (Decoder_Symbol_Wise,
 * src/Decoder_Symbol_Wise.cpp:322-328, 532-533, 573-575, 610, 643) calls them per code block:
 *   encodeBlock(data, G, cw, k, n, t = k-1)  (src/codingOperations.cpp:131-147): d_data nblk x k ->
 *     d_codeword nblk x n = [data, parity] (the relay pre-fills cw with the data, so the k-1
 *     systematic bytes encodeBlock leaves alone are the data too);
 *   decodeBlock(cw, G, cw, erasure, k, n, T = n-1, t = 0)  (src/codingOperations.cpp:149-232):
 *     d_codeword nblk x n + d_erasure nblk x n (1 = erased) -> d_out nblk x n with every data symbol
 *     the reference recovers written in, d_erasure_out (may be NULL) with those flags cleared.
 * G is the codec's generator (init_at_sender for its (T,B,N)). */
int fec_block_encode_batch(fec_codec *codec, const uint8_t *d_data, int64_t nblk, uint8_t *d_codeword,
                           void *hip_stream);
int fec_block_decode_batch(fec_codec *codec, const uint8_t *d_codeword, const uint8_t *d_erasure,
                           int64_t nblk, uint8_t *d_out, uint8_t *d_erasure_out, void *hip_stream);

/* ---- variable-rate (adaptive) coding: BASELINE config 4 --------------------------------------
 * The reference's P2P loop (application_local_simulation.cpp:328-345): Application_Layer_Sender +
 * Variable_Rate_FEC_Encoder (src/Variable_Rate_FEC_Encoder.cpp:74-235) with double coding at every
 * (T,B,N) switch, Application_Layer_Receiver + foreground/background Parameter_Estimator
 * (src/Parameter_Estimator.cpp:58-190, swapped every 100 packets) + Variable_Rate_FEC_Decoder
 * (src/Variable_Rate_FEC_Decoder.cpp:2133-2400), the receiver's 6-byte feedback read by the sender at
 * the next packet.  Everything but the coding bytes depends only on the erasure pattern, so a plan
 * runs the loop symbolically on the host and records the schedule; the byte work then runs batched
 * on the device.  T = T_INITIAL, B = N = -1 for adaptive (else fixed (T,B,N)); the pattern is the
 * receiver's erasure.bin (ERASURE_TYPE 5: packets seq < P+T with pattern byte 1 are dropped); P =
 * NUMBER_OF_ITERATIONS, the packets whose outputs are counted. */
typedef struct fec_vr_plan fec_vr_plan;
int fec_vr_plan_create(int max_payload, int T, int B, int N, int adaptive_mode_MDS,
                       const uint8_t *erasure, int64_t n_erasure, int64_t P, fec_vr_plan **out);
int fec_vr_plan_destroy(fec_vr_plan *plan);
/* Plan again, in place, with the plan's (max_payload, T, B, N, adaptive_mode_MDS) on a new pattern
 * and P: the host buffers, device tables and worker threads of the plan are reused.  async != 0:
 * returns after the serial control loop (instances, frames, sent, switches final); the symbolic
 * decoder instances run on worker threads meanwhile, so fec_vr_encode_batch's launch overlaps them;
 * every call that needs their results (stats, timing, packets, decode) waits for them. */
int fec_vr_plan_rerun(fec_vr_plan *plan, const uint8_t *erasure, int64_t n_erasure, int64_t P, int async);
/* lost: packets among 0..P-1 the receiver outputs empty ("Final FEC loss rate" x P); switches:
 * "Start double coding at the source" count; coding_rate: Variable_Rate_FEC_Encoder's final rate;
 * sent: packets the sender produced; cw_max: the widest codeword row (16-byte multiple). */
int fec_vr_plan_stats(const fec_vr_plan *plan, int64_t *lost, int64_t *switches, double *coding_rate,
                      int64_t *sent, int *n_encoders, int *n_decoders, int *cw_max);
/* wall time of the plan's two phases: the serial control loop (sender, estimators, switches,
 * decoder swaps) and the parallel symbolic decoder instances, in ms */
int fec_vr_plan_timing(const fec_vr_plan *plan, double *control_ms, double *decoders_ms);
/* the control loop's time waiting for the estimator feedback jobs (which run on the plan's worker
 * threads, ahead of its decoder jobs) in the last run */
int fec_vr_plan_feedback_wait(const fec_vr_plan *plan, double *waited_ms);
/* instances, 6 int64 each: T, B, N, first seq, seq from which it is the old one, end seq */
int fec_vr_plan_instances(const fec_vr_plan *plan, int64_t *encoders, int64_t *decoders);
/* per sent packet: frames (6 int32: header T, B, N, counter_for_start_and_end, current encoder,
 * old encoder or -1), erased (1 = dropped); per counted packet x < P: fate (1 received, 2
 * recovered, 3 lost) and the decoder instance that reported it.  NULL pointers are skipped. */
int fec_vr_plan_packets(const fec_vr_plan *plan, int32_t *frames, uint8_t *erased, uint8_t *fate,
                        int32_t *fate_decoder);
/* Device-resident execution.  The frames' codewords live in two compact arrays (no per-row padding
 * beyond 16-byte alignment): row s of d_cw_cur = the codeword of frame s's current encoder, row s
 * of d_cw_old = the old encoder's during double coding (empty otherwise); each row is its
 * instance's CW rounded up to 16 bytes, rows in seq order.  fec_vr_plan_layout gives the two array
 * sizes, fec_vr_plan_row_offsets the per-row byte offsets (sent + 1 each, prefix form).  Encode:
 * d_payload (sent rows of max_payload bytes) -> d_cw_cur / d_cw_old rows, trimmed sizes in
 * d_len_cur / d_len_old (sent each; 0 when no old codeword).  Decode: those arrays + d_erased
 * (sent bytes) -> d_out (P rows of max_payload) and d_out_len (P ints, 0 = lost), the receiver's
 * reported outputs. */
int fec_vr_plan_layout(const fec_vr_plan *plan, int64_t *cur_bytes, int64_t *old_bytes);
int fec_vr_plan_row_offsets(const fec_vr_plan *plan, int64_t *cur_off, int64_t *old_off);
int fec_vr_encode_batch(fec_vr_plan *plan, const uint8_t *d_payload, const int32_t *d_payload_len,
                        uint8_t *d_cw_cur, int32_t *d_len_cur, uint8_t *d_cw_old, int32_t *d_len_old,
                        void *hip_stream);
int fec_vr_decode_batch(fec_vr_plan *plan, const uint8_t *d_cw_cur, const uint8_t *d_cw_old,
                        const uint8_t *d_erased, uint8_t *d_out, int32_t *d_out_len, void *hip_stream);
/* Wire framing above the boundary.  Sender: row s of d_packets (stride >= 10 + 2*cw_max) = the P2P
 * packet Application_Layer_Sender sends (Application_Layer_Sender.cpp:259-269): [seq BE32][T][B][N]
 * [counter_for_start_and_end] + Variable_Rate_FEC_Encoder's frame (Variable_Rate_FEC_Encoder.cpp:
 * 194-217): [size_current BE16][codeword_current (trimmed)][codeword_old (trimmed)]; sizes in
 * d_packet_len.  Receiver: the split of the plan's sent packets into the current / old codeword
 * rows of the compact arrays, zero-padded to their row size (Application_Layer_Receiver.cpp:361-366,
 * Variable_Rate_FEC_Decoder.cpp:2156-2160), header fields to d_header (sent x 5 int32: seq, T, B,
 * N, counter; may be NULL). */
int fec_vr_frames_batch(fec_vr_plan *plan, const uint8_t *d_cw_cur, const int32_t *d_len_cur,
                        const uint8_t *d_cw_old, const int32_t *d_len_old, uint8_t *d_packets,
                        int64_t stride, int32_t *d_packet_len, void *hip_stream);
int fec_vr_parse_batch(fec_vr_plan *plan, const uint8_t *d_packets, int64_t stride, const int32_t *d_packet_len,
                       uint8_t *d_cw_cur, uint8_t *d_cw_old, int32_t *d_header, void *hip_stream);

/* ---- relay: symbol-wise decode-and-forward (SWDF, RELAYING_TYPE 2) ---------------------------
 * Decoder_Symbol_Wise (src/Decoder_Symbol_Wise.cpp) as the relay and the destination drive it
 * (src/Variable_Rate_FEC_Decoder.cpp:950-1601 relay, :1603-1879 destination; one relay frame per
 * seq as with FLAG_FOR_CONSTANT_TRANS = 1, application_local_simulation.cpp:532-587), fixed rate.
 * Hop 1 carries the source's FEC_Encoder(max_payload, T1, N1, N1) codewords; the relay decodes
 * with window n1 = T1+1 and re-encodes for n2 = T2+1 with k = T1-N1+1 = T2-N2+1 (k2 == k, the
 * only case the reference handles).  Batches run a fresh relay / destination over seqs 0..P-1.
 *   fec_swdf_relay_batch: d_cw P rows of cw_stride bytes (the source codewords, zero-padded to at
 *     least S*n1 bytes; rows of erased packets are never read), d_erasure P hop-1 flags ->
 *     d_frames P rows of frame_bytes (the relay's transmitted frame: [size BE16][codeword_new_vector
 *     [n2-1][0..size)], size = (S+1)*n2), d_flag P bytes (may be NULL): 1 when the window held too
 *     many erasures to decode (the relay's loss counter).  d_work: fec_swdf_workspace_bytes(P).
 *   fec_swdf_destination_batch: d_frames + d_erasure P hop-2 flags -> d_out P rows of S*k bytes:
 *     row t = data_with_header ([len BE16][payload][zero pad]) of source packet t - delay, as
 *     symbol_wise_decode_1 + extract_data produce it; d_flag as above (may be NULL). */
typedef struct fec_swdf fec_swdf;
int fec_swdf_create(int max_payload, int T1, int N1, int T2, int N2, fec_swdf **out);
int fec_swdf_destroy(fec_swdf *swdf);
/* delay = n1 + n2 - k - 1: destination row t carries source packet t - delay */
int fec_swdf_geometry(const fec_swdf *swdf, int *k, int *n1, int *n2, int *S, int *frame_bytes,
                      int *delay);
size_t fec_swdf_workspace_bytes(const fec_swdf *swdf, int64_t P);
int fec_swdf_relay_batch(fec_swdf *swdf, const uint8_t *d_cw, int64_t cw_stride, const uint8_t *d_erasure,
                         int64_t P, uint8_t *d_frames, uint8_t *d_flag, void *d_work, size_t work_bytes,
                         void *hip_stream);
int fec_swdf_destination_batch(fec_swdf *swdf, const uint8_t *d_frames, const uint8_t *d_erasure, int64_t P,
                               uint8_t *d_out, uint8_t *d_flag, void *hip_stream);

/* ---- relay: state-dependent symbol-wise decode-and-forward (SD-SWDF, RELAYING_TYPE 3) --------
 * Decoder_Symbol_Wise::symbol_wise_encode_state_dependent (src/Decoder_Symbol_Wise.cpp:178-432) at
 * the relay and symbol_wise_decode_state_dependent + extract_data (:487-546, :653-661) at the
 * destination, as Variable_Rate_FEC_Decoder drives them with one relay frame per seq
 * (src/Variable_Rate_FEC_Decoder.cpp:636-675, 1458-1493 relay; :1703-1721, 1798-1815 destination),
 * fixed rate, k = T1-N1+1 = T2-N2+1, T2 <= T1 <= T_TOT = 10; sdbo = FLAG_FOR_SDBO (FEC_Macro.h:50
 * ships 0).  The control flow depends only on erasure flags and headers: a host planner replays it
 * per packet (serial, like the reference) and the GPU applies the per-packet plans to the bytes.
 * A batch runs a fresh relay / destination over seqs 0..P-1; both calls return when done.
 *   fec_sdswdf_relay_batch: d_cw P rows of cw_stride bytes (source codewords zero-padded to >= S*n1;
 *     erased rows are never read), h_erasure P hop-1 flags (host) -> d_frames P rows of frame_bytes:
 *     [size BE16][header 11 bytes][codeword_new_vector[n2-1][0..size)], size = (S+1)*n2.
 *   fec_sdswdf_destination_batch: d_frames (rows of frame_bytes; the 11 header bytes of every
 *     received frame steer the decode), h_erasure P hop-2 flags (host) -> d_out P rows of S*k
 *     bytes: row t = data_with_header of source packet t - delay (blocks*k decoded, rest zero);
 *     h_flag (host, may be NULL): 1 when a diagonal had too many erasures (the loss counter).
 *   fec_sdswdf_relay_plan / fec_sdswdf_dest_plan: the host plans alone (tests): per seq a record id,
 *     and the distinct records: relay = header[11] + n2 rows of n1 coefficients (frame symbol i of
 *     block j = sum_p coef[i][p] * symbol (j, p) of source packet t-(n1-1)+p+(k-1-i)); destination
 *     = k rows of n2 coefficients (data symbol s of block j = sum_q coef[s][q] * frame symbol
 *     (j, q) of frame t-s-(n2-1-q)). */
typedef struct fec_sdswdf fec_sdswdf;
int fec_sdswdf_create(int max_payload, int T1, int N1, int T2, int N2, int sdbo, fec_sdswdf **out);
int fec_sdswdf_destroy(fec_sdswdf *w);
/* Host-only (no device call): whether a type-3 batch of this geometry runs on the tile kernel
 * (1) or the per-(packet, block) kernel (0), the tile's packets and its dynamic LDS bytes; stride <=
 * 0 = the default row pitch (relay: S*n1, destination: the frame bytes). */
int fec_sdswdf_tile_geometry(int relay, int max_payload, int T1, int N1, int T2, int N2, int64_t stride,
                             int *tile_packets, int *lds_bytes);
int fec_sdswdf_geometry(const fec_sdswdf *w, int *k, int *n1, int *n2, int *S, int *blocks,
                        int *frame_bytes, int *delay);
int fec_sdswdf_relay_batch(fec_sdswdf *w, const uint8_t *d_cw, int64_t cw_stride, const uint8_t *h_erasure,
                           int64_t P, uint8_t *d_frames, void *hip_stream);
int fec_sdswdf_destination_batch(fec_sdswdf *w, const uint8_t *d_frames, const uint8_t *h_erasure, int64_t P,
                                 uint8_t *d_out, uint8_t *h_flag, void *hip_stream);
/* The same over several independent streams laid end to end (fec_relay_vr): a fresh relay /
 * destination takes over at each row of h_starts (sorted); the rows in front of a start that its
 * plans reach must be zero codewords / frames on received (0) flags, as before a stream's seq 0. */
int fec_sdswdf_relay_batch_starts(fec_sdswdf *w, const uint8_t *d_cw, int64_t cw_stride, const uint8_t *h_erasure,
                                  int64_t P, const int64_t *h_starts, int nstarts, uint8_t *d_frames,
                                  void *hip_stream);
int fec_sdswdf_destination_batch_starts(fec_sdswdf *w, const uint8_t *d_frames, const uint8_t *h_erasure,
                                        int64_t P, const int64_t *h_starts, int nstarts, uint8_t *d_out,
                                        uint8_t *h_flag, void *hip_stream);
int fec_sdswdf_relay_plan(fec_sdswdf *w, const uint8_t *h_erasure, int64_t P, int32_t *h_plan,
                          uint8_t *h_records, int64_t records_cap, int64_t *n_records, int *record_bytes);
int fec_sdswdf_dest_plan(fec_sdswdf *w, const uint8_t *h_erasure, const uint8_t *h_headers, int64_t P,
                         int32_t *h_plan, uint8_t *h_flag, uint8_t *h_records, int64_t records_cap,
                         int64_t *n_records, int *record_bytes);

/* ---- relay under variable rate: RELAYING_TYPE 2 / 3 through code switches ---------------------
 * The relay chain of Variable_Rate_FEC_Decoder under a schedule of source codes (:600-740 relay,
 * :1423-1600 and :1772-1873 destination): at a switch to (T, N) at seq s the relay and the
 * destination create fresh Decoder_Symbol_Wise objects for it; for the T_TOT + 1 double-coded seqs
 * s .. s + T_TOT (Variable_Rate_FEC_Encoder.cpp:74-235) the old objects take the old code's
 * codewords and the new ones the new code's, the relay sends [BE16 size_cur][new part][old part]
 * (part = [header 11 bytes, type 3][codeword_new_vector row of size = (S+1)*n2 bytes]), the
 * destination's old object reports; at s + T_TOT + 1 the new objects take over (copy_elements).
 * Hop 1 carries FEC_Encoder(max_payload, T, N, N) codewords, hop 2 the relay's (T, N) re-encoding
 * (T2 = T: the relay-mode estimator fixes T = T_TOT, Parameter_Estimator.cpp:72-75).
 *   fec_relay_vr_create: type 2 or 3; sched = nsw entries (seq, T, N), the first at seq 0, each at
 *     least T_TOT + 1 = 11 after the previous, 1 <= T <= 10, N <= T; P seqs.
 *   fec_relay_vr_run: d_payload P rows of max_payload bytes (source packet t), h_e1 / h_e2 P hop-1 /
 *     hop-2 erasure flags (host) -> d_frames P rows of frame_stride bytes and d_frame_len P sizes
 *     (the relay's frame per seq), d_out P rows of out_stride bytes (what the reporting destination
 *     object's extract_data wrote at seq t: blocks*k bytes of its code, zero after), h_flag P (host,
 *     may be NULL): the reporting object's loss flag.  Returns when done. */
typedef struct fec_relay_vr fec_relay_vr;
int fec_relay_vr_create(int type, int max_payload, const int32_t *sched, int nsw, int64_t P, fec_relay_vr **out);
int fec_relay_vr_destroy(fec_relay_vr *r);
int fec_relay_vr_geometry(const fec_relay_vr *r, int *frame_stride, int *out_stride, int *codes);
int fec_relay_vr_run(fec_relay_vr *r, const uint8_t *d_payload, const uint8_t *h_e1, const uint8_t *h_e2,
                     uint8_t *d_frames, int32_t *d_frame_len, uint8_t *d_out, uint8_t *h_flag, void *hip_stream);

/* ---- the two-hop adaptive relay session (RELAYING_TYPE 2 / 3, N_INITIAL = N_INITIAL_2 = -1) -------
 * application_local_simulation.cpp:71-593 with FLAG_FOR_CONSTANT_TRANS = 1, replacing the loop of
 * Application_Layer_Sender::generate_message_and_encode (:64-282: the 12-byte feedback, the split
 * T = T_TOT - N2, T2 = T_TOT - N), Variable_Rate_FEC_Encoder::encode in relay mode
 * (Variable_Rate_FEC_Encoder.cpp:74-235), Application_Layer_Receiver::receive_message_and_symbol_
 * wise_encode / _decode (Application_Layer_Receiver.cpp:56-319, the relay-mode estimators,
 * Parameter_Estimator.cpp:72-75), Variable_Rate_FEC_Decoder's relay and destination paths
 * (Variable_Rate_FEC_Decoder.cpp:542-1879) and send_sym_wise_message (Application_Layer_Sender.cpp:
 * 284-346).  The control flow runs on the host at create (it depends on the hop erasure patterns
 * only); run does the byte work of the whole session on the GPU.
 *   fec_relay_session_create: relay_type 2 or 3, Q seqs (the reference's loop runs to seq
 *     NUMBER_OF_ITERATIONS + T_TOT + T2 - 1), hop patterns e1 / e2 (received past their end; e1[0]
 *     must be 0).
 *   fec_relay_session_info: stats[16] = {Q, relay_bytes, source switches, relay switches,
 *     destination switches, destination flags, relay calls, lineages, destination outputs,
 *     processed seqs, symbol bytes, encoder instances, longest lineage, relay flags, rate1 count,
 *     rate2 count}; rates[4] = {sum of first-hop rates, of second-hop rates, of min rates, control
 *     plane ms} (the reference's float sums, in its order).
 *   fec_relay_session_relay_offsets: off[Q+1], relay packet t at d_relay[off[t], off[t+1]).
 *   fec_relay_session_hop1_headers: hdr[Q][16], the source's packet headers (:222-244).
 *   fec_relay_session_dest_meta: proc[Q] (1 = the destination's main object extracted an output at
 *     seq t), flag[Q] (its decode flag).
 *   fec_relay_session_run: d_payload Q rows of max_payload bytes (source packet t) -> d_relay
 *     (relay_bytes: every relay packet, 8-byte header + word), d_dest_out Q rows of 320 bytes (the
 *     extracted data_with_header of packet t - T_TOT, zero where not processed), d_dest_lost Q
 *     (calc_missed_chars, Variable_Rate_FEC_Decoder.cpp:2698-2792), *d_lost their count; async on
 *     the stream.
 *   fec_relay_session_hop1: after a run, the source's wire packets (16-byte header + VR frame) at
 *     `stride`, zero padded, sizes in d_len. */
typedef struct fec_relay_session fec_relay_session;
int fec_relay_session_create(int relay_type, int max_payload, int64_t Q, const uint8_t *e1, int64_t n_e1,
                             const uint8_t *e2, int64_t n_e2, fec_relay_session **out);
int fec_relay_session_destroy(fec_relay_session *h);
int fec_relay_session_info(const fec_relay_session *h, int64_t *stats, double *rates);
int fec_relay_session_relay_offsets(const fec_relay_session *h, int64_t *off);
int fec_relay_session_hop1_headers(const fec_relay_session *h, uint8_t *hdr);
int fec_relay_session_dest_meta(const fec_relay_session *h, uint8_t *proc, uint8_t *flag);
int fec_relay_session_run(fec_relay_session *h, const uint8_t *d_payload, uint8_t *d_relay, uint8_t *d_dest_out,
                          uint8_t *d_dest_lost, int64_t *d_lost, void *hip_stream);
int fec_relay_session_hop1(fec_relay_session *h, uint8_t *d_packets, int64_t stride, int32_t *d_len,
                           void *hip_stream);

/* ---- relay per call: the Decoder_Symbol_Wise methods on caller-held state ---------------------
 * What siphon::Decoder_Symbol_Wise (fec_amd_dropin.h) calls: one reference method call each, on
 * the arrays the reference's callers fill (Variable_Rate_FEC_Decoder.cpp:950-1879).  The control
 * flow runs on the host over the flags and headers; the GF work of all the packet's code blocks is
 * one GPU launch (its inputs packed into pinned staging, results back), then the call returns.
 *   fec_sw_state_encode  = symbol_wise_encode_state_dependent (Decoder_Symbol_Wise.cpp:178-432):
 *     slots = codeword_vector_state_dependent [30] (packet at offset 2), er = its flags [30],
 *     header [30] rows of 11 ints (row n2-1 written), cnv = codeword_new_vector[n2-1], cnsw =
 *     codeword_new_symbol_wise;
 *   fec_sw_state_decode  = symbol_wise_decode_state_dependent (:487-546) into buffer, *flag;
 *   fec_sw_encode_1      = symbol_wise_encode_1 (:547-619): cv = codeword_vector [T_TOT+1], er =
 *     temp_erasure_vector, cnv = codeword_new_vector [T_TOT+1] (row n2-1 written);
 *   fec_sw_decode_1      = symbol_wise_decode_1 (:621-651) into buffer, *flag.
 * k2 == k; n <= 11 (types 3) / n <= 17 (type 2); sdbo = FLAG_FOR_SDBO. */
int fec_sw_state_encode(int max_payload, int k, int n, int k2, int n2, int sdbo, uint8_t *const *slots,
                        const uint8_t *er, int *const *header, uint8_t *cnv, uint8_t *cnsw);
int fec_sw_state_decode(int max_payload, int k, int n, uint8_t *const *slots, int *const *header, uint8_t *buffer,
                        int *flag);
int fec_sw_encode_1(int max_payload, int k, int n, int k2, int n2, uint8_t *const *cv, const uint8_t *er,
                    uint8_t *const *cnv, uint8_t *cnsw, int *flag);
int fec_sw_decode_1(int max_payload, int k, int n, uint8_t *const *cv, const uint8_t *er, uint8_t *buffer,
                    int *flag);

/* ---- erasure patterns (inputs of the decode path; host only, no device needed) ---------------
 * Byte-exact restatements of Erasure_File_Generator (src/Erasure_File_Generator.cpp:25-287): out[i]
 * = 1 if packet i is erased.  Same engine (mt19937), same draw order and the same libstdc++
 * uniform_real_distribution<double> arithmetic as the reference; probabilities are float as in
 * its signatures.  The reference writes these bytes to erasure.bin (read back by
 * Erasure_Simulator, src/Erasure_Simulator.cpp:13-30). */
/* generate_IID (:25-63); seed 0 = SEED_ARTIFICIAL_ERASURE */
int fec_erasure_iid(uint8_t *out, int count, float erasure_prob, int seed);
/* generate_three_sections_IID (:65-121) */
int fec_erasure_three_sections_iid(uint8_t *out, int count1, float prob1, int count2, float prob2,
                                   int count3, float prob3, int seed);
/* generate_GE (:123-170) / generate_GE_varying (:172-213); good_state: the generator object's
 * state carried across calls (in/out, NULL = a fresh object, i.e. good) */
int fec_erasure_ge(uint8_t *out, int count, float alpha, float beta, float erasure_prob, int seed,
                   int *good_state);
int fec_erasure_ge_varying(uint8_t *out, int count, float alpha, float beta, float erasure_prob,
                           int seed, int *good_state);
/* generate_Fritchman_varying (:215-264) */
int fec_erasure_fritchman_varying(uint8_t *out, int count, float alpha, float beta,
                                  float erasure_prob, int number_of_states, int seed);
/* generate_periodic (:266-287) */
int fec_erasure_periodic(uint8_t *out, int count, int T, int B, int N);

/* ---- utility (tests / bench only, not on the coding path) ---------------------------------
 * Synthetic payloads: byte b of packet t0+p = low 8 bits of splitmix64(seed ^ ((t0+p)*L + b)). */
int fec_util_fill_payload(uint8_t *d_out, int64_t t0, int64_t count, int L, uint64_t seed,
                          void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif
