/*
 * oracle/fec_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the reference's GF(2^8) streaming-erasure hot path
 * (domanovi/FEC_Erasure_Code_Unit_Test_Relay, src/basicOperations.cpp,
 * src/codingOperations.cpp, src/Encoder*.cpp, src/Decoder*.cpp, src/FEC_Encoder.cpp,
 * src/FEC_Decoder.cpp) plus the five ISA-L 2.23 functions it links.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * See fec_oracle.c for the pinning status.
 */
#ifndef FEC_ORACLE_H
#define FEC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ISA-L restatement (erasure_code/ec_base.c, ISA-L 2.23.0; include/isal.h:10-12). */
uint8_t or_gf_mul(uint8_t a, uint8_t b);
uint8_t or_gf_inv(uint8_t a);
void or_gf_gen_cauchy1_matrix(uint8_t *a, int m, int k);
void or_gf_gen_rs_matrix(uint8_t *a, int m, int k);

/* codingOperations.cpp / basicOperations.cpp restatements. */
void or_gen_G(uint8_t *G, int T, int B, int N, int k, int n);
void or_encode_block(const uint8_t *data, const uint8_t *G, uint8_t *cw, int k, int n, int t);
void or_rref_matrix(const uint8_t *in, uint8_t *out, uint8_t *action, int m, int n);
void or_decode_block(uint8_t *data, const uint8_t *G, uint8_t *cw, uint8_t *erasure, int k, int n,
                     int T, int t);

/* Geometry helper: fills k, n, S (= number of sub-streams), CW (= untrimmed codeword bytes). */
void or_geometry(int max_payload, int T, int B, int N, int *k, int *n, int *S, int *CW);

/* FEC_Encoder (src/FEC_Encoder.cpp:22-68) over a reference-structured encoder. */
typedef struct or_encoder or_encoder;
or_encoder *or_encoder_new(int max_payload, int T, int B, int N);
void or_encoder_free(or_encoder *e);
/* Writes the untrimmed CW-byte codeword to cw_out; returns the trimmed wire size. */
int or_encoder_transmit(or_encoder *e, const uint8_t *data, int payload, int seq, uint8_t *cw_out);

/* FEC_Decoder (src/FEC_Decoder.cpp:26-72) over a reference-structured decoder.
 * loss_only != 0 runs only the sub-streams that decide the packet's fate (sub-stream 0, and 1 when
 * k == 1); the returned payload is then only meaningful as zero/non-zero. */
typedef struct or_decoder or_decoder;
or_decoder *or_decoder_new(int max_payload, int T, int B, int N, int loss_only);
void or_decoder_free(or_decoder *d);
/* Returns the payload length of packet seq-T (0 = lost / not yet available); copies the
 * payload bytes (max_payload bytes, zero beyond the payload) to out when out != NULL. */
int or_decoder_receive(or_decoder *d, const uint8_t *cw, int cw_size, int seq, int erasure,
                       uint8_t *out);

/* Synthetic payload generator shared by the oracle harness, the tests and bench.py:
 * byte b of packet t = low 8 bits of splitmix64(seed ^ (t * L + b)). */
void or_fill_payload(uint8_t *buf, int64_t t0, int64_t count, int L, uint64_t seed);

/* Whole-stream harness.  Feeds seq 0 .. P+T-1 (erasure of seq t = pattern[t] for t < pattern_len,
 * else 0) through FEC_Encoder -> FEC_Decoder, and returns the payload length recovered for packets
 * 0 .. P-1 in out_len (P ints).  When out_data != NULL (P*max_payload bytes) the recovered payload
 * bytes are stored too; cw_out (optional, (P+T)*CW bytes) receives the untrimmed codewords and
 * cw_len (optional, P+T ints) the trimmed wire sizes. Returns the number of lost packets. */
int64_t or_run_stream(int max_payload, int T, int B, int N, int64_t P, const uint8_t *pattern,
                      int64_t pattern_len, uint64_t seed, int loss_only, int *out_len,
                      uint8_t *out_data, uint8_t *cw_out, int *cw_len);

/* Encode-only harness (timed as the CPU baseline): P packets from seq0, returns total wire bytes. */
int64_t or_encode_stream(int max_payload, int T, int B, int N, int64_t seq0, int64_t P,
                         uint64_t seed, uint8_t *cw_out, int *cw_len);

/* Decoder_Symbol_Wise (src/Decoder_Symbol_Wise.cpp): relay SWDF and destination symbol-wise
 * decode, reference-structured (see fec_oracle.c for the defined-away undefined behaviour). */
typedef struct or_swdf or_swdf;
or_swdf *or_swdf_new(int max_payload, int k, int n, int n2);
void or_swdf_free(or_swdf *s);
void or_swdf_push(or_swdf *s, const uint8_t *message, int size, int n, int n2);
void or_swdf_rotate(or_swdf *s, int n, int n2);
int or_swdf_encode_1(or_swdf *s);
int or_swdf_frame(const or_swdf *s, uint8_t *frame);
int or_swdf_decode_1(or_swdf *s, uint8_t *out);
int or_swdf_run(int max_payload, int T1, int N1, int T2, int N2, int64_t P, const uint8_t *e1,
                const uint8_t *e2, uint64_t seed, uint8_t *frames, uint8_t *relay_flag,
                uint8_t *dest_out, uint8_t *dest_flag);

/* Decoder_Symbol_Wise state-dependent relay (SD-SWDF, RELAYING_TYPE 3; Decoder_Symbol_Wise.cpp
 * :178-546), reference-structured, and its fixed-rate chain (see fec_oracle.c). */
typedef struct or_sdswdf or_sdswdf;
or_sdswdf *or_sdswdf_new(int max_payload, int k, int n, int n2);
void or_sdswdf_free(or_sdswdf *s);
void or_sdswdf_set_garbage(int v);
void or_sdswdf_relay_push(or_sdswdf *s, const uint8_t *cw, int size, int erased);
void or_sdswdf_dest_push(or_sdswdf *s, const uint8_t *frame, int frame_bytes, int erased);
void or_sdswdf_encode(or_sdswdf *s, int sdbo);
int or_sdswdf_frame(const or_sdswdf *s, uint8_t *frame);
int or_sdswdf_decode(or_sdswdf *s, uint8_t *out);
int or_sdswdf_run(int max_payload, int T1, int N1, int T2, int N2, int64_t P, const uint8_t *e1,
                  const uint8_t *e2, uint64_t seed, int sdbo, uint8_t *frames, uint8_t *dest_out,
                  uint8_t *dest_flag);

/* The four Decoder_Symbol_Wise methods over the caller's arrays (the member layout of
 * include/Decoder_Symbol_Wise.h), with the signatures of the product's per-call C ABI (fec_sw_* in
 * include/fec_amd.h), so that a relay driver can run over either. */
int or_sw_state_encode(int max_payload, int k, int n, int k2, int n2, int sdbo, uint8_t *const *slots,
                       const uint8_t *er, int *const *header, uint8_t *cnv, uint8_t *cnsw);
int or_sw_state_decode(int max_payload, int k, int n, uint8_t *const *slots, int *const *header, uint8_t *buffer,
                       int *flag);
int or_sw_encode_1(int max_payload, int k, int n, int k2, int n2, uint8_t *const *cv, const uint8_t *er,
                   uint8_t *const *cnv, uint8_t *cnsw, int *flag);
int or_sw_decode_1(int max_payload, int k, int n, uint8_t *const *cv, const uint8_t *er, uint8_t *buffer,
                   int *flag);

/* The adaptive P2P loop (BASELINE config 4), reference-structured on real bytes: returns the
 * packets lost among 0..P-1; out_len[P] (0 = lost), out_data (P*max_payload or NULL); packets
 * (packets_cap bytes, or NULL) receives the first max_sent P2P wire packets [seq BE32][T][B][N]
 * [counter][size_current BE16][codeword_current][codeword_old] back to back, packet_off
 * (max_sent + 1 entries, or NULL) their offsets; stats = {lost, switches, sent}. */
int64_t or_vr_run(int max_payload, int T, int B, int N, int mds, const uint8_t *pattern, int64_t n_pattern,
                  int64_t P, uint64_t seed, int *out_len, uint8_t *out_data, uint8_t *packets,
                  int64_t packets_cap, int64_t *packet_off, int64_t max_sent, int64_t *stats, double *coding_rate);

/* The two-hop adaptive relay session (RELAYING_TYPE 2 / 3, application_local_simulation.cpp:71-593
 * with FLAG_FOR_CONSTANT_TRANS = 1): Q seqs, hop erasure patterns e1 / e2 (received past their
 * end), payloads or_fill_payload(seed).  Per-seq outputs (each array optional, Q entries):
 * hop1_len / hop1_hdr[16] = the source's packet (16-byte header + VR frame); relay_len /
 * relay_hdr[8] = the relay's packet to the destination (8-byte header + stored word);
 * dest_proc = 1 when the destination's main object extracted an output at seq t (a received
 * frame, or a missing seq before one), dest_flag its decode flag, dest_lost = calc_missed_chars'
 * verdict on packet t - T_TOT, dest_out [Q][OR_SESSION_DW] = the extracted blocks*k bytes (zero
 * beyond).  crc[ceil(Q/OR_SESSION_BLOCK)]: per block of seqs the CRC-32 of every seq's [hop-1
 * len LE32][hop-1 packet][relay len LE32][relay packet]; crc2 (needs dest_out, dest_proc): of
 * [proc][flag][lost][dest_out row].  Returns 0, -2 when hop-1 seq 0 is erased, -3 / -4 when a
 * relay / destination call has no restatement (status_seq = the loop index). */
#define OR_SESSION_DW 320
#define OR_SESSION_BLOCK 100
typedef struct {
    int64_t Q;
    int32_t *hop1_len;
    uint8_t *hop1_hdr;
    int32_t *relay_len;
    uint8_t *relay_hdr;
    uint8_t *dest_proc, *dest_flag, *dest_lost, *dest_out;
    uint32_t *crc, *crc2;
    uint8_t *hop1_pkts, *relay_pkts; /* optional: every packet at these strides (bytes past it zero) */
    int64_t hop1_stride, relay_stride;
    int64_t lost, src_switches, relay_switches, dest_switches, relay_flags, dest_flags, status_seq;
    float rate1, rate2, min_rate;
    int64_t rate1_n, rate2_n, min_rate_n;
} or_session_out;
int or_relay_session_run(int relay_type, int max_payload, int64_t Q, const uint8_t *e1, int64_t n_e1,
                         const uint8_t *e2, int64_t n_e2, uint64_t seed, or_session_out *o);

#ifdef __cplusplus
}
#endif
#endif
