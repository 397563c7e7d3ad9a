/*
 * mp3_oracle.h -- CPU restatement of llehouerou/go-mp3 (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle for the MI355X path, NOT product code: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker / the timed CPU baseline.  The product
 * (libmp3g.so) never links or calls it.
 *
 * Semantics follow the reference as compiled by gc for linux/amd64 with
 * GOAMD64=v1: every float32 +,-,* rounded individually (no FMA contraction;
 * build with -ffp-contract=off), requantization in float64, int(float32)
 * truncation.  See SURVEY.md Appendix A/B.
 *
 * Parity status: the reference's own tests pin NO PCM sample values
 * (SURVEY.md 8c); PCM parity of this restatement is "unpinned" except through
 * the properties the reference tests assert (PCM lengths, silence, durations,
 * seek repeatability, bit-reader / header KATs) plus the table-margin proofs
 * and the independent float64 spec-formula check in tests/.
 */
#ifndef MP3_ORACLE_H
#define MP3_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/mp3g.h"

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (mirror the Go error classes that decode.go distinguishes) */
#define ORC_OK 0
#define ORC_EOF 1            /* io.EOF (incl. mapped UnexpectedEOF / sync limit) */
#define ORC_ERR 2            /* any other error returned by the reference       */
#define ORC_ERR_PANIC 3      /* input on which the reference panics (not decodable) */

typedef struct orc_decoder orc_decoder;

/* mp3.NewDecoder(bytes.NewReader(data)) (decode.go:361-388); seekable=0 wraps
 * the reader so it is not an io.Seeker (time_seek_test.go:45-52). */
int orc_decoder_new(const uint8_t* data, size_t len, int seekable, orc_decoder** out);
void orc_decoder_free(orc_decoder* d);
/* Decoder.Read (decode.go:70-80): returns ORC_OK with *n >= 1, or ORC_EOF/ORC_ERR. */
int orc_decoder_read(orc_decoder* d, uint8_t* buf, size_t cap, size_t* n);
/* Decoder.Seek (decode.go:89-145). */
int orc_decoder_seek(orc_decoder* d, int64_t offset, int whence, int64_t* newpos);
int orc_decoder_sample_rate(const orc_decoder* d);
int64_t orc_decoder_length(const orc_decoder* d);
int64_t orc_decoder_bytes_per_frame(const orc_decoder* d);
int64_t orc_decoder_pos(const orc_decoder* d);
int64_t orc_decoder_n_frames(const orc_decoder* d);
/* time API in nanoseconds (decode.go:234-354) */
int64_t orc_decoder_duration_ns(const orc_decoder* d);
int64_t orc_decoder_position_ns(const orc_decoder* d);
int orc_decoder_seek_to_time_ns(orc_decoder* d, int64_t t);
int orc_decoder_seek_to_sample(orc_decoder* d, int64_t s);
/* Capture: while enabled, every frame parsed by this decoder appends its
 * boundary input (granule descriptors + int16 coefficients) before Decode
 * runs.  Retrieve with orc_decoder_captured(). */
void orc_decoder_capture(orc_decoder* d, int enable);
size_t orc_decoder_captured(const orc_decoder* d, const mp3g_granule** g, const int16_t** coef);

/* Convenience: NewDecoder + io.ReadAll.  *pcm is malloc'd (free with orc_free). */
int orc_decode_all(const uint8_t* data, size_t len, uint8_t** pcm, size_t* pcm_len);
/* Same, additionally returning the captured boundary input of every frame. */
int orc_decode_all_capture(const uint8_t* data, size_t len, uint8_t** pcm, size_t* pcm_len,
                           mp3g_granule** granules, int16_t** coeffs, size_t* n_granules);
void orc_free(void* p);

/* DSP only (Frame.Decode restated per granule, frame.go:121-688):
 * decode n granules of one stream in order starting from *state (mutated). */
void orc_dsp_granules(const mp3g_granule* g, const int16_t* coef, size_t n, mp3g_state* state,
                      int16_t* pcm);
/* Batched form with the exact semantics of mp3g_decode_host (streams, flags). */
int orc_dsp_streams(const mp3g_granule* g, const int16_t* coef, const mp3g_stream* streams,
                    uint32_t n_streams, const mp3g_state* state_in, mp3g_state* state_out,
                    int16_t* pcm);
/* Stages before the polyphase (requantize .. frequency inversion) only:
 * float32 lines [n][2][576] as subbandSynthesis reads them (test inputs). */
void orc_hybrid_streams(const mp3g_granule* g, const int16_t* coef, const mp3g_stream* streams,
                        uint32_t n_streams, const mp3g_state* state_in, float* is_out);
/* The stateless front end only (requantize, reorder, stereo, antialias;
 * frame.go:140-452): the float32 lines the IMDCT reads, [n][2][576]
 * (mono: [g][1][*] = 0).  Test / analysis input (magnitude thresholds). */
void orc_frontend_granules(const mp3g_granule* g, const int16_t* coef, size_t n, float* xr_out);
/* subbandSynthesis alone (frame.go:630-688): the semantics of
 * mp3g_plan_synth_execute (vvec carried; store passed through). */
int orc_synth_streams(const mp3g_granule* g, const float* is, const mp3g_stream* streams,
                      uint32_t n_streams, const mp3g_state* state_in, mp3g_state* state_out,
                      int16_t* pcm);
/* Multi-threaded wrapper (one stream per task) used only as the CPU baseline. */
int orc_dsp_streams_mt(const mp3g_granule* g, const int16_t* coef, const mp3g_stream* streams,
                       uint32_t n_streams, int16_t* pcm, int n_threads);

/* Tables exactly as the reference initialises them (for margin tests). */
void orc_tables(float synth_nwin[64][32], float synth_d[512], float imdct_win[4][36],
                float cos12[6][12], float cos36[18][36], double* powtab34 /*8207*/);
/* Bit reader KAT hook (bits.go): read `num` bits sequence from `data`. */
int orc_bits_read(const uint8_t* data, size_t len, const int* nums, int n, int* out, int* err);
/* Frame header helpers (frameheader.go) for KAT tests. */
int orc_header_info(uint32_t h, int* valid, int* samples_per_frame, int* frame_size,
                    int* bytes_per_frame, int* sample_rate, int64_t* frame_duration_ns);

#ifdef __cplusplus
}
#endif
#endif
