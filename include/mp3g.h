/*
 * mp3g.h -- C-ABI of the MI355X-native MP3 Layer III granule-decode path.
 *
 * This library replaces the per-frame DSP seam of llehouerou/go-mp3:
 *
 *   func (f *Frame) Decode() []byte              reference internal/frame/frame.go:121-138
 *
 * i.e. requantize -> reorder -> MS/intensity stereo -> antialias -> hybrid
 * IMDCT + overlap -> frequency inversion -> 32-subband polyphase synthesis ->
 * s16le stereo PCM, for a BATCH of granules from many independent streams, on
 * a gfx950 GPU.  The bitstream parse (frame header, side info, scale factors,
 * Huffman, bit reservoir) stays on the host: the caller hands over exactly
 * the fields `Decode` reads (reference frame.go:140-688)
 * as packed granule descriptors plus int16 coefficients.
 *
 * Plain C types only: no torch, no HIP types in the signatures.  Every call
 * returns an mp3g_status (0 = OK); nothing throws across the ABI and no caller
 * pointer is retained after a call returns (cgo rule).
 *
 * Threading: a context / plan is single-threaded like mp3.Decoder
 * (reference decode.go:27-33); distinct contexts may be used concurrently.
 * Executions of one fast-mode plan (mp3g_plan_execute) must also be ordered
 * on the device: one stream, or streams synchronised between them -- its
 * launches share the plan's zone list (ABI 5).  One plan per stream for
 * concurrent launches.
 */
#ifndef MP3G_H
#define MP3G_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: mp3g_lame_toc_offset returns a status and writes the offset through an
 *    out-parameter (version 1 returned the offset); the fast-mode hot-granule
 *    fallback (no signature change).
 * 3: streaming input -- mp3g_reader + mp3g_decoder_new_reader, MP3G_ERR_READ;
 *    MP3G_FLAG_KERNEL_V1 retired.
 * 4: main-data kernel stages for high bitrates -- MP3G_HUFF_STAGE_MID /
 *    MP3G_HUFF_STAGE_WIDE flags of mp3g_huffman_execute_ex and the advice
 *    mp3g_huffman_stage_flags.
 * 5: mp3g_plan_hot_stats and MP3G_FLAG_HOT_STATS (the fast kernel's
 *    hot-granule fallback counters); a fast-mode plan owns a zone list its
 *    launches share, so executions of one plan must be stream-ordered.
 *    (Compatible additions since: the diagnostic mp3g_debug_clock_probe.) */
#define MP3G_ABI_VERSION 5

/* ---- status codes ------------------------------------------------------ */
typedef enum mp3g_status {
  MP3G_OK = 0,
  MP3G_ERR_INVALID_ARGUMENT = 1, /* null pointer, bad sizes, bad plan       */
  MP3G_ERR_INVALID_GRANULE = 2,  /* descriptor field out of range (checked mode) */
  MP3G_ERR_NO_DEVICE = 3,        /* no gfx950 device / HIP init failed      */
  MP3G_ERR_DEVICE = 4,           /* HIP runtime error (see mp3g_last_error) */
  MP3G_ERR_OUT_OF_MEMORY = 5,
  MP3G_ERR_PARSE = 6,            /* host bitstream parse error (decoder API) */
  MP3G_EOF = 7,                  /* end of stream (decoder API, io.EOF)      */
  MP3G_ERR_UNSUPPORTED = 8,      /* MPEG 2.5, layer I/II, free format, ...   */
  MP3G_ERR_NO_XING_HEADER = 9,   /* lameinfo.ErrNoXingHeader                 */
  MP3G_ERR_UNEXPECTED_EOF = 10, /* io.ErrUnexpectedEOF (lameinfo.ParseFromReader) */
  MP3G_ERR_READ = 11             /* the caller's reader callback failed (decoder API;
                                    decode.go:48-63 returns a reader's error as is) */
} mp3g_status;

/* ---- boundary input: one granule descriptor ---------------------------- */
/*
 * Per-channel fields read by the DSP.  Field <- reference source:
 *   count1           sideinfo.SideInfo.Count1, set by maindata/huffman.go:451
 *   global_gain      sideinfo.go:115            scalefac_scale  sideinfo.go:151
 *   preflag          sideinfo.go:149 (MPEG-1) / maindata.go:136 (MPEG-2)
 *   win_switch_flag  sideinfo.go:117            block_type      sideinfo.go:119,143
 *   mixed_block_flag sideinfo.go:120            subblock_gain   sideinfo.go:125
 *   scalefac_l       maindata.MainData.ScalefacL[gr][ch] (maindata.go:34)
 *   scalefac_s       maindata.MainData.ScalefacS[gr][ch] (maindata.go:35)
 * 72 bytes, no padding.
 */
typedef struct mp3g_channel {
  uint16_t count1;          /* 0..576: first line of the zero region          */
  uint8_t global_gain;      /* 0..255                                         */
  uint8_t scalefac_scale;   /* 0/1                                            */
  uint8_t preflag;          /* 0/1                                            */
  uint8_t win_switch_flag;  /* 0/1                                            */
  uint8_t block_type;       /* 0..3                                           */
  uint8_t mixed_block_flag; /* 0/1                                            */
  uint8_t subblock_gain[3]; /* 0..7                                           */
  uint8_t scalefac_l[22];   /* 0..15                                          */
  uint8_t scalefac_s[13][3];/* [sfb][win], 0..15                              */
} mp3g_channel;

/*
 * One granule = half an MPEG-1 frame (or a whole MPEG-2 LSF frame).
 *   header : the raw 32-bit frameheader.FrameHeader (frameheader.go:29-137);
 *            the DSP reads lsf, sampling-frequency index, mode, mode_ext from it.
 *   gr     : granule index inside its frame (0/1), informational.
 * 160 bytes (16-byte multiple so a descriptor is ten 16-B loads).
 */
typedef struct mp3g_granule {
  uint32_t header;
  uint32_t gr;
  mp3g_channel ch[2];
  uint8_t reserved[8];
} mp3g_granule;

/* Coefficients: int16 [n_granules][2][576], the integer Huffman output that
 * the reference keeps as float32 in MainData.Is (maindata.go:36).  |x| <= 8206
 * (15 + 13 linbits).  Mono granules leave [g][1][*] unread. */
#define MP3G_LINES 576
#define MP3G_COEF_PER_GRANULE (2 * MP3G_LINES)
/* PCM: int16 [n_granules][576][2] = the bytes Decode() returns, concatenated
 * (frame.go:134: granule gr at byte 2304*gr; mono duplicated, frame.go:671-678). */
#define MP3G_PCM_BYTES_PER_GRANULE (MP3G_LINES * 2 * 2)

/* ---- cross-granule DSP state (reference Frame.store / Frame.vVec) ------- */
/* Layout identical to the reference fields (frame.go:48-49): copying a
 * Frame's state in/out is a memcpy.  12,800 bytes.  A state_in is a state a
 * decoder produced (Frame.store / vVec are only ever written by Decode): its
 * vVec blocks are V = synthNWin * S, whose 64 entries hold 33 distinct values,
 * and the one-wave kernels (fast v3, exact v4) keep only those; the workgroup
 * kernel (MP3G_FLAG_KERNEL_V2) carries all 64 of any vvec. */
typedef struct mp3g_state {
  float store[2][32][18]; /* IMDCT overlap                          */
  float vvec[2][1024];    /* polyphase FIFO, newest V block at [0:64] */
} mp3g_state;

/* ---- streams ------------------------------------------------------------ */
/* A stream is a run of consecutive granules of one MP3 stream; the granules
 * of stream s are [first_granule, first_granule + n_granules) in the granule
 * and coefficient arrays, and its PCM goes to the same granule slots of the
 * output.  State is carried inside the run exactly as frame.Read carries it
 * (frame.go:110-113). */
#define MP3G_STREAM_STATE_IN  1u /* start from state_in[s] (else zero state, = stream start / after Seek, decode.go:106-108) */
#define MP3G_STREAM_STATE_OUT 2u /* write the state after the last granule to state_out[s] */
typedef struct mp3g_stream {
  uint64_t first_granule;
  uint32_t n_granules;
  uint32_t flags;
} mp3g_stream;

/* ---- decode modes -------------------------------------------------------- */
#define MP3G_MODE_EXACT 0u   /* bit-exact vs the reference (linux/amd64 float semantics) */
#define MP3G_MODE_FAST  1u   /* reassociated fast transforms; |dPCM| <= 1 LSB            */
#define MP3G_FLAG_CHECKED 0x100u /* validate descriptor ranges on the host first      */
#define MP3G_FLAG_KERNEL_V1 0x200u /* retired in ABI 3 (the per-phase v1 cross-check kernel):
                                      mp3g_plan_create returns MP3G_ERR_UNSUPPORTED */
#define MP3G_FLAG_KERNEL_V2 0x800u /* exact mode via the workgroup v2 kernel (cross-check; the
                                      default exact kernel is v4, one wave per chunk) */
#define MP3G_FLAG_HOST_HUFFMAN 0x400u /* decoder: scale factors + Huffman on the host (mp3g_parse_*)
                                         instead of the GPU main-data kernel (cross-check) */
#define MP3G_FLAG_HOT_STATS 0x1000u /* fast-mode plans: count the hot-granule fallback's work
                                       (mp3g_plan_hot_stats; a kernel build that costs ~1.5 %) */

/* ---- library / device ---------------------------------------------------- */
int mp3g_abi_version(void);
/* Human-readable text for a status code; static storage. */
const char* mp3g_status_string(int status);
/* Last HIP/runtime error text of this thread (empty if none); static storage. */
const char* mp3g_last_error(void);
/* Number of visible gfx950 devices. */
int mp3g_device_count(int* out_count);

/* ---- checked-mode validation (host only, no GPU) ------------------------- */
/* Returns MP3G_OK or MP3G_ERR_INVALID_GRANULE and the first bad index. */
int mp3g_validate(const mp3g_granule* granules, const int16_t* coeffs,
                  uint64_t n_granules, uint64_t* bad_index);

/* ---- plans: device-resident work decomposition ---------------------------
 * A plan splits every stream into chunks processed by independent waves /
 * workgroups.  granules_per_chunk: 0 < k < 2^31 = every stream cut into
 * ceil(n / k) chunks of equal length +-1 (so at most k granules each);
 * 0 = automatic (a length from the launch-cost model, then the chunk count
 * rounded to whole rounds of resident chunks and every stream cut into
 * chunks of equal length +-1); MP3G_PLAN_CHUNKS(c) = about c chunks in total,
 * spread over the streams by length, equal lengths +-1 (c < 2^31).  Every
 * chunk holds < 2^32 granules (MP3G_ERR_UNSUPPORTED otherwise).  A chunk that does
 * not start a stream re-derives its entry state from the two preceding
 * granules (bit-identical to serial decode; DESIGN.md "halo").  The plan lives
 * on `device` and can be executed many times (graph-capturable). */
#define MP3G_PLAN_CHUNKS(c) (0x80000000u | (uint32_t)(c))
typedef struct mp3g_plan mp3g_plan;
int mp3g_plan_create(int device, const mp3g_stream* streams, uint32_t n_streams,
                     uint32_t granules_per_chunk, uint32_t mode, mp3g_plan** out_plan);
int mp3g_plan_destroy(mp3g_plan* plan);
/* Number of chunks (= workgroups launched) and granules incl. halo work. */
int mp3g_plan_info(const mp3g_plan* plan, uint64_t* n_chunks, uint64_t* n_granules,
                   uint64_t* n_halo_granules);

/* Asynchronous execution on device-resident buffers.  All pointers are device
 * pointers; `hip_stream` is a hipStream_t (NULL = default stream).  state_in /
 * state_out may be NULL when no stream of the plan uses the flag.
 * Fast mode (ABI 5): a launch's hot zones go through a zone list owned by the
 * plan and emptied by the launch itself (graph replays are fine), so two
 * executions of ONE plan must not overlap on the device -- issue them on one
 * stream or synchronise the streams; concurrent launches need a plan each.
 * If the zone launch cannot be enqueued, the list is reset on the stream
 * before the error is returned (the next execution starts clean). */
int mp3g_plan_execute(mp3g_plan* plan, const mp3g_granule* d_granules,
                      const int16_t* d_coeffs, const mp3g_state* d_state_in,
                      mp3g_state* d_state_out, int16_t* d_pcm, void* hip_stream);

/* Standalone polyphase synthesis: go-mp3's subbandSynthesis
 * (internal/frame/frame.go:630-688, called per channel at frame.go:133) over
 * the granules of a fast-mode plan, without the stages before it.
 * d_lines: float32 [n_granules][2][576], the frequency-inverted hybrid output
 * that subbandSynthesis reads (MainData.Is after frame.go:132; mono granules
 * leave [g][1][*] unread).  PCM as mp3g_plan_execute (+-1 LSB, fast mode).
 * State: vvec carried as in mp3g_plan_execute; state_out.store is
 * state_in.store (or zero), since this stage does not touch it. */
int mp3g_plan_synth_execute(mp3g_plan* plan, const mp3g_granule* d_granules,
                            const float* d_lines, const mp3g_state* d_state_in,
                            mp3g_state* d_state_out, int16_t* d_pcm, void* hip_stream);

/* Fast-mode plans: the work of the hot-granule fallback (granules whose
 * hybrid output exceeds the fast transforms' magnitude bound are decoded
 * again in the reference's operation order), summed over
 * the plan's launches since creation or the last reset, for plans created
 * with MP3G_FLAG_HOT_STATS (others: always 0).  out4[0]: granules whose PCM
 * that pass rewrites; out4[1]: hot zones (runs of such granules); out4[2]: hot
 * granules the fast pass flagged; out4[3]: granules re-run inside a chunk's
 * own wave -- always 0 since the zone list holds every chunk's zones (kept
 * for ABI 5 layout).
 * Synchronises the device; reset != 0 zeroes the counters after reading.
 * A fast-mode plan's launches share its zone list (emptied by each launch
 * itself: graph replays are fine): executions of one plan must be ordered
 * (one stream, or synchronised between streams).  No reference
 * counterpart: go-mp3 has one arithmetic (frame.go:140-688). */
int mp3g_plan_hot_stats(mp3g_plan* plan, uint64_t* out4, int reset);

/* ---- synchronous host-buffer decode (the cgo drop-in entry) --------------
 * Copies the batch to `device`, decodes it and copies PCM (and state_out)
 * back before returning.  Equivalent to calling Frame.Decode on every frame of
 * every stream in order.  mode = MP3G_MODE_* | optional MP3G_FLAG_CHECKED. */
int mp3g_decode_host(int device, const mp3g_granule* granules, const int16_t* coeffs,
                     uint64_t n_granules, const mp3g_stream* streams, uint32_t n_streams,
                     const mp3g_state* state_in, mp3g_state* state_out, int16_t* pcm,
                     uint32_t mode);

/* ---- host bitstream parse (CPU only) -----------------
 * The part of go-mp3's frame.Read that feeds Decode: tags (source.go:42-83),
 * sync search + header (frameheader.go:279-328), side info (sideinfo.go),
 * bit reservoir (maindata.go:290-323), scale factors and Huffman decoding
 * (maindata.go:119-288, maindata/huffman.go:27-138).  Output buffers are
 * allocated by the library (free with mp3g_free).  *end_status is MP3G_EOF
 * when the stream ended the way decode.go maps to io.EOF, MP3G_ERR_PARSE for
 * any other frame.Read error, MP3G_ERR_UNSUPPORTED where the reference would
 * panic; the granules of every frame before that point are returned. */
int mp3g_parse_stream(const uint8_t* data, size_t len, mp3g_granule** granules, int16_t** coeffs,
                      uint64_t* n_granules, int* end_status);
/* Many independent streams on n_threads host threads (0 = all cores); the
 * stream table describes where each stream's granules landed. */
int mp3g_parse_streams(uint32_t n_streams, const uint8_t* const* datas, const size_t* lens, int n_threads,
                       mp3g_granule** granules, int16_t** coeffs, uint64_t* n_granules, mp3g_stream* streams,
                       int* end_status);
void mp3g_free(void* p);

/* ---- main-data decode on the GPU --------------------
 * Splits frame.Read (frame.go:67-115) at the bit reservoir:
 *   host   (mp3g_scan_streams): tags, sync search, header, side info and the
 *          reservoir resolution -- sequential but byte-level, no Huffman;
 *   device (mp3g_huffman_execute): scale factors (maindata.go:119-288) and
 *          Huffman decoding (maindata/huffman.go:27-138, huffman/huffman.go:
 *          348-419) of every (granule, channel) in parallel, completing the
 *          granule descriptors and writing the int16 coefficients that
 *          mp3g_plan_execute consumes.
 * The result is byte-identical to mp3g_parse_streams.  The main data of each
 * stream is concatenated into one byte buffer; frame f's bit buffer (the
 * reference's `prev.Tail(main_data_begin) ++ buf`, or `prev ++ buf` on a
 * reservoir underflow, maindata.go:290-323) is always a suffix of that
 * concatenation ending at bit_end, so jobs address it with absolute bit
 * positions.
 *
 * One job per (granule, channel), jobs[2*g + ch]; 48 bytes. */
#define MP3G_SF_NONE 0        /* channel absent (mono): zero coefficients      */
#define MP3G_SF_MPEG1_LONG 1  /* maindata.go:233-279 (scfsi copies from gr 0) */
#define MP3G_SF_MPEG1_SHORT 2 /* maindata.go:221-231                          */
#define MP3G_SF_MPEG1_MIXED 3 /* maindata.go:207-220                          */
#define MP3G_SF_MPEG2_LONG 4  /* maindata.go:132-172, 22 scale factors        */
#define MP3G_SF_MPEG2_SHORT 5 /* maindata.go:173-179, 39 scale factors        */
typedef struct mp3g_hjob {
  uint64_t part2_start;     /* absolute bit position of the scale factors (maindata.go:202) */
  uint64_t bit_end;         /* end of the frame's main-data bits: reads at/after it yield 0
                               and do not advance (bits.go:45-77) */
  uint32_t scf0_delta;      /* MPEG-1 granule 1 with scfsi: granule 0's part2_start is
                               part2_start - scf0_delta */
  uint16_t part2_3_length;  /* sideinfo.go:114 */
  uint16_t big_values;      /* <= 288 (more is a frame error, found by the scan) */
  uint16_t region1_start;   /* lines (maindata/huffman.go:39-64) */
  uint16_t region2_start;
  uint8_t table_select[3];
  uint8_t count1_table;     /* count1table_select */
  uint8_t sf_kind;          /* MP3G_SF_* */
  uint8_t scfsi;            /* granule 1: bit k = scale-factor part k copied from granule 0 */
  uint8_t slen[4];          /* bits per scale factor: MPEG-1 {slen1, slen2}; MPEG-2 per part */
  uint8_t nsf[4];           /* MPEG-2: scale factors per part (ISO 13818-3 Table 6) */
  uint8_t sf0_kind;         /* granule 0's sf_kind and slen (for the scfsi copy) */
  uint8_t sf0_slen[2];
  uint8_t reserved[3];
} mp3g_hjob;

/* Host scan of many streams on n_threads host threads (0 = all cores).  The
 * scan owns its buffers until mp3g_scan_free; mp3g_scan_buffers returns:
 *   granules   [n_granules] descriptors with the side-info fields set (scale
 *              factors and count1 are written by mp3g_huffman_execute)
 *   jobs       [2 * n_granules]
 *   main_data  [main_data_bytes] (incl. 16 zero bytes of padding)
 *   streams    [n_streams] where each stream's granules landed
 *   end_status [n_streams] as mp3g_parse_streams.
 * A frame the reference rejects (frame.Read error or panic) ends its stream
 * exactly where mp3g_parse_streams ends it. */
typedef struct mp3g_scan mp3g_scan;
int mp3g_scan_streams(uint32_t n_streams, const uint8_t* const* datas, const size_t* lens, int n_threads,
                      mp3g_scan** out);
int mp3g_scan_buffers(const mp3g_scan* scan, uint64_t* n_granules, uint64_t* main_data_bytes,
                      const mp3g_granule** granules, const mp3g_hjob** jobs, const uint8_t** main_data,
                      const mp3g_stream** streams, const int** end_status);
void mp3g_scan_free(mp3g_scan* scan);

/* Device decode of the 2 * n_granules jobs (device pointers; d_granules holds
 * the scan's descriptors and is completed in place).  Asynchronous on
 * hip_stream (NULL = default stream). */
int mp3g_huffman_execute(int device, const mp3g_hjob* d_jobs, uint64_t n_granules, const uint8_t* d_main_data,
                         mp3g_granule* d_granules, int16_t* d_coeffs, void* hip_stream);
/* The same with flags.  MP3G_HUFF_ROWS_COUNT1: each coefficient row is
 * written only up to its count1 plus padding (the zero tail is left as it
 * was): what the default plan kernels (MP3G_MODE_FAST, and MP3G_MODE_EXACT
 * without MP3G_FLAG_KERNEL_V2) read, since lines at and above count1
 * are zero (maindata/huffman.go:127-134).  The batch and decoder APIs use it
 * for those modes (c3 main-data kernel -13 %). */
#define MP3G_HUFF_ROWS_COUNT1 1u
/* Main-data stage per 256-job block (ABI 4): by default 28 KB of LDS (16
 * waves per CU); MP3G_HUFF_STAGE_MID 42 KB (12 waves per CU);
 * MP3G_HUFF_STAGE_WIDE 68 KB (8 waves per CU).  A block whose main data does
 * not fit its stage reads it from global memory, which is slower: 256 jobs
 * span ~25 KB at 128 kbps, ~40 KB at 192, ~67 KB at 320.
 * mp3g_huffman_stage_flags tells which suits a batch. */
#define MP3G_HUFF_STAGE_WIDE 2u
#define MP3G_HUFF_STAGE_MID 4u
int mp3g_huffman_execute_ex(int device, const mp3g_hjob* d_jobs, uint64_t n_granules, const uint8_t* d_main_data,
                            mp3g_granule* d_granules, int16_t* d_coeffs, uint32_t flags, void* hip_stream);
/* Host-side advice for mp3g_huffman_execute_ex: the stage (0,
 * MP3G_HUFF_STAGE_MID or MP3G_HUFF_STAGE_WIDE) of least modelled time for the
 * batch's 256-job blocks, from their main-data spans (each block staged when
 * it fits, read from global memory otherwise; the stage's waves per CU).
 * `jobs`: the scan's jobs (host memory, 2 * n_granules). */
uint32_t mp3g_huffman_stage_flags(const mp3g_hjob* jobs, uint64_t n_granules);

/* Bitstreams in, PCM out (the batch drop-in): scan on the host, Huffman + DSP
 * on `device`.  *pcm (library-allocated, free with mp3g_free) holds
 * n_granules blocks of 576 stereo s16 samples; streams / end_status as
 * mp3g_parse_streams. */
int mp3g_decode_streams(int device, uint32_t n_streams, const uint8_t* const* datas, const size_t* lens,
                        int n_threads, uint32_t mode, int16_t** pcm, uint64_t* n_granules,
                        mp3g_stream* streams, int* end_status);

/* The same into caller memory, pipelined: the streams are decoded in groups
 * and each group's host scan overlaps the transfers and kernels of the group
 * before it.  The output layout comes from a header-only pre-pass: stream k
 * starts at block streams[k].first_granule of `pcm` (576 stereo s16 samples
 * per block); a stream its side info ends early (a parse error or a
 * reference panic after its last good frame) decodes its n_granules blocks
 * and leaves the rest of its range zero.  `pcm` (host memory; pinned memory
 * keeps the device-to-host copies at PCIe speed and asynchronous) must hold
 * pcm_cap_granules blocks; if that is too few, nothing is decoded and the
 * call returns MP3G_ERR_INVALID_ARGUMENT with *n_granules = the blocks
 * needed.  n_groups = 0 picks the group count. */
int mp3g_decode_streams_into(int device, uint32_t n_streams, const uint8_t* const* datas, const size_t* lens,
                             int n_threads, uint32_t mode, uint32_t n_groups, int16_t* pcm,
                             uint64_t pcm_cap_granules, uint64_t* n_granules, mp3g_stream* streams,
                             int* end_status);

/* mp3g_decode_streams_into keeps its staging (page-locked) and device
 * buffers per device between calls; this frees them (idle sets only). */
void mp3g_release_cached_buffers(void);

/* ---- decoder: mp3.NewDecoder / io.Reader / io.Seeker (decode.go:27-388) ----
 * Scans on the host with read-ahead (headers, side info, reservoir) and
 * decodes batches of frames on `device`: scale factors + Huffman codes with
 * the main-data kernel, then the DSP (mode = MP3G_MODE_EXACT | MP3G_MODE_FAST,
 * | MP3G_FLAG_HOST_HUFFMAN for the host parse instead of the Huffman kernel).  `data` is copied.
 * seekable = 0 models a reader that is not an io.Seeker (Length = -1).
 * Read returns MP3G_OK with *n >= 1, MP3G_EOF, or the error of the frame
 * that failed (after all PCM before it was delivered) -- like Decoder.Read. */
typedef struct mp3g_decoder mp3g_decoder;
int mp3g_decoder_new(const uint8_t* data, size_t len, int seekable, int device, uint32_t mode,
                     mp3g_decoder** out);

/* Streaming input: the caller's io.Reader (and io.Seeker) as callbacks, so a
 * decoder runs on input it has not got yet -- a pipe, a socket, a live radio
 * stream -- and pulls bytes as it needs them, like the reference's source
 * (source.go:99-122, io.ReadFull on the reader).  mp3.NewDecoder(r)
 * (decode.go:361-388) is mp3g_decoder_new_reader: it returns once the tags
 * and frame 0 are in (for a seeker, after the header walk of
 * ensureFrameStartsAndLength, decode.go:154-216, as the reference does).
 *   read : io.Reader.Read -- write up to `cap` bytes to `buf`, return the
 *          count; 0 = io.EOF; < 0 = an error (the decoder call in progress
 *          returns MP3G_ERR_READ; a later call asks the reader again).
 *   seek : io.Seeker.Seek (whence 0/1/2), the new offset or < 0 on error; NULL
 *          when the reader is no io.Seeker (Length = -1, Seek fails as the
 *          reference's does, source.go:28-33).
 *   user : passed back to the callbacks verbatim, never dereferenced (for
 *          cgo: a runtime/cgo.Handle, not a Go pointer).
 * Read-ahead policy: with a seek callback (a file-like source) the decoder
 * reads ahead in batches; without one it calls `read` only when it holds no
 * complete frame it has not decoded -- exactly when the reference's
 * Decoder.Read blocks on its reader -- so every frame whose bytes have
 * arrived is delivered without waiting for more input.  The callbacks run on
 * the thread that calls into the decoder, only during that call. */
typedef struct mp3g_reader {
  int64_t (*read)(void* user, uint8_t* buf, size_t cap);
  int64_t (*seek)(void* user, int64_t offset, int whence);
  void* user;
} mp3g_reader;
int mp3g_decoder_new_reader(const mp3g_reader* reader, int device, uint32_t mode, mp3g_decoder** out);
void mp3g_decoder_free(mp3g_decoder* dec);
int mp3g_decoder_read(mp3g_decoder* dec, uint8_t* buf, size_t cap, size_t* n);
/* io.ReadFull over Decoder.Read (Go's io.ReadFull loops Read the same way):
 * repeated reads until `cap` bytes, EOF or an error.  Returns MP3G_OK with
 * *n == cap, or the status that ended it (MP3G_EOF / the frame's error) with
 * *n = the bytes delivered before it.  One call instead of one per frame. */
int mp3g_decoder_read_full(mp3g_decoder* dec, uint8_t* buf, size_t cap, size_t* n);
/* whence: 0 = io.SeekStart, 1 = io.SeekCurrent, 2 = io.SeekEnd */
int mp3g_decoder_seek(mp3g_decoder* dec, int64_t offset, int whence, int64_t* newpos);
/* SampleRate, Length (-1 if unknown), BytesPerFrame, current position (bytes) */
int mp3g_decoder_info(const mp3g_decoder* dec, int* sample_rate, int64_t* length, int64_t* bytes_per_frame,
                      int64_t* position);
/* time API; durations are time.Duration nanoseconds */
int64_t mp3g_decoder_duration_ns(const mp3g_decoder* dec);
int64_t mp3g_decoder_position_ns(const mp3g_decoder* dec);
int64_t mp3g_decoder_remaining_ns(const mp3g_decoder* dec);
double mp3g_decoder_progress(const mp3g_decoder* dec);
int64_t mp3g_decoder_sample_position(const mp3g_decoder* dec);
int64_t mp3g_decoder_sample_count(const mp3g_decoder* dec);
int mp3g_decoder_seek_to_sample(mp3g_decoder* dec, int64_t sample);
int mp3g_decoder_seek_to_time_ns(mp3g_decoder* dec, int64_t t_ns);
int mp3g_decoder_skip_ns(mp3g_decoder* dec, int64_t delta_ns);

/* ---- diagnostics (not part of the decode contract) -----------------------
 * Runs a FAST-mode plan once through the s_memtime-instrumented build of the
 * fast kernel and returns, per kernel phase, the shader cycles summed over
 * all chunks (out_cycles[0..7]: parameters, requantize, stereo+antialias,
 * IMDCT, S rows into the ring, matrixing (DCT-32), window+store, history
 * shift).  PCM is written as by mp3g_plan_execute.  Synchronous. */
int mp3g_plan_debug_phases(mp3g_plan* plan, const mp3g_granule* d_granules, const int16_t* d_coeffs,
                           int16_t* d_pcm, uint64_t* out_cycles, void* hip_stream);
/* The same instrumented launch; per chunk (out_ticks[4 * chunk + 0..3]) the
 * wave's s_memrealtime (100 MHz) at kernel entry, at the start and the end of
 * its granule loop and at exit: the launch's ramp, per-wave span and tail. */
int mp3g_plan_debug_timeline(mp3g_plan* plan, const mp3g_granule* d_granules, const int16_t* d_coeffs,
                             int16_t* d_pcm, uint64_t* out_ticks, void* hip_stream);

/* Shader clock under load: launches n_waves one-wave workgroups on
 * hip_stream that spin until the device word *d_flag turns non-zero (set it
 * from another stream after the work to be measured) or max_ms (<= 10,000)
 * pass, each writing 5 uint64 to d_out[5 * wg ..]: s_memtime (shader cycles)
 * and s_memrealtime (100 MHz) at the start and the end of its window, and
 * whether it saw the flag.  Asynchronous. */
int mp3g_debug_clock_probe(int device, const uint32_t* d_flag, uint64_t* d_out, uint32_t n_waves,
                           uint32_t max_ms, void* hip_stream);

/* ---- Xing / Info / LAME tag (lameinfo/lameinfo.go) ----
 * The reference's lameinfo package: the tag in the first frame (encoder delay
 * and padding for gapless playback, frame / byte counts, the VBR seek TOC).
 * The decoder never reads it (decode.go decodes the tag frame as silence);
 * callers trim with the two totals.  140 bytes. */
#define MP3G_XING_FRAME_COUNT 0x0001u /* lameinfo.FlagFrameCount */
#define MP3G_XING_BYTE_COUNT 0x0002u  /* FlagByteCount */
#define MP3G_XING_TOC 0x0004u         /* FlagTOC */
#define MP3G_XING_VBR_SCALE 0x0008u   /* FlagVBRScale */
#define MP3G_LAME_DECODER_DELAY 529   /* lameinfo.DecoderDelay */
typedef struct mp3g_lame_info {
  uint32_t is_xing;         /* Info.IsXing: tag "Xing" (VBR) vs "Info" (CBR) */
  uint32_t flags;           /* Info.Flags */
  uint32_t frame_count;     /* Info.FrameCount */
  uint32_t byte_count;      /* Info.ByteCount */
  uint8_t toc[100];         /* Info.TOC */
  uint32_t vbr_scale;       /* Info.VBRScale */
  uint32_t has_lame;        /* Info.HasLAMEInfo(): LAMEVersion != "" */
  char lame_version[12];    /* Info.LAMEVersion: the 9 bytes as stored (may hold NULs), zero padded */
  uint16_t encoder_delay;   /* Info.EncoderDelay */
  uint16_t encoder_padding; /* Info.EncoderPadding */
} mp3g_lame_info;

/* lameinfo.Parse (lameinfo.go:139-270): one whole frame incl. its header.
 * MP3G_OK or MP3G_ERR_NO_XING_HEADER. */
int mp3g_lame_parse(const uint8_t* frame, size_t len, mp3g_lame_info* out);
/* lameinfo.ParseFromReader (lameinfo.go:288-328) on a reader positioned at
 * `data`: reads the header, sizes the frame, reads the frame, parses it.
 * MP3G_OK, MP3G_ERR_NO_XING_HEADER, MP3G_EOF (io.EOF) or
 * MP3G_ERR_UNEXPECTED_EOF; *consumed (may be NULL) = bytes read. */
int mp3g_lame_parse_reader(const uint8_t* data, size_t len, mp3g_lame_info* out, size_t* consumed);
/* Info.TotalDelay / Info.TotalPadding (lameinfo.go:92-111) */
int mp3g_lame_total_delay(const mp3g_lame_info* info);
int mp3g_lame_total_padding(const mp3g_lame_info* info);
/* Gapless trim of n_samples decoded samples (per channel) of a stream whose
 * first frame held the tag: keep [*first, *first + *count); tag_frame_samples
 * = what the decoder produced for the tag frame (1152 MPEG-1, 576 MPEG-2).
 * The reference only exposes the two totals; this applies them. */
int mp3g_lame_trim(const mp3g_lame_info* info, uint64_t n_samples, uint32_t tag_frame_samples, uint64_t* first,
                   uint64_t* count);
/* Xing TOC seek: *offset = byte offset of `percent` (0..100) of the playback
 * time, from Info.TOC (lameinfo.go:33-35) scaled by the tag's byte count
 * (flag 0x2) or, when the tag carries none, by `stream_bytes` (the caller's
 * audio byte length); linear without a TOC.  MP3G_ERR_INVALID_ARGUMENT (and
 * *offset = 0) when neither byte count is known. */
int mp3g_lame_toc_offset(const mp3g_lame_info* info, double percent, uint64_t stream_bytes, uint64_t* offset);

#ifdef __cplusplus
}
#endif
#endif /* MP3G_H */
