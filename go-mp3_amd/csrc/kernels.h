// kernels.h -- device-side work descriptors and kernel entry points.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mp3g.h"
#include "dsp_tables.h"
#include "huff_lut.h"

namespace mp3g {

constexpr uint32_t kChunkStateIn = 1u;   // stream starts from state_in[stream]
constexpr uint32_t kChunkStateOut = 2u;  // this chunk ends its stream and exports state

// One workgroup's work: decode granules [out_first, out_first + n_out) of the
// stream that starts at stream_first (32 bytes).
struct ChunkDesc {
  uint64_t out_first;
  uint64_t stream_first;
  uint32_t n_out;
  uint32_t stream;
  uint32_t flags;
  uint32_t reserved;
};
static_assert(sizeof(ChunkDesc) == 32, "ChunkDesc layout");

// Host-side launchers (defined next to the kernels; no RDC needed).
hipError_t upload_tables(const DspTables& tables);
// Exact-mode kernel variants: v2 = fused/register-blocked workgroup kernel
// (kept as the cross-check: MP3G_FLAG_KERNEL_V2), v4 = one wave per chunk
// (default).  (v1, the per-phase version, was retired in round 4.)
constexpr int kVariantV2 = 2;
// fast mode (MP3G_MODE_FAST): one wave per chunk, reassociated transforms, +-1 LSB
constexpr int kVariantFast = 3;
// exact mode v4 (default): one wave per chunk, the reference's operation order
constexpr int kVariantExact4 = 4;
// The hot zones of a fast-mode launch (granule_fast.hip): the fast kernel
// appends each chunk's zones -- granules whose PCM depends on a hot granule's
// hybrid output -- to the list as chunks of their own, counting them; a
// second launch (the exact v4 kernel over the list) decodes them in the
// reference's order and, when its last workgroup is done, empties the list
// for the next launch.  zone_list_capacity entries (the pieces of the
// kZoneListPerChunk zones a chunk records at most) never overflow it, and
// launch_fast refuses a list of fewer than kZoneListPerChunk per chunk (the
// production kernel has no in-wave fallback).  Device memory of the plan (or pipeline) that
// owns it, laid out as
//   uint32 [0] zones listed, [1] zone-launch workgroups done, [2] capacity,
//   [3] unused, [4..7] hot-granule counters (kHotCounters), then the list
// (zone_scratch_init writes a fresh one); launches that share it must be
// stream-ordered.
constexpr uint32_t kZoneListPerChunk = 8;
// A zone goes into the list in pieces of at most kZonePiece granules (round
// 6): each piece replays its own two-granule halo in the zone launch, whose
// waves then take short pieces instead of one long zone serially (with
// 128-granule chunks a saturated chunk's last zone runs to the chunk end).
#ifndef MP3G_ZONE_PIECE
#define MP3G_ZONE_PIECE 16
#endif
constexpr uint32_t kZonePiece = MP3G_ZONE_PIECE;
// The list entries a chunk can need: its <= kZoneListPerChunk zones lie in
// its output range, so their pieces number at most ceil(n_out / kZonePiece)
// + kZoneListPerChunk.
inline uint64_t zone_list_capacity(const ChunkDesc* c, size_t n) {
  uint64_t cap = 0;
  for (size_t i = 0; i < n; i++) cap += kZoneListPerChunk + (c[i].n_out + kZonePiece - 1) / kZonePiece;
  return cap < 64 ? 64 : cap;
}
struct ZoneScratch {
  uint32_t* aux;  // the header above; the list at aux + 8
  uint32_t cap;
};
inline size_t zone_scratch_bytes(uint32_t cap) { return 32 + (size_t)cap * sizeof(ChunkDesc); }
// Zero header + capacity (synchronous; once per allocation).
hipError_t zone_scratch_init(void* p, uint32_t cap);
// zones: the fast kernel's deferred hot zones (required in fast mode, with
// room for kZoneListPerChunk per chunk: hipErrorInvalidValue otherwise); hot_stats: run the counting build, which adds
// its hot-granule work to the scratch's counters (the other kernels ignore both)
hipError_t launch_granule(int variant, const ChunkDesc* d_chunks, uint32_t n_chunks,
                          const mp3g_granule* d_gran, const int16_t* d_coef,
                          const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm,
                          const ZoneScratch* zones, bool hot_stats, hipStream_t stream);
// The fast kernel's hot-granule counters (granule_fast.hip, MP3G_FLAG_HOT_STATS):
// [0] granules whose PCM the reference-order pass rewrites, [1] hot zones,
// [2] hot granules the fast pass flagged, [3] granules re-run inside a wave
// (zones that did not fit the zone list, with their replays).
constexpr int kHotCounters = 4;

// Copy of `bytes` (a multiple of 16; both pointers 16-B aligned) from device
// memory to device-accessible pinned host memory (`dst`: its device address)
// by a kernel of `blocks` 256-thread workgroups (kernels.hip).
hipError_t launch_copy_out(const void* d_src, void* dst, size_t bytes, int blocks, hipStream_t stream);
// diagnostic: shader clock under load (mp3g_debug_clock_probe)
hipError_t launch_clock_probe(const uint32_t* d_flag, unsigned long long* d_out, uint32_t n_waves,
                              unsigned long long max_ticks, hipStream_t stream);

// Chunks of `variant` resident per CU (one per wave for the fast kernel, one
// per workgroup for the exact kernels), from the kernel's VGPR / LDS usage.
int chunks_per_cu(int variant);

// Main-data decode (huffman_dev.hip): one lane per (granule, channel) job.
// full_rows = false: rows written only up to count1 (+ padding), enough for
// the one-wave plan kernels (fast v3, exact v4) -- MP3G_HUFF_ROWS_COUNT1.
// stage: 0 = the default 28 KB instantiation, 1 = 42 KB (MP3G_HUFF_STAGE_MID),
// 2 = 68 KB (MP3G_HUFF_STAGE_WIDE).
hipError_t launch_huffman(const mp3g_hjob* d_jobs, uint64_t n_jobs, const uint8_t* d_md, mp3g_granule* d_gran,
                          int16_t* d_coef, bool full_rows, int stage, hipStream_t stream);
// The main-data kernel's blocks (jobs per block, LDS stage in 64-bit words:
// default and wide), for the host-side stage advice.
constexpr int kHuffJobsPerBlock = 256;
constexpr int kHuffStageWords = 3584;       // 28 KB: 256 jobs span ~25 KB at 128 kbps
constexpr int kHuffStageWordsMid = 5376;   // 42 KB: ~40 KB at 192 kbps (3 blocks per CU)
constexpr int kHuffStageWordsWide = 8704;  // 68 KB: ~67 KB at 320 kbps

// Diagnostic: fast kernel with per-phase s_memtime sums (8 per chunk) in d_stamps.
constexpr int kFastPhases = 8;
// per chunk: kFastPhases cycle sums, then s_memrealtime (100 MHz) at kernel
// entry, loop start, loop end and exit
constexpr int kFastStampSlots = kFastPhases + 4;
hipError_t launch_fast_stamped(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                               const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out,
                               int16_t* d_pcm, unsigned long long* d_stamps, hipStream_t stream);

// The fast kernel's TU (kernels_fast.hip): its table copy, attributes and launch
// (d_stamps = nullptr: the production build).
// (req: DspTables::req, the exact requantization table of the hot-granule fallback)
hipError_t upload_fast_tables(const FastTables& fast, const float* req);
hipError_t fast_kernel_attributes(hipFuncAttributes* a, int* waves_per_block);
hipError_t launch_fast(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                       const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out,
                       int16_t* d_pcm, unsigned long long* d_stamps, const ZoneScratch* zones, bool hot_stats,
                       hipStream_t stream);

// Exact mode v4 (granule_wexact.hip, same TU as the fast kernel).
hipError_t wexact_kernel_attributes(hipFuncAttributes* a, int* waves_per_block);
hipError_t launch_wexact(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                         const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out,
                         int16_t* d_pcm, hipStream_t stream);

// Standalone polyphase synthesis (granule_synth.hip, same TU): float32
// frequency-inverted lines [n][2][576] -> s16 PCM, over a fast-mode plan.
hipError_t launch_synth(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran, const float* d_lines,
                        const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm, hipStream_t stream);

}  // namespace mp3g
