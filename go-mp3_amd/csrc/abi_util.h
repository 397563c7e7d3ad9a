// abi_util.h -- shared helpers of the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/mp3g.h"

namespace mp3g {
struct ChunkDesc;  // kernels.h
// Records `what` as this thread's mp3g_last_error() text and returns status.
int abi_fail(int status, const char* what);
// Whether the plan kernel of `mode` reads only coefficient lines below count1
// (fast v3, exact v4): the main-data kernel may then skip the zero tails
// (MP3G_HUFF_ROWS_COUNT1).
bool mode_reads_to_count1(unsigned mode);
// The device's constant tables uploaded (once per device).
int ensure_device_ready(int device);
// A plan's chunk table, built on the host (mp3g_plan_create's checks and
// chunking: granules_per_chunk 0 = the cost model), and the launch of a table
// already on the device -- for pipelines that upload tables asynchronously
// (mp3g_decode_streams_into) instead of through a plan's blocking copy.
int plan_chunks(int device, const mp3g_stream* streams, uint32_t n_streams, uint32_t granules_per_chunk,
                uint32_t mode, std::vector<ChunkDesc>* chunks, uint64_t* n_granules, uint64_t* n_halo);
struct ZoneScratch;  // kernels.h
int plan_launch(uint32_t mode, const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm,
                const ZoneScratch* zones, hipStream_t stream);
}  // namespace mp3g
