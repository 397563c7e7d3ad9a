// kernels_fast.hip -- device translation unit of the one-wave-per-chunk
// granule kernels: fast mode v3 (granule_fast.hip, MP3G_MODE_FAST), the
// standalone polyphase kernel (granule_synth.hip) and exact mode v4
// (granule_wexact.hip, the default MP3G_MODE_EXACT kernel), with their own
// copy of the fast tables.
//
// Own TU so it gets its own codegen options (Makefile): it is compiled with
// machine LICM off.  The kernel's packed-FP32 transforms take their constants
// from SGPR pairs (VOP3P has no literal operand); hoisted out of the granule
// loop, ~90 of them overflow the wave's SGPRs and were spilled to VGPR lanes,
// costing a v_readlane (VALU) per use inside the loop.  Left in place they are
// s_mov_b32 (SALU) next to their use.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/mp3g.h"
#include "dsp_tables.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace mp3g {
__constant__ FastTables g_fast;
// DspTables::req (131 KB, global memory): the exact requantization of the
// reference-order fallback for hot granules (granule_fast.hip)
__device__ float g_req[4][8207];
}  // namespace mp3g

#include "granule_hdr.h"
#include "granule_fast.hip"
#include "granule_synth.hip"
#include "granule_wexact.hip"

#ifndef MP3G_ZONE_CHUNKS_PER_WG
// zone-launch workgroups: one per this many chunks (16 .. 512).  32 since the
// round-6 chunk model halved c3's chunk count (128 granules per chunk): c3
// keeps its 512 workgroups (at 256 the ~10 %-hot batch took 8.2 ms instead of
// 6.3), c2 gets 128
#define MP3G_ZONE_CHUNKS_PER_WG 32
#endif

namespace mp3g {

hipError_t upload_fast_tables(const FastTables& fast, const float* req) {
  const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_fast), &fast, sizeof(FastTables), 0, hipMemcpyHostToDevice);
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_req), req, sizeof(float) * 4 * 8207, 0, hipMemcpyHostToDevice);
}

hipError_t fast_kernel_attributes(hipFuncAttributes* a, int* waves_per_block) {
  *waves_per_block = v3::kWaves;
  return hipFuncGetAttributes(a, reinterpret_cast<const void*>(&v3::granule_fast_kernel<false>));
}

hipError_t zone_scratch_init(void* p, uint32_t cap) {
  uint32_t h[8] = {0, 0, cap, 0, 0, 0, 0, 0};
  return hipMemcpy(p, h, sizeof(h), hipMemcpyHostToDevice);
}

hipError_t launch_fast(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                       const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out,
                       int16_t* d_pcm, unsigned long long* d_stamps, const ZoneScratch* zones, bool hot_stats,
                       hipStream_t stream) {
  if (n_chunks == 0) return hipSuccess;
  const dim3 grid((n_chunks + v3::kWaves - 1) / v3::kWaves), block(64 * v3::kWaves);
  // the production builds defer every hot zone to the plan's zone list: a
  // fast launch without one is the diagnostic (stamped) build only
  if (!d_stamps && (!zones || !zones->aux || zones->cap < (uint64_t)kZoneListPerChunk * n_chunks)) return hipErrorInvalidValue;
  uint32_t* aux = zones ? zones->aux : nullptr;
  if (d_stamps)  // (diagnostic: zones in the wave, no list)
    hipLaunchKernelGGL(v3::granule_fast_kernel<true>, grid, block, 0, stream, d_chunks, n_chunks, d_gran, d_coef,
                       d_state_in, d_state_out, d_pcm, static_cast<void*>(d_stamps));
  else if (hot_stats && aux)
    hipLaunchKernelGGL((v3::granule_fast_kernel<false, true>), grid, block, 0, stream, d_chunks, n_chunks, d_gran,
                       d_coef, d_state_in, d_state_out, d_pcm, static_cast<void*>(aux));
  else
    hipLaunchKernelGGL(v3::granule_fast_kernel<false>, grid, block, 0, stream, d_chunks, n_chunks, d_gran, d_coef,
                       d_state_in, d_state_out, d_pcm, static_cast<void*>(aux));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !zones || d_stamps) return e;
  // the zone launch: the exact v4 kernel over the list, its waves taking zone
  // after zone; one workgroup of 8 waves per MP3G_ZONE_CHUNKS_PER_WG chunks of
  // the launch, at most two per CU (an empty list ends every workgroup at
  // once: the fewer, the cheaper -- c2's 4,096 chunks get 128)
  const uint32_t blocks = std::max(16u, std::min<uint32_t>(n_chunks / MP3G_ZONE_CHUNKS_PER_WG, 512u));
  hipLaunchKernelGGL(v4::granule_wexact_kernel<true>, dim3(blocks), dim3(64 * v4::kXWaves), 0, stream,
                     reinterpret_cast<const ChunkDesc*>(aux + 8), zones->cap, d_gran, d_coef, d_state_in,
                     d_state_out, d_pcm, aux);
  e = hipGetLastError();
  // the fast kernel ran (or will) and may have listed zones that no zone
  // launch will empty: reset the count and done words behind it on the
  // stream, so that the next launch does not decode stale zones into its own
  // buffers (the error is returned either way)
  if (e != hipSuccess) (void)hipMemsetAsync(aux, 0, 2 * sizeof(uint32_t), stream);
  return e;
}

hipError_t wexact_kernel_attributes(hipFuncAttributes* a, int* waves_per_block) {
  *waves_per_block = v4::kXWaves;
  return hipFuncGetAttributes(a, reinterpret_cast<const void*>(&v4::granule_wexact_kernel<false>));
}

hipError_t launch_wexact(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                         const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out,
                         int16_t* d_pcm, hipStream_t stream) {
  if (n_chunks == 0) return hipSuccess;
  const dim3 grid((n_chunks + v4::kXWaves - 1) / v4::kXWaves), block(64 * v4::kXWaves);
  hipLaunchKernelGGL(v4::granule_wexact_kernel<false>, grid, block, 0, stream, d_chunks, n_chunks, d_gran, d_coef,
                     d_state_in, d_state_out, d_pcm, nullptr);
  return hipGetLastError();
}

hipError_t launch_synth(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran, const float* d_lines,
                        const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm, hipStream_t stream) {
  if (n_chunks == 0) return hipSuccess;
  const dim3 grid((n_chunks + v3::kSynthWaves - 1) / v3::kSynthWaves), block(64 * v3::kSynthWaves);
  hipLaunchKernelGGL(v3::granule_synth_kernel, grid, block, 0, stream, d_chunks, n_chunks, d_gran, d_lines, d_state_in,
                     d_state_out, d_pcm);
  return hipGetLastError();
}

hipError_t launch_fast_stamped(const ChunkDesc* d_chunks, uint32_t n_chunks, const mp3g_granule* d_gran,
                               const int16_t* d_coef, const mp3g_state* d_state_in, mp3g_state* d_state_out,
                               int16_t* d_pcm, unsigned long long* d_stamps, hipStream_t stream) {
  return launch_fast(d_chunks, n_chunks, d_gran, d_coef, d_state_in, d_state_out, d_pcm, d_stamps, nullptr, false,
                     stream);
}

}  // namespace mp3g
