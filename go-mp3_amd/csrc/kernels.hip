// kernels.hip -- device translation unit of the exact-mode and main-data
// kernels of libmp3g.so.
//
// Holds their constant tables (uploaded once per device), the workgroup
// exact-mode kernel v2 (granule_fused.hip), kept as the on-device cross-check
// of the default exact kernel v4 (kernels_fast.hip; the per-phase v1 was
// retired in round 4), and the main-data (scale factor + Huffman) kernel
// (huffman_dev.hip).  One TU so they reach g_tab / g_huff without
// relocatable device code.  The fast-mode kernel v3 has a TU of its own
// (kernels_fast.hip: its own table copy g_fast and codegen options).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>

#include "../../include/mp3g.h"
#include "dsp_tables.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace mp3g {
__device__ DspTables g_tab;
__device__ HuffLut g_huff;
}  // namespace mp3g

#include "granule_common.hip"
#include "granule_fused.hip"
#include "huffman_dev.hip"

namespace mp3g {

hipError_t upload_tables(const DspTables& tables) {
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_tab), &tables, sizeof(DspTables), 0, hipMemcpyHostToDevice);
  if (e != hipSuccess) return e;
  // (54 KB: on the heap, not on the stack of whichever thread first uses the device)
  FastTables* fast = new (std::nothrow) FastTables;
  if (!fast) return hipErrorOutOfMemory;
  build_fast_tables(tables, fast);
  e = upload_fast_tables(*fast, &tables.req[0][0]);
  delete fast;
  if (e != hipSuccess) return e;
  HuffLut* lut = new HuffLut;
  if (!build_huff_lut(lut)) {
    delete lut;
    return hipErrorInvalidValue;
  }
  e = hipMemcpyToSymbol(HIP_SYMBOL(g_huff), lut, sizeof(HuffLut), 0, hipMemcpyHostToDevice);
  delete lut;
  return e;
}

// PCM copy-out into device-accessible pinned host memory: 16 B per lane,
// non-temporal.  HIP's own device -> host hipMemcpyAsync runs on a DMA engine
// at ~30 GB/s on MI355X; this kernel writes the same pinned buffer at
// 54-55 GB/s from as few as 16 CUs (tools/copy_exp.hip), so the pipelined
// drop-in runs it on a stream limited to a few CUs beside the decode kernels.
typedef unsigned int copy_u4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) pcm_copy_out_kernel(const copy_u4* __restrict__ src, copy_u4* __restrict__ dst,
                                                           size_t n16) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(src[i], &dst[i]);
}

hipError_t launch_copy_out(const void* d_src, void* dst, size_t bytes, int blocks, hipStream_t stream) {
  if (!bytes) return hipSuccess;
  hipLaunchKernelGGL(pcm_copy_out_kernel, dim3(std::max(1, blocks)), dim3(256), 0, stream,
                     static_cast<const copy_u4*>(d_src), static_cast<copy_u4*>(dst), bytes / 16);
  return hipGetLastError();
}

// Shader clock under load (diagnostic, mp3g_debug_clock_probe): one wave per
// workgroup spins beside whatever the device runs until *flag turns non-zero
// (or max_ticks of the 100 MHz real-time counter pass) and reports its
// s_memtime (shader cycles) and s_memrealtime at both ends of the window:
// clock = d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS
// item 6).  Lane 0 stores four dwords pairs per workgroup with vector stores.
__global__ void __launch_bounds__(64) clock_probe_kernel(const uint32_t* flag, unsigned long long* out,
                                                         unsigned long long max_ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long r = r0;
  uint32_t seen = 0;
  while (r - r0 < max_ticks) {
    seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen) break;
    __builtin_amdgcn_s_sleep(8);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    unsigned long long* o = out + 5 * blockIdx.x;
    o[0] = t0;
    o[1] = t1;
    o[2] = r0;
    o[3] = r1;
    o[4] = seen;
  }
}

hipError_t launch_clock_probe(const uint32_t* d_flag, unsigned long long* d_out, uint32_t n_waves,
                              unsigned long long max_ticks, hipStream_t stream) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(n_waves), dim3(64), 0, stream, d_flag, d_out, max_ticks);
  return hipGetLastError();
}

int chunks_per_cu(int variant) {
  hipFuncAttributes a;
  hipError_t e;
  int waves_per_block;
  const bool per_wave = variant == kVariantFast || variant == kVariantExact4;
  if (variant == kVariantFast) {
    e = fast_kernel_attributes(&a, &waves_per_block);
  } else if (variant == kVariantExact4) {
    e = wexact_kernel_attributes(&a, &waves_per_block);
  } else {
    e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&v2::granule_fused_kernel));
    waves_per_block = 4;
  }
  if (e != hipSuccess || a.numRegs <= 0) return 1;
  // MI355X_MICROARCH.md: 512 VGPRs per lane per SIMD in granules of 8, four
  // SIMDs and 160 KiB of LDS per CU, at most 8 waves per SIMD
  const int vgpr = (a.numRegs + 7) / 8 * 8;
  const int waves_per_simd = std::min(8, 512 / vgpr);
  int blocks = waves_per_simd * 4 / waves_per_block;
  if (a.sharedSizeBytes > 0) blocks = std::min<int>(blocks, (int)(163840 / a.sharedSizeBytes));
  blocks = std::max(blocks, 1);
  return per_wave ? blocks * waves_per_block : blocks;
}

hipError_t launch_granule(int variant, const ChunkDesc* d_chunks, uint32_t n_chunks,
                          const mp3g_granule* d_gran, const int16_t* d_coef,
                          const mp3g_state* d_state_in, mp3g_state* d_state_out, int16_t* d_pcm,
                          const ZoneScratch* zones, bool hot_stats, hipStream_t stream) {
  if (n_chunks == 0) return hipSuccess;
  if (variant == kVariantFast)
    return launch_fast(d_chunks, n_chunks, d_gran, d_coef, d_state_in, d_state_out, d_pcm, nullptr, zones, hot_stats,
                       stream);
  if (variant == kVariantExact4)
    return launch_wexact(d_chunks, n_chunks, d_gran, d_coef, d_state_in, d_state_out, d_pcm, stream);
  hipLaunchKernelGGL(v2::granule_fused_kernel, dim3(n_chunks), dim3(256), 0, stream, d_chunks,
                     d_gran, d_coef, d_state_in, d_state_out, d_pcm);
  return hipGetLastError();
}

}  // namespace mp3g
