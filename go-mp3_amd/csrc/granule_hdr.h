// granule_hdr.h -- frame-header fields the granule kernels read
// (internal/frameheader/frameheader.go:82-137).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mp3g {
namespace common {

__device__ __forceinline__ int hdr_mode(uint32_t h) { return (int)((h >> 6) & 3u); }
__device__ __forceinline__ int hdr_nch(uint32_t h) { return hdr_mode(h) == 3 ? 1 : 2; }
// line-table combination: lsf * 3 + sampling-frequency index (consts.go:68-97)
__device__ __forceinline__ int hdr_combo(uint32_t h) {
  const int lsf = ((h >> 19) & 3u) == 3u ? 0 : 1;
  int sf = (int)((h >> 10) & 3u);
  sf = sf > 2 ? 2 : sf;
  return lsf * 3 + sf;
}

}  // namespace common
}  // namespace mp3g
