// xlane.h -- cross-lane moves of a 64-lane wave on gfx950 without the LDS
// crossbar (ds_bpermute): DPP row/wave controls and the CDNA4 permlane swaps
// are VALU operations, so none of them waits on lgkmcnt.
#pragma once
#include <hip/hip_runtime.h>

namespace mp3g {
namespace xl {

__device__ __forceinline__ int dpp_ctrl_wave_shr1() { return 0x138; }

// value of lane l-1 (lane 0: 0)
__device__ __forceinline__ float from_prev(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
}
// value of lane l+1 (lane 63: 0)
__device__ __forceinline__ float from_next(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
}
// value of lane l^32 (the other half-wave): v_permlane32_swap swaps the upper
// half of its first operand with the lower half of its second.
__device__ __forceinline__ float xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
__device__ __forceinline__ int xor32i(int v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}
// value of lane l^31 (mirror inside each half-wave): row_mirror reverses each
// 16-lane row, v_permlane16_swap exchanges rows 0<->1 and 2<->3.
__device__ __forceinline__ float xor31(float v) {
  const int m = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xf, 0xf, false);
  const auto r = __builtin_amdgcn_permlane16_swap(m, m, false, false);
  return __int_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}

}  // namespace xl
}  // namespace mp3g
