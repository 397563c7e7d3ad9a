// xlane.h -- cross-lane moves of a 64-lane wave on gfx950 without the LDS
// crossbar (ds_bpermute): DPP row/wave controls and the CDNA4 permlane swaps
// are VALU operations, so none of them waits on lgkmcnt.
#pragma once
#include <hip/hip_runtime.h>

namespace mp3g {
namespace xl {

__device__ __forceinline__ int dpp_ctrl_wave_shr1() { return 0x138; }

// value of lane l-1 (lane 0: 0).  bound_ctrl writes the 0 of the lane with
// no source itself (an "old" operand of 0 instead costs a v_mov per use)
__device__ __forceinline__ float from_prev(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
// value of lane l+1 (lane 63: 0)
__device__ __forceinline__ float from_next(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
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

// DPP row_ror:n (1 <= n <= 15, compile-time): lane r of each 16-lane row gets
// lane (r - n) & 15 of the same row
template <int N>
__device__ __forceinline__ float row_ror_c(float v) {
  // mov_dpp (no "old" operand) with bound_ctrl: lets the DPP combine fold the
  // move into the consuming VOP2 FMA (every source lane of a rotation is valid)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x120 + N, 0xf, 0xf, true));
}
__device__ __forceinline__ float row_ror(float v, int n) {
  switch (n) {
    case 1: return row_ror_c<1>(v);
    case 2: return row_ror_c<2>(v);
    case 3: return row_ror_c<3>(v);
    case 4: return row_ror_c<4>(v);
    case 5: return row_ror_c<5>(v);
    case 6: return row_ror_c<6>(v);
    case 7: return row_ror_c<7>(v);
    case 8: return row_ror_c<8>(v);
    case 9: return row_ror_c<9>(v);
    case 10: return row_ror_c<10>(v);
    case 11: return row_ror_c<11>(v);
    case 12: return row_ror_c<12>(v);
    case 13: return row_ror_c<13>(v);
    case 14: return row_ror_c<14>(v);
    default: return row_ror_c<15>(v);
  }
}

// acc{x,y}[n & 1] += row_ror(e{x,y}, n) * c[n] for n = 1..15 as v_fmac_f32_dpp
// (the compiler does not fold the rotation into the FMA on gfx950; a separate
// v_mov_b32_dpp per term doubles the VALU cost).  The leading s_nop covers
// the VALU-write -> DPP-read hazard of ex / ey, which the asm then only reads.
__device__ __forceinline__ void rot_fma15(float& ax0, float& ax1, float& ay0, float& ay1, float ex, float ey,
                                          const float c[16]) {
  asm volatile(
      "s_nop 1\n"
      "v_fmac_f32_dpp %1, %4, %6 row_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %6 row_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %0, %4, %7 row_ror:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %2, %5, %7 row_ror:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %1, %4, %8 row_ror:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %8 row_ror:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %0, %4, %9 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %2, %5, %9 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %1, %4, %10 row_ror:5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %10 row_ror:5 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %0, %4, %11 row_ror:6 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %2, %5, %11 row_ror:6 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %1, %4, %12 row_ror:7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %12 row_ror:7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %0, %4, %13 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %2, %5, %13 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %1, %4, %14 row_ror:9 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %14 row_ror:9 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %0, %4, %15 row_ror:10 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %2, %5, %15 row_ror:10 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %1, %4, %16 row_ror:11 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %16 row_ror:11 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %0, %4, %17 row_ror:12 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %2, %5, %17 row_ror:12 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %1, %4, %18 row_ror:13 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %18 row_ror:13 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %0, %4, %19 row_ror:14 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %2, %5, %19 row_ror:14 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %1, %4, %20 row_ror:15 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_fmac_f32_dpp %3, %5, %20 row_ror:15 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      : "+v"(ax0), "+v"(ax1), "+v"(ay0), "+v"(ay1)
      : "v"(ex), "v"(ey), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7]), "v"(c[8]),
        "v"(c[9]), "v"(c[10]), "v"(c[11]), "v"(c[12]), "v"(c[13]), "v"(c[14]), "v"(c[15]));
}

}  // namespace xl
}  // namespace mp3g
