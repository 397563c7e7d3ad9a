// pk.h -- packed float pairs for the fast kernel's transforms (gfx950
// v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two float32 lanes per VGPR
// pair, either half of a source selectable by op_sel).  Complex values are
// (re, im); __host__ __device__ so the transforms also build for the CPU
// tests (tests/native/*.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace mp3g {
namespace pk {

typedef float f2 __attribute__((ext_vector_type(2)));

#define MP3G_PK __host__ __device__ __forceinline__

MP3G_PK f2 mk(float a, float b) { return (f2){a, b}; }
MP3G_PK f2 swp(f2 v) { return __builtin_shufflevector(v, v, 1, 0); }
MP3G_PK f2 blo(f2 v) { return __builtin_shufflevector(v, v, 0, 0); }
MP3G_PK f2 bhi(f2 v) { return __builtin_shufflevector(v, v, 1, 1); }
MP3G_PK f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// (-i) * (x + iy) = y - ix
MP3G_PK f2 mulmi(f2 v) { return mk(v.y, -v.x); }
// (r + is) * (c + id)
MP3G_PK f2 cmul(f2 z, float c, float d) { return fma2(bhi(z), mk(-d, c), blo(z) * mk(c, d)); }
// pre-twiddle of a DCT-IV: (a + ib) e^{-i theta} = a (c, -s) + b (s, c), (c, s) = (cos, sin) theta
MP3G_PK f2 pre_tw(float a, float b, float c, float s) { return fma2(mk(b, b), mk(s, c), mk(a, a) * mk(c, -s)); }
// post-twiddle of a DCT-IV, leaving (Re, -Im) of v e^{-i theta} = vr (c, s) + vi (s, -c)
MP3G_PK f2 post_tw(f2 v, float c, float s) { return fma2(bhi(v), mk(s, -c), blo(v) * mk(c, s)); }

}  // namespace pk
}  // namespace mp3g
