// pk.h -- packed float pairs for the fast kernel's transforms (gfx950
// v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two float32 lanes per VGPR
// pair, either half of a source selectable by op_sel).  Complex values are
// (re, im); __host__ __device__ so the transforms also build for the CPU
// tests (tests/native/*.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

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

// The twiddles and the (-i) rotations below, on the device, as single
// VOP3P instructions whose source modifiers do the shuffling: one SGPR pair
// (c, s) per twiddle read as (c, s), (s, c), (c, -s) or (s, -c) through
// op_sel / op_sel_hi / neg_hi (tools/pk_opsel.hip checks gfx950 honours them
// on SGPR sources), and a + (-i) b as one v_pk_add_f32.  Left to the
// compiler, each twiddle took two constant pairs (four s_mov_b32) and each
// (-i) rotation a v_xor + v_mov before its add.
#if defined(__HIP_DEVICE_COMPILE__)
MP3G_PK uint64_t cpair(float c, float s) {
  return (uint64_t)__builtin_bit_cast(uint32_t, s) << 32 | __builtin_bit_cast(uint32_t, c);
}
#endif

// a + (-i) b = (a.x + b.y, a.y - b.x)
MP3G_PK f2 add_mi(f2 a, f2 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return a + mulmi(b);
#endif
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
MP3G_PK f2 sub_mi(f2 a, f2 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return a - mulmi(b);
#endif
}

// t + k (-i) d = (t.x + k d.y, t.y - k d.x); kNeg: t - k (-i) d
template <bool kNeg>
MP3G_PK f2 fma_mi(float k, f2 d, f2 t) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t kk = cpair(k, k);
  f2 r;
  if constexpr (kNeg)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0]"
        : "=v"(r)
        : "v"(d), "s"(kk), "v"(t));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[1,0,0]"
        : "=v"(r)
        : "v"(d), "s"(kk), "v"(t));
  return r;
#else
  return fma2(mk(kNeg ? -k : k, kNeg ? -k : k), mulmi(d), t);
#endif
}

// (r + is) * (c + id)
MP3G_PK f2 cmul(f2 z, float c, float d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t cd = cpair(c, d);
  f2 t, r;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"  // (r c, r d)
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"  // + (-s d, s c)
      : "=v"(r), "=&v"(t)
      : "v"(z), "s"(cd));
  return r;
#else
  return fma2(bhi(z), mk(-d, c), blo(z) * mk(c, d));
#endif
}
// pre-twiddle of a DCT-IV: (a + ib) e^{-i theta} = a (c, -s) + b (s, c), (c, s) = (cos, sin) theta
MP3G_PK f2 pre_tw(float a, float b, float c, float s) { return fma2(mk(b, b), mk(s, c), mk(a, a) * mk(c, -s)); }
// the same with a = A[HA], b = B[HB] (halves of two pairs)
template <int HA, int HB>
MP3G_PK f2 pre_tw2(f2 A, f2 B, float c, float s) {
  static_assert((HA == 0 || HA == 1) && (HB == 0 || HB == 1), "half");
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(HA == 0 && HB == 1, "the halves the transforms use");
  // t = (a c, -a s); r = (b s, b c) + t -- one statement: hipcc pads a wait
  // state after every inline asm whose outputs a VALU reads next, so the
  // product and the FMA share a block (a VALU result feeding the next VALU
  // needs no wait state of its own)
  const uint64_t cs = cpair(c, s);
  f2 t, r;
  asm("v_pk_mul_f32 %1, %2, %4 op_sel_hi:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_fma_f32 %0, %3, %4, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1]"
      : "=v"(r), "=&v"(t)
      : "v"(A), "v"(B), "s"(cs));
  return r;
#else
  return pre_tw(HA ? A.y : A.x, HB ? B.y : B.x, c, s);
#endif
}
// post-twiddle of a DCT-IV, leaving (Re, -Im) of v e^{-i theta} = vr (c, s) + vi (s, -c)
MP3G_PK f2 post_tw(f2 v, float c, float s) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t cs = cpair(c, s);
  f2 t, r;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"  // (vr c, vr s)
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[0,1,0]"  // + (vi s, -vi c)
      : "=v"(r), "=&v"(t)
      : "v"(v), "s"(cs));
  return r;
#else
  return fma2(bhi(v), mk(s, -c), blo(v) * mk(c, s));
#endif
}

}  // namespace pk
}  // namespace mp3g
