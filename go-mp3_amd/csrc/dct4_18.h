// dct4_18.h -- IMDCT constants of the fast kernel: the 18-point DCT-IV for long blocks
// (granule_fast.hip).  The reference's IMDCT-36 (imdct.go:21-108) sums
// x[m] cosN36[m][p] over m = 0..17 directly; its 18 distinct outputs are a
// DCT-IV of size 18,
//   X[k] = sum_m x[m] cos(pi/72 (2k+1)(2m+1)),
// with out[q] = X[9+q] and out[18+q] = -X[8-q] (q = 0..8).  Here it runs as
// the standard half-length complex FFT form -- pre-twiddle, 9-point FFT (3x3
// Cooley-Tukey), post-twiddle -- with every constant an instruction literal:
// no coefficient table, so none of the 81 broadcast LDS reads per granule the
// direct form needs (the fast kernel is LDS-bound).  Reassociated like the
// rest of the fast mode (+-1 LSB of PCM).
#pragma once
#include <hip/hip_runtime.h>

#include "pk.h"

namespace mp3g {
namespace dct4 {

// pre-twiddles e^{-i pi (4n+1)/72}: (cos, sin)
constexpr float kPre[9][2] = {{9.990482216e-01f, 4.361938737e-02f}, {9.762960071e-01f, 2.164396139e-01f},
                              {9.238795325e-01f, 3.826834324e-01f}, {8.433914458e-01f, 5.372996083e-01f},
                              {7.372773368e-01f, 6.755902076e-01f}, {6.087614290e-01f, 7.933533403e-01f},
                              {4.617486132e-01f, 8.870108332e-01f}, {3.007057995e-01f, 9.537169507e-01f},
                              {1.305261922e-01f, 9.914448614e-01f}};
// post-twiddles e^{-i pi k/18}: (cos, sin)
constexpr float kPost[9][2] = {{1.000000000e+00f, 0.000000000e+00f}, {9.848077530e-01f, 1.736481777e-01f},
                               {9.396926208e-01f, 3.420201433e-01f}, {8.660254038e-01f, 5.000000000e-01f},
                               {7.660444431e-01f, 6.427876097e-01f}, {6.427876097e-01f, 7.660444431e-01f},
                               {5.000000000e-01f, 8.660254038e-01f}, {3.420201433e-01f, 9.396926208e-01f},
                               {1.736481777e-01f, 9.848077530e-01f}};
// FFT-9 twiddles W^e = e^{-2 pi i e/9} for e = n2 * k1 = 1, 2, 4: (cos, sin)
constexpr float kW[3][2] = {{7.660444431e-01f, -6.427876097e-01f},
                            {1.736481777e-01f, -9.848077530e-01f},
                            {-9.396926208e-01f, -3.420201433e-01f}};
constexpr float kH = 8.660254038e-01f;  // sqrt(3)/2

// 3-point DFT (W3 = e^{-2 pi i/3}) of (a, b, c), in place
__host__ __device__ __forceinline__ void dft3(float& ar, float& ai, float& br, float& bi, float& cr, float& ci) {
  const float sr = br + cr, si = bi + ci, dr = br - cr, di = bi - ci;
  const float tr = __builtin_fmaf(-0.5f, sr, ar), ti = __builtin_fmaf(-0.5f, si, ai);
  ar += sr;
  ai += si;
  br = __builtin_fmaf(kH, di, tr);
  bi = __builtin_fmaf(-kH, dr, ti);
  cr = __builtin_fmaf(-kH, di, tr);
  ci = __builtin_fmaf(kH, dr, ti);
}

// (r + i s) *= (c + i d)
__host__ __device__ __forceinline__ void cmul(float& r, float& s, float c, float d) {
  const float nr = __builtin_fmaf(r, c, -s * d);
  s = __builtin_fmaf(r, d, s * c);
  r = nr;
}

// X[k] = sum_m x[m] cos(pi/72 (2k+1)(2m+1)), k = 0..17
__host__ __device__ __forceinline__ void dct4_18(const float x[18], float X[18]) {
  float zr[9], zi[9];
#pragma unroll
  for (int n = 0; n < 9; n++) {  // (x[2n] + i x[17-2n]) e^{-i pi (4n+1)/72}
    const float a = x[2 * n], b = x[17 - 2 * n], c = kPre[n][0], s = kPre[n][1];
    zr[n] = __builtin_fmaf(a, c, b * s);
    zi[n] = __builtin_fmaf(b, c, -a * s);
  }
  // 9-point FFT, n = 3 n1 + n2, k = k1 + 3 k2: DFT-3 over n1, twiddle W^(n2 k1), DFT-3 over n2
#pragma unroll
  for (int n2 = 0; n2 < 3; n2++) dft3(zr[n2], zi[n2], zr[3 + n2], zi[3 + n2], zr[6 + n2], zi[6 + n2]);
  // z[3 k1 + n2] now holds T[n2][k1]
  cmul(zr[4], zi[4], kW[0][0], kW[0][1]);  // n2 = 1, k1 = 1: W^1
  cmul(zr[7], zi[7], kW[1][0], kW[1][1]);  // n2 = 1, k1 = 2: W^2
  cmul(zr[5], zi[5], kW[1][0], kW[1][1]);  // n2 = 2, k1 = 1: W^2
  cmul(zr[8], zi[8], kW[2][0], kW[2][1]);  // n2 = 2, k1 = 2: W^4
#pragma unroll
  for (int k1 = 0; k1 < 3; k1++)
    dft3(zr[3 * k1], zi[3 * k1], zr[3 * k1 + 1], zi[3 * k1 + 1], zr[3 * k1 + 2], zi[3 * k1 + 2]);
  // z[3 k1 + k2] = Y[k1 + 3 k2]; X[2k] = Re(Y_k e^{-i pi k/18}), X[17-2k] = -Im(...)
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int at = 3 * (k % 3) + k / 3;
    const float yr = zr[at], yi = zi[at], c = kPost[k][0], s = kPost[k][1];
    X[2 * k] = __builtin_fmaf(yr, c, yi * s);
    X[17 - 2 * k] = __builtin_fmaf(yr, s, -yi * c);
  }
}

// The same transform on packed float pairs (pk.h; ~80 v_pk_* instead of ~160
// scalar operations): P[k] = (X[2k], X[17-2k]), k = 0..8.
__host__ __device__ __forceinline__ void dft3p(pk::f2& a, pk::f2& b, pk::f2& c) {
  const pk::f2 s = b + c, d = b - c;  // (the (-i) rotation of d rides on the FMAs)
  const pk::f2 t = pk::fma2(pk::mk(-0.5f, -0.5f), s, a);
  a += s;
  b = pk::fma_mi<false>(kH, d, t);  // t + kH (-i) d
  c = pk::fma_mi<true>(kH, d, t);
}
__host__ __device__ __forceinline__ void dct4_18_pk(const float x[18], pk::f2 P[9]) {
  pk::f2 z[9];
#pragma unroll
  for (int n = 0; n < 9; n++) {
    const pk::f2 ab = pk::mk(x[2 * n], x[17 - 2 * n]);
    z[n] = pk::pre_tw2<0, 1>(ab, ab, kPre[n][0], kPre[n][1]);
  }
#pragma unroll
  for (int n2 = 0; n2 < 3; n2++) dft3p(z[n2], z[3 + n2], z[6 + n2]);
  z[4] = pk::cmul(z[4], kW[0][0], kW[0][1]);
  z[7] = pk::cmul(z[7], kW[1][0], kW[1][1]);
  z[5] = pk::cmul(z[5], kW[1][0], kW[1][1]);
  z[8] = pk::cmul(z[8], kW[2][0], kW[2][1]);
#pragma unroll
  for (int k1 = 0; k1 < 3; k1++) dft3p(z[3 * k1], z[3 * k1 + 1], z[3 * k1 + 2]);
#pragma unroll
  for (int k = 0; k < 9; k++) P[k] = pk::post_tw(z[3 * (k % 3) + k / 3], kPost[k][0], kPost[k][1]);
}

// Short blocks (imdct.go:88-94): the 12-point IMDCT of each window as a
// direct sum with literal coefficients (6 inputs; no table in LDS either).
// cosN12[m][p] of imdct.go as [p][m] (dsp_tables.cpp build_tables values)
constexpr float kCos12[12][6] = {{6.087614298e-01f, -9.238795042e-01f, -1.305261850e-01f, 9.914448857e-01f, -3.826834261e-01f, -7.933533192e-01f},
                                   {3.826834261e-01f, -9.238795042e-01f, 9.238795042e-01f, -3.826834261e-01f, -3.826834261e-01f, 9.238795042e-01f},
                                   {1.305261850e-01f, -3.826834261e-01f, 6.087614298e-01f, -7.933533192e-01f, 9.238795042e-01f, -9.914448857e-01f},
                                   {-1.305261850e-01f, 3.826834261e-01f, -6.087614298e-01f, 7.933533192e-01f, -9.238795042e-01f, 9.914448857e-01f},
                                   {-3.826834261e-01f, 9.238795042e-01f, -9.238795042e-01f, 3.826834261e-01f, 3.826834261e-01f, -9.238795042e-01f},
                                   {-6.087614298e-01f, 9.238795042e-01f, 1.305261850e-01f, -9.914448857e-01f, 3.826834261e-01f, 7.933533192e-01f},
                                   {-7.933533192e-01f, 3.826834261e-01f, 9.914448857e-01f, 1.305261850e-01f, -9.238795042e-01f, -6.087614298e-01f},
                                   {-9.238795042e-01f, -3.826834261e-01f, 3.826834261e-01f, 9.238795042e-01f, 9.238795042e-01f, 3.826834261e-01f},
                                   {-9.914448857e-01f, -9.238795042e-01f, -7.933533192e-01f, -6.087614298e-01f, -3.826834261e-01f, -1.305261850e-01f},
                                   {-9.914448857e-01f, -9.238795042e-01f, -7.933533192e-01f, -6.087614298e-01f, -3.826834261e-01f, -1.305261850e-01f},
                                   {-9.238795042e-01f, -3.826834261e-01f, 3.826834261e-01f, 9.238795042e-01f, 9.238795042e-01f, 3.826834261e-01f},
                                   {-7.933533192e-01f, 3.826834261e-01f, 9.914448857e-01f, 1.305261850e-01f, -9.238795042e-01f, -6.087614298e-01f}};
// the short-block window (imdct.go block type 2)
constexpr float kWin12[12] = {1.305261850e-01f, 3.826834261e-01f, 6.087614298e-01f, 7.933533192e-01f, 9.238795042e-01f, 9.914448857e-01f, 9.914448857e-01f, 9.238795042e-01f, 7.933533192e-01f, 6.087614298e-01f, 3.826834261e-01f, 1.305261850e-01f};

}  // namespace dct4
}  // namespace mp3g
