// dct32.h -- the polyphase matrixing of the fast kernel as a fast DCT-II of
// size 32, evaluated inside one lane on packed float pairs (granule_fast.hip).
//
// The reference computes V = synthNWin * S, a 64 x 32 matrix-vector product
// per time slot (internal/frame/frame.go:488-497, :642-648).  V has only 32
// distinct values (dsp_tables.h FastTables):
//   X[m] = sum_k S[k] cos(pi m (2k+1) / 64),  m = 0..31,
// the unnormalised DCT-II of S, with V[i] = X[16+i] (i < 16), 0 (i = 16),
// -X[48-i] (16 < i < 48), -X[i-48] (i >= 48).  Here X comes out of the
// standard recursive split
//   DCT2_N(x)[2t]   = DCT2_N/2(x[q] + x[N-1-q])[t]
//   DCT2_N(x)[2t+1] = DCT4_N/2(x[q] - x[N-1-q])[t]
// with DCT4_M(y)[t] = sum_q y[q] cos(pi (2t+1)(2q+1) / 4M) as a pre-twiddle,
// an M/2-point complex FFT and a post-twiddle (M = 16, 8), and DCT4_4,
// DCT2_4 directly: ~250 flops per slot instead of the 32 x 16 multiply-adds
// of the folded direct form.  Every step operates on float pairs (complex
// values as (re, im), real values as neighbours), so on gfx950 it is ~130
// v_pk_* instructions.  Reassociated like the rest of the fast mode (+-1 LSB
// of PCM; tests/test_dct32.py checks it against float64).
//
// Output order: X leaves as 16 pairs (kPairM[t][0], kPairM[t][1]); the fast
// kernel stores pair t in ring columns kColX[t], kColY[t] (kPosOfM: X[m]'s column).
#pragma once
#include <hip/hip_runtime.h>

#include "pk.h"

namespace mp3g {
namespace dct32 {

using pk::blo;
using pk::bhi;
using pk::f2;
using pk::fma2;
using pk::mk;
using pk::add_mi;
using pk::sub_mi;
using pk::swp;

#define MP3G_D32 __host__ __device__ __forceinline__

// m of the two values of output pair t
constexpr int kPairM[16][2] = {{1, 31},  {5, 27},  {9, 23},  {13, 19}, {17, 15}, {21, 11}, {25, 7},  {29, 3},
                               {2, 30},  {10, 22}, {18, 14}, {26, 6},  {4, 12},  {20, 28}, {0, 16},  {8, 24}};
// Positions in the fast kernel's ring column set (32 columns, 34 dwords
// apart, granule_fast.hip): pair t goes to columns (kColX[t], kColY[t]), so
// X[m] sits in column kPosOfM[m].  The window's odd taps read X[0..16] in one
// column each; 34c mod 32 = 2c mod 32 puts columns c and c + 16 in one bank,
// and this assignment gives those 17 values 16 distinct banks (one pair
// shares: 17 > 16).
constexpr int kColX[16] = {18, 4, 21, 6, 22, 9, 24, 11, 27, 12, 28, 15, 0, 16, 2, 31};
constexpr int kColY[16] = {19, 5, 20, 7, 23, 8, 25, 10, 26, 13, 29, 14, 1, 17, 3, 30};
constexpr int kPosOfM[32] = {2,  18, 27, 10, 0,  4,  14, 25, 31, 21, 12, 8,  1, 6,  29, 23,
                             3,  22, 28, 7,  16, 9,  13, 20, 30, 24, 15, 5,  17, 11, 26, 19};

// Twiddles, float literals: e^{-i pi (4n+1)/64} (pre, DCT4_16), e^{-i pi k/16}
// (post, DCT4_16), e^{-i pi (4n+1)/32} and e^{-i pi k/8} (DCT4_8): (cos, sin).
constexpr float kPre16[8][2] = {{9.987954562e-01f, 4.906767433e-02f}, {9.700312532e-01f, 2.429801799e-01f},
                                {9.039892931e-01f, 4.275550934e-01f}, {8.032075315e-01f, 5.956993045e-01f},
                                {6.715589548e-01f, 7.409511254e-01f}, {5.141027442e-01f, 8.577286100e-01f},
                                {3.368898534e-01f, 9.415440652e-01f}, {1.467304745e-01f, 9.891765100e-01f}};
constexpr float kPost16[8][2] = {{1.000000000e+00f, 0.000000000e+00f}, {9.807852804e-01f, 1.950903220e-01f},
                                 {9.238795325e-01f, 3.826834324e-01f}, {8.314696123e-01f, 5.555702330e-01f},
                                 {7.071067812e-01f, 7.071067812e-01f}, {5.555702330e-01f, 8.314696123e-01f},
                                 {3.826834324e-01f, 9.238795325e-01f}, {1.950903220e-01f, 9.807852804e-01f}};
constexpr float kPre8[4][2] = {{9.951847267e-01f, 9.801714033e-02f}, {8.819212643e-01f, 4.713967368e-01f},
                               {6.343932842e-01f, 7.730104534e-01f}, {2.902846773e-01f, 9.569403357e-01f}};
constexpr float kPost8[4][2] = {{1.000000000e+00f, 0.000000000e+00f}, {9.238795325e-01f, 3.826834324e-01f},
                                {7.071067812e-01f, 7.071067812e-01f}, {3.826834324e-01f, 9.238795325e-01f}};
// DCT4_4: cos(pi (2t+1)(2q+1) / 16), [q][t]
constexpr float kC4[4][4] = {{9.807852804e-01f, 8.314696123e-01f, 5.555702330e-01f, 1.950903220e-01f},
                             {8.314696123e-01f, -1.950903220e-01f, -9.807852804e-01f, -5.555702330e-01f},
                             {5.555702330e-01f, -9.807852804e-01f, 1.950903220e-01f, 8.314696123e-01f},
                             {1.950903220e-01f, -5.555702330e-01f, 8.314696123e-01f, -9.807852804e-01f}};
constexpr float kR2 = 7.071067812e-01f;   // cos(pi/4)
constexpr float kC1 = 9.238795325e-01f;   // cos(pi/8)
constexpr float kC3 = 3.826834324e-01f;   // cos(3 pi/8)

// in-place 4-point complex FFT (forward) of z0..z3
MP3G_D32 void fft4(f2& z0, f2& z1, f2& z2, f2& z3) {
  const f2 e0 = z0 + z2, e1 = z0 - z2, o0 = z1 + z3, d = z1 - z3;
  z0 = e0 + o0;
  z2 = e0 - o0;
  z1 = add_mi(e1, d);  // e1 + (-i) d
  z3 = sub_mi(e1, d);
}

// DCT4_16 of d (pairs dp[j] = (d[2j], d[2j+1])) -> 8 output pairs
MP3G_D32 void dct4_16(const f2 dp[8], f2 out[8]) {
  f2 v[8];
#pragma unroll
  for (int n = 0; n < 8; n++) v[n] = pk::pre_tw2<0, 1>(dp[n], dp[7 - n], kPre16[n][0], kPre16[n][1]);
  // 8-point FFT, decimation in time: E = FFT4(v even), O = FFT4(v odd)
  fft4(v[0], v[2], v[4], v[6]);
  fft4(v[1], v[3], v[5], v[7]);
  // V[k] = E[k] + W8^k O[k], V[k+4] = E[k] - W8^k O[k]; W8 = (1 - i)/sqrt2
  // (o2 = (-i) v5 and o3 = (-i) w7 ride on the adds: add_mi / sub_mi)
  const f2 o0 = v[1];
  const f2 o1 = add_mi(v[3], v[3]) * mk(kR2, kR2);
  const f2 w7 = add_mi(v[7], v[7]) * mk(kR2, kR2);
  const f2 V[8] = {v[0] + o0,          v[2] + o1, add_mi(v[4], v[5]), add_mi(v[6], w7),
                   v[0] - o0,          v[2] - o1, sub_mi(v[4], v[5]), sub_mi(v[6], w7)};
#pragma unroll
  for (int k = 0; k < 8; k++) out[k] = pk::post_tw(V[k], kPost16[k][0], kPost16[k][1]);
}

// DCT4_8 of b (pairs bp[j] = (b[2j], b[2j+1])) -> 4 output pairs (X[2k], X[7-2k])
MP3G_D32 void dct4_8(const f2 bp[4], f2 out[4]) {
  f2 v[4];
#pragma unroll
  for (int n = 0; n < 4; n++) v[n] = pk::pre_tw2<0, 1>(bp[n], bp[3 - n], kPre8[n][0], kPre8[n][1]);
  fft4(v[0], v[1], v[2], v[3]);
#pragma unroll
  for (int k = 0; k < 4; k++) out[k] = pk::post_tw(v[k], kPost8[k][0], kPost8[k][1]);
}

// X[m] = sum_k S[k] cos(pi m (2k+1) / 64) for one slot.  sp[j] = (S[2j], S[2j+1]);
// out(t, xp) receives pair t = (X[kPairM[t][0]], X[kPairM[t][1]]) as soon as it
// is computed (the caller stores it: fewer values live at once).
template <class Out>
MP3G_D32 void dct2_32_to(const f2 sp[16], Out out) {
  // fold 32 -> even part e (DCT2_16) and odd part d (DCT4_16)
  f2 ep[8], dp[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const f2 r = swp(sp[15 - j]);  // (S[31-2j], S[30-2j])
    ep[j] = sp[j] + r;
    dp[j] = sp[j] - r;
  }
  {
    f2 x4[8];
    dct4_16(dp, x4);  // pairs 0..7: m = 4k+1, 31-4k
#pragma unroll
    for (int t = 0; t < 8; t++) out(t, x4[t]);
  }
  // DCT2_16(e): fold -> a (DCT2_8), b (DCT4_8)
  f2 ap[4], bp[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const f2 r = swp(ep[7 - j]);
    ap[j] = ep[j] + r;
    bp[j] = ep[j] - r;
  }
  {
    f2 x8[4];
    dct4_8(bp, x8);  // pairs 8..11: m = 8k+2, 30-8k
#pragma unroll
    for (int t = 0; t < 4; t++) out(8 + t, x8[t]);
  }
  // DCT2_8(a): fold -> a' (DCT2_4), a'' (DCT4_4)
  const f2 r1 = swp(ap[3]), r0 = swp(ap[2]);
  const f2 a1p0 = ap[0] + r1, a1p1 = ap[1] + r0;  // a'[0..3] as pairs
  const f2 a2p0 = ap[0] - r1, a2p1 = ap[1] - r0;  // a''[0..3]
  // DCT4_4(a'') direct: pairs (Y0, Y1) -> m = 4, 12 and (Y2, Y3) -> m = 20, 28
  {
    f2 y01 = mk(a2p0.x, a2p0.x) * mk(kC4[0][0], kC4[0][1]);
    f2 y23 = mk(a2p0.x, a2p0.x) * mk(kC4[0][2], kC4[0][3]);
    y01 = fma2(bhi(a2p0), mk(kC4[1][0], kC4[1][1]), y01);
    y23 = fma2(bhi(a2p0), mk(kC4[1][2], kC4[1][3]), y23);
    y01 = fma2(blo(a2p1), mk(kC4[2][0], kC4[2][1]), y01);
    y23 = fma2(blo(a2p1), mk(kC4[2][2], kC4[2][3]), y23);
    y01 = fma2(bhi(a2p1), mk(kC4[3][0], kC4[3][1]), y01);
    y23 = fma2(bhi(a2p1), mk(kC4[3][2], kC4[3][3]), y23);
    out(12, y01);
    out(13, y23);
  }
  // DCT2_4(a'): fold -> u (DCT2_2: m = 0, 16), w (DCT4_2: m = 8, 24)
  const f2 u = a1p0 + swp(a1p1);  // (a'0 + a'3, a'1 + a'2)
  const f2 w = a1p0 - swp(a1p1);  // (a'0 - a'3, a'1 - a'2)
  out(14, (blo(u) + mk(u.y, -u.y)) * mk(1.0f, kR2));
  out(15, fma2(bhi(w), mk(kC3, -kC1), blo(w) * mk(kC1, kC3)));
}

MP3G_D32 void dct2_32(const f2 sp[16], f2 xp[16]) {
  dct2_32_to(sp, [&](int t, f2 v) { xp[t] = v; });
}

}  // namespace dct32
}  // namespace mp3g
