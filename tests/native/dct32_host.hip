// dct32_host.hip -- TEST INFRASTRUCTURE: the fast kernel's in-lane DCT-II-32
// (go-mp3_amd/csrc/dct32.h, __host__ __device__) compiled for the CPU, so
// tests/test_dct32.py can check it against float64 without a GPU.  Not linked
// into libmp3g.so.
#include "../../go-mp3_amd/csrc/dct32.h"

using mp3g::dct32::f2;

// S[n][32] -> X[n][32] in natural m order
extern "C" void dct32_host(const float* S, float* X, int n) {
  for (int i = 0; i < n; i++) {
    f2 sp[16], xp[16];
    for (int j = 0; j < 16; j++) sp[j] = (f2){S[32 * i + 2 * j], S[32 * i + 2 * j + 1]};
    mp3g::dct32::dct2_32(sp, xp);
    for (int t = 0; t < 16; t++) {
      X[32 * i + mp3g::dct32::kPairM[t][0]] = xp[t].x;
      X[32 * i + mp3g::dct32::kPairM[t][1]] = xp[t].y;
    }
  }
}

// col_m[c] = the m stored in ring column c (from kPairM, kColX, kColY)
extern "C" void dct32_tables(int* col_m, int* pos_of_m) {
  for (int t = 0; t < 16; t++) {
    col_m[mp3g::dct32::kColX[t]] = mp3g::dct32::kPairM[t][0];
    col_m[mp3g::dct32::kColY[t]] = mp3g::dct32::kPairM[t][1];
  }
  for (int m = 0; m < 32; m++) pos_of_m[m] = mp3g::dct32::kPosOfM[m];
}

#include "../../go-mp3_amd/csrc/dct4_18.h"

// x[n][18] -> X[n][18]: the scalar and the packed DCT-IV-18 of the IMDCT
extern "C" void dct4_18_host(const float* x, float* X, float* Xp, int n) {
  for (int i = 0; i < n; i++) {
    mp3g::dct4::dct4_18(x + 18 * i, X + 18 * i);
    mp3g::pk::f2 P[9];
    mp3g::dct4::dct4_18_pk(x + 18 * i, P);
    for (int k = 0; k < 9; k++) {
      Xp[18 * i + 2 * k] = P[k].x;
      Xp[18 * i + 17 - 2 * k] = P[k].y;
    }
  }
}
