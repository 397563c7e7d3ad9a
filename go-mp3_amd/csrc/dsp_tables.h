// dsp_tables.h -- constant tables of the granule DSP, computed on the host
// exactly as the reference initialises them, then uploaded once per device.
//
// Reference initialisers:
//   synthNWin      internal/frame/frame.go:488-497
//   synthDtbl      internal/frame/frame.go:499-628   (ISO 11172-3 Table B.3)
//   imdctWinData   internal/imdct/imdct.go:21-57
//   cosN12/cosN36  internal/imdct/imdct.go:59-79
//   powtab34       internal/frame/frame.go:31-40
//   isRatios       internal/frame/frame.go:304-306
//   cs/ca          internal/frame/frame.go:422-425
//   SfBandIndices  internal/consts/consts.go:68-97
#pragma once
#include <cstdint>

namespace mp3g {

// Line tables per (lsf, sampling-frequency index) combination: combo = lsf*3 + sfreq.
constexpr int kCombos = 6;

struct DspTables {
  // Requantization: req[r][a] = float32(pow(2, r/4) * powtab34[a]), r = 0..3,
  // a = 0..8206.  float32(pow(2, n/4) * powtab34[a]) == ldexp(req[n&3][a], n>>2)
  // for every n the bitstream can produce (tests/test_tables.py proves it
  // exhaustively against the oracle's direct float64 evaluation).
  float req[4][8207];
  float nwin[64][32];
  float synth_d[512];
  float imdct_win[4][36];
  float cos12[6][12];
  float cos36[18][36];
  float is_ratio[7][2];     // [is_pos][ch]: f32 ratios as stereoProcessIntensity* computes them
  float aa_cs[8], aa_ca[8];
  uint16_t sfb_long[kCombos][23];
  uint16_t sfb_short[kCombos][14];
  uint8_t line_long_sfb[kCombos][576];   // long scale-factor band of line i
  // short-block info of line i in source (window-major) order:
  //   bits 0..3 short sfb, bits 4..5 window, bits 6..15 reordered destination
  uint16_t line_short[kCombos][576];
  // inverse of the reorder permutation, indexed by DESTINATION line d:
  //   bits 0..3 short sfb, bits 4..5 window of the source, bits 6..15 source line
  uint16_t line_short_inv[kCombos][576];
  int8_t pretab[22];
  // distinct rows of synthNWin (rows 0..16 and 32..48); the others follow
  // bit-exactly: row 16+k = -row 16-k, row 48+k = row 48-k (k = 1..15)
  float nwin_distinct[34][32];
  // the 18 distinct columns of cosN36 (p = 0..8 and 18..26):
  // col(17-p) = -col(p), col(53-p) = col(p)
  float cos36_distinct[18][18];  // [m][q'], q' < 9 -> p = q', else p = 18 + (q' - 9)
  // lines no antialias butterfly touches (80 of them), ascending
  uint16_t aa_singles[80];
};

// Fills `t` (deterministic, thread-safe).
void build_tables(DspTables* t);

// Tables of the fast mode (MP3G_MODE_FAST, granule_fast.hip), derived from the
// exact tables above with exact sign/index identities only, so every constant
// is the reference's own float32 value.
//   V = synthNWin * S (64 x 32) is computed from its 32 distinct values
//   X[m] = sum_k cos((2k+1) m pi / 64) s[k], folded even/odd:
//   X[m] = sum_{k<16} dct[m][k] * (m even ? s[k] + s[31-k] : s[k] - s[31-k]),
//   dct[m][k] = nwin[m-16][k] (m >= 16), -nwin[48-m][k] (m < 16).
//   V[i] = X[16+i] (i < 16), 0 (i = 16), -X[48-i] (16 < i < 48), -X[i-48] (i >= 48).
//   The window sum pcm[i] = sum_j D[32j+i] * (j even ? V_j[i] : V_j[32+i])
//   reads X_j[a_i] (j even) and X_j[b_i] (j odd) with the signs folded into
//   dwin[i][j] (a_i = 16+i | 48-i, b_i = 16-i | i-16).
// slots per ring column of the fast kernel (granule_fast.hip kSlots)
constexpr int kFastRingSlots = 34;
// entries of the fast kernel's |x|^(4/3) table (MP3G_FAST_P43_N: 256 = |x| < 128)
#ifndef MP3G_FAST_P43_N
#define MP3G_FAST_P43_N 256
#endif
constexpr int kFastP43 = MP3G_FAST_P43_N;
static_assert(kFastP43 == 256 || kFastP43 == 512, "p43 table size");
struct FastTables {
  float c36[18][18];   // distinct cosN36 columns (= DspTables::cos36_distinct)
  float cos12[6][12];
  float win[4][36];
  float dct[32][16];
  float dwin[32][16];
  // reference-order fallback (hot granules, granule_fast.hip): the full rows
  // of the 32 distinct V values, X[m] = sum_j nrow[m][j] S[j] in the
  // reference's summation order -- nrow[m] = synthNWin[m-16] (m >= 16),
  // -synthNWin[48-m] (m < 16), negated rows giving bit-negated sums
  float nrow[32][32];
  // exact mode (v4, granule_wexact.hip) also carries V[16], the residue of
  // synthNWin's row 16 (~1e-16, not zero: tests/test_tables.py): that row and
  // the synthesis-window taps of output 16 that read it (synthDtbl[32 j + 16],
  // j even)
  float nrow16[32];
  float dwin16[8];
  float aa_cs[8], aa_ca[8];
  float is_ratio[8][2];           // [is_pos][ch] (rows 0..6 used)
  // per (combo, output line L): the line's long band (bits 0..4), short band
  // (5..8), window of the reorder SOURCE line (9..10), the line's own
  // window in window-major order (11..12), reorder source line (13..22)
  uint32_t linfo[kCombos][576];
  // the same for short, non-mixed blocks, pre-resolved for the fast kernel's
  // reorder gather: short band (bits 0..3), 3 band + window of the source line
  // (4..9) and of the line itself (10..15), the source line's int16 index in
  // the staged ring (16..27: 2 kFastRingSlots (src / 18) + src % 18)
  uint32_t sinfo[kCombos][576];
  // per (combo, subband): long band of the subband's first line (bits 0..4)
  // and a mask of the lines j = 1..17 that start a new long band (bits 5+j)
  uint32_t lband[kCombos][32];
  uint16_t sfb_long[kCombos][23];
  uint16_t sfb_short[kCombos][14];
  int8_t pretab[22];
  // the fast kernel's long-block requantize: p43[x + kFastP43 / 2] = sign(x) |x|^(4/3)
  // as float32 (= +-req[0][|x|]) for x = -kFastP43 / 2 .. kFastP43 / 2 - 1
  float p43[kFastP43];
};
void build_fast_tables(const DspTables& t, FastTables* f);

}  // namespace mp3g
