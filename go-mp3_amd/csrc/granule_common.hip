// granule_common.hip -- per-line front-end helpers shared by the v2 (exact)
// and v3 (fast) granule kernels.  Everything here is bit-exact in both modes:
// requantization, reorder, MS/IS stereo are integer/table work plus single
// float32 multiplications, so the fast mode keeps them identical to the
// reference (internal/frame/frame.go:140-420).
// (compiled as part of kernels.hip)
#include "granule_hdr.h"

namespace mp3g {
namespace common {


// int(sum * 32767) clamped to [-32767, 32767] (frame.go:663-669); Go's
// out-of-range float->int conversion yields INT64_MIN -> -32767.
__device__ __forceinline__ int pcm_sample(float sum) {
  const float t = sum * 32767.0f;
  if (!(t == t) || fabsf(t) >= 9.2233720368547758e18f) return -32767;
  return (int)fminf(fmaxf(t, -32767.0f), 32767.0f);
}

// Requantized value of OUTPUT line L (after the short-block reorder) of one
// channel, computed in gather form from the raw Huffman integers `raw`
// (frame.go:140-302).  Mirrors the count1-bounded loops exactly: lines the
// reference does not requantize keep their integer value, lines a short
// block's reorder does not move keep their own window.
__device__ __forceinline__ float requant_line(const int16_t* raw, const mp3g_channel& C, int L,
                                              int combo) {
  const bool shortblk = C.win_switch_flag == 1 && C.block_type == 2;
  const bool mixed = C.mixed_block_flag != 0;
  const int count1 = C.count1;
  int src = L, sfb, win = 0;
  bool process, is_long;
  if (!shortblk) {
    process = L < count1;
    is_long = true;
    sfb = g_tab.line_long_sfb[combo][L];
  } else if (mixed && L < 36) {
    process = true;
    is_long = true;
    sfb = g_tab.line_long_sfb[combo][L];
  } else {
    const int inv = g_tab.line_short_inv[combo][L];
    sfb = inv & 15;
    const int bstart = 3 * (int)g_tab.sfb_short[combo][sfb];
    process = bstart < count1;
    const bool reordered = sfb == (mixed ? 3 : 0) || bstart < count1;
    if (reordered) {
      src = inv >> 6;
      win = (inv >> 4) & 3;
    } else {
      win = (g_tab.line_short[combo][L] >> 4) & 3;  // not moved: window of L itself
    }
    is_long = false;
  }
  const int x = raw[src];
  if (!process) return (float)x;
  const int sfmul = C.scalefac_scale != 0 ? 4 : 2;
  int n4;
  if (is_long)
    n4 = (int)C.global_gain - 210 -
         sfmul * ((int)C.scalefac_l[sfb] + (int)C.preflag * (int)g_tab.pretab[sfb]);
  else
    n4 = (int)C.global_gain - 210 - 8 * (int)C.subblock_gain[win] - sfmul * (int)C.scalefac_s[sfb][win];
  float v = ldexpf(g_tab.req[n4 & 3][min(abs(x), 8206)], n4 >> 2);
  return x < 0 ? -v : v;
}

// MS / intensity stereo of line L (frame.go:304-420), both channels given.
// Reference quirks kept: IS reads channel-0 scale factors and scales each
// channel by its own ratio; MS covers i < max(count1); IS bands start at
// channel 1's count1; LSF uses the MPEG-1 ratio table.
__device__ __forceinline__ void stereo_line(const mp3g_granule& d, uint32_t h, int combo, int L,
                                            float& l, float& r) {
  if (hdr_mode(h) != 1) return;
  const mp3g_channel& C0 = d.ch[0];
  const int c1r = d.ch[1].count1;
  if ((h & 0x20u) && L < max((int)C0.count1, c1r)) {
    const float inv_sqrt2 = 0.70710678118654752440f;
    const float nl = (l + r) * inv_sqrt2;
    const float nr = (l - r) * inv_sqrt2;
    l = nl;
    r = nr;
  }
  if (h & 0x10u) {
    const bool short0 = C0.win_switch_flag == 1 && C0.block_type == 2;
    const bool mixed0 = C0.mixed_block_flag != 0;
    const int sfl = g_tab.line_long_sfb[combo][L];
    const int info = g_tab.line_short[combo][L];
    const int sfs = info & 15, win = (info >> 4) & 3;
    const bool long_pass = !short0 ? (sfl < 21) : (mixed0 && sfl < 8);
    if (long_pass && (int)g_tab.sfb_long[combo][sfl] >= c1r) {
      const int pos = C0.scalefac_l[sfl];
      if (pos < 7) {
        l = l * g_tab.is_ratio[pos][0];
        r = r * g_tab.is_ratio[pos][1];
      }
    }
    const bool short_pass = short0 && sfs < 12 && (!mixed0 || sfs >= 3);
    if (short_pass && 3 * (int)g_tab.sfb_short[combo][sfs] >= c1r) {
      const int pos = C0.scalefac_s[sfs][win];
      if (pos < 7) {
        l = l * g_tab.is_ratio[pos][0];
        r = r * g_tab.is_ratio[pos][1];
      }
    }
  }
}

}  // namespace common
}  // namespace mp3g
