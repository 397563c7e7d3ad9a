// granule_fast.hip -- MP3G_MODE_FAST granule decode, v3 (gfx950).
//
// Same contract, chunk/halo decomposition and front end as the exact kernels
// (reference internal/frame/frame.go:121-688), but the three transforms are
// evaluated in reassociated, FMA-contracted float32, so PCM is within +-1 LSB
// of the reference instead of bit-identical (north star tolerance; measured
// by tests/test_gpu_parity.py::test_fast_mode_*).
//
// Work decomposition: ONE WAVE PER CHUNK, eight independent waves (chunks)
// per 512-thread workgroup sharing the read-only tables, 16 waves per CU
// (<= 128 VGPRs, 9.1 KB of LDS per wave + 4 KB shared).  A wave walks its
// chunk granule by granule with wave-level LDS ordering only:
//   front end   lane = (ch, sb): the 18 lines of its subband from registers
//               (prefetched one granule ahead) -- long blocks requantized as
//               p43[x] * 2^(n4/4) (sign(x)|x|^(4/3) for |x| < 128 from a 1-KB
//               LDS table times the band gain; a lane holding a larger |x|
//               redoes its lines arithmetically), short blocks as
//               x 2^(log2|x|/3 + n4/4) through an LDS gather (the reorder);
//               MS pairs through v_permlane32_swap, intensity stereo per
//               lane; antialias butterflies via DPP wave shifts;
//   IMDCT       lane = (ch, sb): long blocks as a packed DCT-IV-18
//               (dct4_18.h), the overlap `store` in the lane's VGPRs for the
//               whole chunk, frequency inversion folded into window signs;
//   matrixing   V = synthNWin * S has 32 distinct values X: lane = (ch, slot)
//               runs an in-lane fast DCT-II-32 on float pairs (dct32.h) over
//               its column of the X ring, in place;
//   window      lane = (ch, i): 16 taps (V->X signs and x32767 folded in)
//               over operand pairs of the column-major ring, s16 (L, R) pairs
//               through one v_permlane32_swap per slot pair, stored at once.
// Hot granules (hybrid output above the magnitude bound kHotS / kHotL1) are
// not redone here: the wave records their zones (the granules whose PCM
// depends on them) and appends them to the launch's zone list, and a second
// launch -- the exact v4 kernel over the list (kernels_fast.hip launch_fast)
// -- decodes every zone in the reference's operation order from its replay
// start and overwrites its PCM: within +-1 LSB on every valid input.  (The
// in-wave pass with the *_exact functions is compiled into the diagnostic
// kStamp build only.)
// (compiled in its own TU, kernels_fast.hip)
#pragma clang fp contract(fast)
#include <type_traits>

#include "dct32.h"
#include "dct4_18.h"
#include "xlane.h"

// cache policy of the PCM stores (2 = nt: streamed past the caches)
#ifndef MP3G_PCM_STORE_AUX
#define MP3G_PCM_STORE_AUX 2
#endif

namespace mp3g {
namespace v3 {
// Independent chunks (one per wave) per workgroup, sharing the read-only
// tables.  8 waves: 2 workgroups (16 waves) per CU, the shared tables held
// twice per CU instead of four times (2-3 % faster than 4-wave workgroups on
// c2 and c3, tools/gpu_ab.sh; 16 waves measured the same).
#ifndef MP3G_FAST_PRIO
#define MP3G_FAST_PRIO 1  // progress-balanced s_setprio (0: A/B experiments)
#endif
// The granule descriptors one dword per lane in a VGPR (lane i < 40 holds
// dword i of the 160-B mp3g_granule), loaded one granule ahead by a single
// buffer load: the header and channel words come out by v_readlane, the long
// bands' scale factors by ds_bpermute -- no LDS round trip and no LDS copy of
// the next descriptors per granule.  The rare paths that index the scale
// factors per line (short blocks, intensity stereo) first drop the descriptor
// into the wave's LDS slot.  0: the descriptors staged in LDS (round 5).
#ifndef MP3G_FAST_DESC_VGPR
#define MP3G_FAST_DESC_VGPR 1
#endif
#ifndef MP3G_FAST_WG_WAVES
#define MP3G_FAST_WG_WAVES 8
#endif
constexpr int kWaves = MP3G_FAST_WG_WAVES;  // independent chunks (one per wave) per workgroup; they share the tables
namespace {

using common::hdr_combo;
using common::hdr_mode;
using common::hdr_nch;
// int(sum * 32767) clamped to +-32767 (frame.go:663-669).  The exact kernels
// also reproduce Go's result for NaN / |t| >= 2^63; no decodable input gets
// near that (|sum| < 1e12), so the fast path is clamp + truncate.
__device__ __forceinline__ int pcm_sample(float sum) {
  return (int)__builtin_amdgcn_fmed3f(sum * 32767.0f, -32767.0f, 32767.0f);
}

constexpr int kLanes = 64;
// Packed FP32: one v_pk_fma_f32 does two FMAs in the issue slot of one
// v_fma_f32 (measured on MI355X: 122 vs 51-69 TFLOP/s, tools/valu_bench.hip),
// so the IMDCT, matrixing and window sums are written on float pairs.
using pk::f2;
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bcast(float v) { return (f2){v, v}; }
// pretab[22] (frame.go:39) packed 2 bits per band: no per-lane table load
__device__ __forceinline__ int kPretab(int sfb) { return (int)((0x2fe95400000ull >> (2 * sfb)) & 3u); }
// The X ring, column-major: ring[ch][m][u] = X_u[m], the value m (in
// dct32::kPosOfM order) of time slot u.  Slots 1..15 hold the previous
// granule's last 15 slots (slot 0 is unused), 16..33 the current granule; the
// window of slot ss reads slots 16+ss-j, j = 0..15, so 15 history slots
// suffice (the 16th V block of Frame.vVec is never read again).
//  * every operand pair of the window is two consecutive slots of one column:
//    (16+v, 17+v), v even, is one 8-B aligned ds_read_b64, (15+v, 16+v) one
//    ds_read2_b32;
//  * 34 dwords per column (34 = 2 mod 32): the columns the 32 lanes of a
//    channel read start in distinct even banks (conflict-free b64 reads);
//  * the matrixing lane of slot u reads and writes its slot across the 32
//    columns: consecutive lanes hit consecutive dwords;
//  * 2 x 32 x 34 x 4 = 8,704 B per wave, which with the raw coefficients in
//    registers (no LDS copy) brings an 8-wave workgroup to 75 KB: 2
//    workgroups = 16 waves per CU.
constexpr int kHist = 16;
// 16 waves per CU: <= 128 VGPRs (MI355X_MICROARCH.md register
// table) next to the 40.5 KB of LDS per workgroup
#ifndef MP3G_FAST_WAVES_PER_SIMD
#define MP3G_FAST_WAVES_PER_SIMD 4
#endif
constexpr int kSlots = kHist + 18;
static_assert(kSlots == kFastRingSlots, "FastTables::sinfo indexes the staged ring");
#ifndef MP3G_FAST_PCM_D16
#define MP3G_FAST_PCM_D16 0  // (A/B) PCM as per-channel 16-bit stores instead of swap + merge
#endif
#ifndef MP3G_FAST_P43
#define MP3G_FAST_P43 1  // long-block requantize through the p43 LDS table (0: arithmetic, A/B)
#endif
#ifndef MP3G_P43_SCHED
#define MP3G_P43_SCHED 0
#endif
#ifndef MP3G_FAST_DWIN_STRIDE
#define MP3G_FAST_DWIN_STRIDE 20
#endif
constexpr int kDwinStride = MP3G_FAST_DWIN_STRIDE;

// read-only tables, one copy per workgroup
struct __align__(16) SharedSmem {
  // imdctWinData (imdct.go:21-57) per block type and subband parity as
  // (Wp, Wn) pairs per q = 0..8 (see the IMDCT): Wp = (W[q], -W[17-q]),
  // Wn = (-W[18+q], -W[35-q]), each element times the frequency-inversion
  // sign of its line in an odd subband (frame.go:480-486)
  float4 winp[4][2][9];
  float isr[8][2];
  // FastTables::dwin rows, pre-scaled by 32767, padded to 20 floats: the
  // lanes of a ds_read_b128 group (4 x 16) then hit 16 distinct bank quads
  // (16-float rows put every fourth row on one quad: 4-way conflicts)
  float dwin[32][kDwinStride];
  // FastTables::lband: read per lane every granule, so it lives in LDS -- a
  // vector global load there would wait (vmcnt is in order) for the previous
  // granule's PCM stores
  // per subband: .x = lband (first band | bit 5 + j: line j = 1..17 starts a
  // band), .y = the band-start bits of the even lines 2i = 2..16 (only even
  // lines start a band) at bits 4 (i - 1) .. 4 i - 1, four bits each: the
  // popcount of a prefix is then the byte offset of a float32 band gain, so a
  // line pair's gain address is one v_and + one v_bcnt (accumulating the
  // base) instead of a bit-field extract, a popcount and a shift-add; one
  // ds_read_b64 reads both
  uint2 lbd[kCombos][32];
  __device__ uint32_t lband_at(int c, int k) const { return lbd[c][k].x; }
  // FastTables::p43: sign(x) |x|^(4/3) of x = -128..127 at byte offset
  // 4 x + 512 -- the long-block requantize is a table read and one multiply
  float p43[kFastP43];
};
// per-wave working set 9.1 KB.  The workgroup (8 waves + shared tables) must
// stay <= 64 x 1280 B (gfx950 LDS allocation granule) for 2 workgroups
// (16 waves) per CU.
struct __align__(16) WaveSmem {
  // the current granule's slots of a column (16..33) first receive S (the
  // IMDCT output of subband k = column, one value per slot) and the matrixing
  // turns them into X in place; before that they stage the raw coefficients
  // of short-block granules (reorder gather) and the intensity-stereo pass
  float ring[2][32][kSlots];
  mp3g_granule desc;  // 16-B aligned: the channels' first 8 bytes are one 8-B read each
  // the next granule's descriptor, one granule ahead: its count1s bound the
  // next granule's coefficient prefetch (lines at and above count1 are zero by
  // the parse's guarantee, maindata/huffman.go:127-134, so they are neither
  // read here nor written by the main-data kernel, MP3G_HUFF_ROWS_COUNT1;
  // c3 -0.4 % against whole rows, tools/gpu_r03z.sh)
#if !MP3G_FAST_DESC_VGPR
  mp3g_granule descn;
#endif
  // requantization exponents n4 / 4 (float16, exact) of the long bands
  // [ch][sfb] and short bands [ch][sfb][win]; in the fast loop's all-long
  // granules the long bands' gains 2^(n4 / 4) as float32 [ch][sfb] instead
  // (expo_gain(): the first 176 of these 244 bytes)
  _Float16 expo[2 * 22 + 2 * 39];
  __device__ float* expo_gain() { return reinterpret_cast<float*>(expo); }
  __device__ const float* expo_gain() const { return reinterpret_cast<const float*>(expo); }
  // hot-granule zones [start, end) of this chunk, recorded by the fast pass
  // and redone in the reference's order after it (kHotS)
  uint32_t zone[8][2];
};
constexpr uint32_t kZones = 8;
// the plan's zone list holds kZoneListPerChunk zones per chunk (kernels.h): a
// wave records at most kZones, so the list cannot overflow
static_assert(kZones <= kZoneListPerChunk, "zone list smaller than a chunk's zones");

// Raw coefficients of lane (ch, sb) of granule g: its 18 lines, 36 B at
// coef[g][ch][18 sb], as 9 dwords (two int16 each) by three 12-B buffer loads
// through a per-granule resource (SGPR base, 32-bit lane offset).
// (nbytes = 0: a resource without records -- the loads return 0 and touch no memory)
__device__ __forceinline__ void load_lines(const int16_t* coef, uint32_t g, int lane, uint32_t cw[9],
                                           int nbytes = (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t))) {
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int16_t*>(coef + (size_t)g * MP3G_COEF_PER_GRANULE), (short)0, nbytes,
      0x00020000);
  const int off = (lane >> 5) * 1152 + (lane & 31) * 36;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(rc, off + 12 * i, 0, 0);
    cw[3 * i] = v[0];
    cw[3 * i + 1] = v[1];
    cw[3 * i + 2] = v[2];
  }
}

// The same, reading only the lines below `lim` (the lane's channel's count1;
// 0 for a channel the granule does not have): lines >= count1 are zero (the
// bitstream parse's guarantee, maindata/huffman.go:127-134, which mp3g_validate
// checks), so a 6-line piece starting at or above it is not fetched -- its
// offset is pushed past the records and the load returns 0 without touching
// memory.  At 128 kbps about 40 % of the coefficient bytes are skipped.
constexpr int kNoRecord = 0x40000000;
__device__ __forceinline__ void load_lines_lim(const int16_t* coef, uint32_t g, int lane, uint32_t cw[9], int nbytes,
                                               int lim) {
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int16_t*>(coef + (size_t)g * MP3G_COEF_PER_GRANULE), (short)0, nbytes,
      0x00020000);
  const int l0 = 18 * (lane & 31);
  const int off = (lane >> 5) * 1152 + 2 * l0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(rc, l0 + 6 * i < lim ? off + 12 * i : kNoRecord, 0, 0);
    cw[3 * i] = v[0];
    cw[3 * i + 1] = v[1];
    cw[3 * i + 2] = v[2];
  }
}
// Lane i < 40: dword i of granule g's descriptor (0 on the other lanes, and
// everywhere when !valid: a resource without records).
__device__ __forceinline__ uint32_t load_desc_dword(const mp3g_granule* gran, uint32_t g, int lane, bool valid) {
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<mp3g_granule*>(gran + g), (short)0, valid ? (int)sizeof(mp3g_granule) : 0, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b32(rd, 4 * lane, 0, 0);
}
// dword k of a descriptor held one dword per lane (wave-uniform k): an SGPR
__device__ __forceinline__ uint32_t desc_word(uint32_t dv, int k) {
  return (uint32_t)__builtin_amdgcn_readlane((int)dv, k);
}
// byte b of a descriptor held one dword per lane, per lane (b may differ by lane)
__device__ __forceinline__ uint32_t desc_byte(uint32_t dv, int b) {
  return ((uint32_t)__builtin_amdgcn_ds_bpermute((b >> 2) << 2, (int)dv) >> (8 * (b & 3))) & 0xffu;
}
static_assert(sizeof(mp3g_granule) == 160 && offsetof(mp3g_granule, ch) == 8 && sizeof(mp3g_channel) == 72 &&
                  offsetof(mp3g_channel, scalefac_l) == 11,
              "descriptor dword layout");

// the line limit of lane (ch, sb) in granule g (wave-uniform g: scalar loads)
__device__ __forceinline__ int count1_lim(const mp3g_granule* gran, uint32_t g, int lane) {
  const uint32_t h = gran[g].header;
  const int c0 = gran[g].ch[0].count1, c1 = gran[g].ch[1].count1;
  return (lane >> 5) ? (common::hdr_nch(h) == 2 ? c1 : 0) : c0;
}

// Replay start of a chunk (same decision as v2::plan_prologue, with wave
// ballots instead of a workgroup scan).
__device__ void prologue(const ChunkDesc& cd, const mp3g_granule* gran, uint64_t* w_out, int init_in[2],
                         int lane) {
  const uint64_t c0 = cd.out_first, s0 = cd.stream_first;
  const bool have_in = cd.flags & kChunkStateIn;
  if (c0 == s0) {
    *w_out = c0;
    init_in[0] = init_in[1] = have_in;
    return;
  }
  const uint64_t start0 = (c0 >= 2 && c0 - 2 > s0) ? c0 - 2 : s0;
  const bool st1 = hdr_nch(gran[c0 - 1].header) == 2;
  const bool st2 = (c0 >= 2 && c0 - 2 >= s0) ? hdr_nch(gran[c0 - 2].header) == 2 : false;
  if (st1 && st2) {
    *w_out = start0;
    init_in[0] = init_in[1] = (start0 == s0) && have_in;
    return;
  }
  int any = 0;
  for (uint32_t k = lane; k < cd.n_out; k += kLanes) any |= hdr_nch(gran[c0 + k].header) == 2;
  const bool need1 = __ballot(any) != 0 || (cd.flags & kChunkStateOut);
  uint64_t start1 = c0;
  bool ch1_from_in = false;
  if (need1) {
    int found = 0;
    uint64_t p2 = 0;
    for (uint64_t hi = c0; hi > s0 && found < 2;) {
      const uint64_t lo = hi - s0 > kLanes ? hi - kLanes : s0;
      const uint64_t g = hi - 1 - lane;
      const bool stereo = ((uint64_t)lane < hi - lo) && hdr_nch(gran[g].header) == 2;
      uint64_t m = __ballot(stereo);
      while (m && found < 2) {
        const int b = __ffsll((unsigned long long)m) - 1;
        found++;
        if (found == 2) p2 = hi - 1 - b;
        m &= m - 1;
      }
      hi = lo;
    }
    if (found == 2) start1 = p2;
    else if (found == 1) start1 = s0;
    else ch1_from_in = true;
  }
  const uint64_t w = start0 < start1 ? start0 : start1;
  *w_out = w;
  init_in[0] = (w == s0) && have_in;
  init_in[1] = ch1_from_in ? have_in : ((w == s0) && have_in);
}

// LDS ordering inside the single-wave workgroup.  A wave's LDS operations
// complete in issue order, so making one lane's ds_write visible to another
// lane's later ds_read only needs the COMPILER not to reorder them: no
// s_waitcnt on the wave's outstanding global loads (the prefetch) or PCM
// stores, which __syncthreads() would drain every phase.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Branch-free selects (v_bfi_b32 / v_cndmask): keeps the compiler from turning
// a per-lane choice between two cheap values into exec-mask branches.
__device__ __forceinline__ float self(bool c, float a, float b) {
  const int m = -(int)c;
  return __int_as_float((__float_as_int(a) & m) | (__float_as_int(b) & ~m));
}
__device__ __forceinline__ int seli(bool c, int a, int b) {
  const int m = -(int)c;
  return (a & m) | (b & ~m);
}

// sign(x) |x|^(4/3) 2^(n4/4) = x 2^(1/3 log2|x| + n4/4): two transcendental
// VALU ops instead of the float64 table gather of the reference
// (frame.go:148-155); relative error ~1e-6 (x = 0 -> exactly 0).  The factor
// x carries the sign (a v_mul_f32 instead of the v_bfi_b32 of a copysign,
// which issues at the slower VOP3 rate, tools/valu_cost.hip).  The band
// exponent arrives as e = n4 / 4 in float16 (exact: n4 is an integer in
// [-390, 45], so e needs 11 significant bits), and the power goes through one
// exp2.  For the values that reach the PCM (|e| and |t| below ~32) the input
// rounding of t adds <= 2^-19 relative error.
__device__ __forceinline__ float requant_fast(int xi, _Float16 e) {
  const float xf = (float)xi;
  const float t = __builtin_fmaf(__builtin_amdgcn_logf(fabsf(xf)), 1.0f / 3.0f, (float)e);
  return xf * __builtin_amdgcn_exp2f(t);
}

// sign(x) |x|^(4/3) g of the int16 in the low half of xw (the long-block
// requantize's lanes outside the p43 table)
__device__ __forceinline__ float requant_gain(uint32_t xw, float g) {
  const float xf = (float)(int16_t)xw;
  return xf * __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(fabsf(xf)) * (1.0f / 3.0f)) * g;
}

// The lane id, recomputed where it is used (asm volatile: not hoisted out of
// the granule loop).  Values derived from it once and kept for the whole loop
// cost a VGPR each; at the 128-VGPR budget the allocator spilled some to
// scratch, and a reload is a VMEM load whose s_waitcnt also waits for the
// in-flight PCM stores and prefetch.
__device__ __forceinline__ int lane_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// X of a V block: X[m] = V[m-16] (m >= 16), -V[48-m] (m < 16).
__device__ __forceinline__ float x_from_v(const float* v, int m) { return m >= 16 ? v[m - 16] : -v[48 - m]; }
// V of an X vector (inverse identity; V[16] = 0).
// x: one slot of the column-major ring (X[m] at x[kS * kPosOfM[m]], kS the
// ring's column stride).
template <int kS = kSlots>
__device__ __forceinline__ float v_from_x(const float* x, int i) {
  if (i < 16) return x[kS * dct32::kPosOfM[16 + i]];
  if (i == 16) return 0.0f;
  if (i < 48) return -x[kS * dct32::kPosOfM[48 - i]];
  return -x[kS * dct32::kPosOfM[i - 48]];
}

// ---- reference-order fallback for hot granules ------------------------------
// The reassociated transforms err in proportion to the magnitudes they sum,
// while the reference's own float32 rounding is reproduced only by its own
// operation order.  A granule whose hybrid output S (what the matrixing
// reads) exceeds kHotS in any line of either channel is "hot": its PCM and
// that of the next granule (whose window reads its V blocks) are computed in
// the reference's order after the chunk's fast pass (the hot zones), from
// entry state that is itself exact: a zone replays the granules that state
// depends on from its replay start (the chunk-halo rule: S_g needs x_{g-1}'s
// overlap, V_{g-1} needs x_{g-2}'s).
// Below kHotS the fast transforms stay within +-1 LSB: an adversarial search
// that drives every line of a granule to just under the bound (dense random
// signs, rows of synthNWin, alternating subbands, tools/adversarial_tolerance.py)
// found 2 LSB at a bound of 8 (the standalone polyphase kernel) and at most 1
// at 6 and at 4; 4 is kept (DESIGN.md "Fast mode on every valid input").
#ifndef MP3G_HOT_S
#define MP3G_HOT_S 4.0f
#endif
constexpr float kHotS = MP3G_HOT_S;
#ifndef MP3G_HOT_CHECK
#define MP3G_HOT_CHECK 1  // 0: timing experiments only (no hot zones: +-1 LSB not guaranteed)
#endif
// The second, exact test of a granule over kHotS (rare): the largest sum
// over the 32 subbands of |S| in one time slot -- what the matrixing adds up
// and a bound on every |X| the window adds up.  Dense loud granules exceed
// it; a few large lines in quiet surroundings (linbits values: every hot
// granule of the synthetic c3 streams) do not, and the fast transforms are
// measured within +-1 LSB on those up to |S| = 56 (tools/fast_tolerance.py,
// spike patterns).  So a granule is hot when max |S| > kHotS (all lines at
// most 4: per-slot sums <= 128, within +-1 LSB on the adversarial dense
// patterns) AND some slot's sum exceeds kHotL1 (|X| <= 64 otherwise).
#ifndef MP3G_HOT_L1
#define MP3G_HOT_L1 64.0f
#endif
constexpr float kHotL1 = MP3G_HOT_L1;

// one rounding per operation in the order written: these helpers (and the
// *_exact functions) are compiled with contraction off
__device__ __forceinline__ float rmul(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float radd(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float rsub(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

// float32(pow(2, n4 / 4) * powtab34[|x|]) with sign (frame.go:148-155,
// :166-173): the proven table form ldexp(req[n4 & 3][|x|], n4 >> 2)
// (dsp_tables.h, tests/test_tables.py); e = n4 / 4 exactly in float16
__device__ __forceinline__ float requant_exact(int xi, _Float16 e) {
  const int n4 = (int)((float)e * 4.0f);
  const float v = __builtin_ldexpf(g_req[n4 & 3][min(abs(xi), 8206)], n4 >> 2);
  return xi < 0 ? -v : v;
}

// The exact path's tables through a base pointer the compiler cannot prove
// loop-invariant: scalar loads issued where they are used, not hoisted out
// of the zone loop as hundreds of live SGPRs.
__device__ __forceinline__ const float* vtab(const float* p) {
  asm volatile("" : "+s"(p));
  return p;
}
// The same for tables every lane reads at the same index: a constant-address-
// space pointer, so the reads are scalar loads (SGPR operands), not vector
// loads into ~hundreds of VGPRs.
typedef const float __attribute__((address_space(4))) cfloat4;
__device__ __forceinline__ cfloat4* stab(const float* p) {
  cfloat4* q = (cfloat4*)p;
  asm volatile("" : "+s"(q));
  return q;
}

// The per-slot test on S in the ring's current slots (wave-uniform); kS the
// column stride, cur the first current slot.
template <int kS = kSlots>
__device__ __forceinline__ bool slot_sums_hot(const float (&ring)[2][32][kS], int nch, int cur = kHist) {
  const int lane = lane_fresh();
  const int c = lane >> 5, slot = lane & 31;
  float sum = 0.0f;
  if (c < nch && slot < 18) {
#pragma unroll
    for (int sb = 0; sb < 32; sb++) sum += fabsf(ring[c][sb][cur + slot]);
  }
  return __builtin_amdgcn_ballot_w64(sum > kHotL1) != 0;
}

// max |v| over the lane's 18 values (v_max3 with abs modifiers)
__device__ __forceinline__ float max_abs18(const float* v) {
  float m = 0.0f;
#pragma unroll
  for (int j = 0; j < 18; j++) m = fmaxf(m, fabsf(v[j]));
  return m;
}

// imdct.Win + overlap-add + frequency inversion of subband k in the
// reference's order (imdct.go:83-108, frame.go:454-486): every sum from 0.0
// over m ascending, product and sum rounded separately.  stp holds the
// overlap with the frequency-inversion signs folded in (see the kernel);
// negation commutes with rounding, so folding the sign is exact.
__device__ __forceinline__ void imdct_exact(const float x[18], int bt, int k, bool act, f2 stp[9], float o[18]) {
#pragma clang fp contract(off)
  const float sodd = (k & 1) ? -1.0f : 1.0f;
  const float* c12 = vtab(&g_fast.cos12[0][0]);
  const float* c36 = vtab(&g_fast.c36[0][0]);
  const float* win = vtab(&g_fast.win[0][0]) + 36 * bt;
  float st[18];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    st[q] = stp[q].x;
    st[17 - q] = stp[q].y;
  }
  if (bt == 2) {
    // out[6 wi + p + 6] += (sum_m in[wi + 3m] cosN12[m][p]) win[2][p], wi ascending
#pragma unroll
    for (int pos = 0; pos < 36; pos++) {
      float raw = 0.0f;
#pragma unroll
      for (int wi = 0; wi < 3; wi++) {
        const int p = pos - 6 - 6 * wi;
        if (p < 0 || p >= 12) continue;
        float sum = 0.0f;
#pragma unroll
        for (int m = 0; m < 6; m++) sum = sum + x[wi + 3 * m] * c12[12 * m + p];
        raw = raw + sum * win[p];
      }
      const float f = (pos & 1) ? raw * sodd : raw;
      if (pos < 18) o[pos] = f + st[pos];
      else if (act) st[pos - 18] = f;
    }
  } else {
    // the 18 distinct columns of cosN36 (DspTables::cos36_distinct):
    // col(17 - p) = -col(p), col(53 - p) = col(p) bit for bit
    float d[18];
#pragma unroll
    for (int q = 0; q < 18; q++) {
      float s = 0.0f;
#pragma unroll
      for (int m = 0; m < 18; m++) s = s + x[m] * c36[18 * m + q];
      d[q] = s;
    }
#pragma unroll
    for (int pos = 0; pos < 36; pos++) {
      const float v = pos < 9 ? d[pos] : pos < 18 ? -d[17 - pos] : pos < 27 ? d[pos - 9] : d[44 - pos];
      const float raw = v * win[pos];
      const float f = (pos & 1) ? raw * sodd : raw;
      if (pos < 18) o[pos] = f + st[pos];
      else if (act) st[pos - 18] = f;
    }
  }
#pragma unroll
  for (int q = 0; q < 9; q++) stp[q] = (f2){st[q], st[17 - q]};
}

// V = synthNWin * S of one time slot in the reference's order
// (frame.go:642-648), as its 32 distinct values X (in place in the ring
// column slot `colu`: S[j] at colu[kS j], X[m] to colu[kS kPosOfM[m]]).
template <int kS = kSlots>
__device__ __forceinline__ void matrix_exact(float* colu) {
#pragma clang fp contract(off)
  float S[32];
#pragma unroll
  for (int j = 0; j < 32; j++) S[j] = colu[kS * j];
  for (int m = 0; m < 32; m++) {
    const float* row = vtab(&g_fast.nrow[m][0]);
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; j++) s = s + row[j] * S[j];
    colu[kS * dct32::kPosOfM[m]] = s;
  }
}

// The 16-tap window of output i = k for the 18 slots of a granule in the
// reference's order (frame.go:649-669): U *= D rounded, summed j = 0..15
// from 0.0, times 32767 rounded; acc2[p] = slots (2p, 2p + 1) as in the fast
// window (RA / RB: the X columns of V_j[i], j even, and V_j[32 + i], j odd;
// the V -> X signs are folded into FastTables::dwin, exactly).  V[16] (the
// reference's ~1e-16 |S| residue of a zero row) is taken as 0.
// (cur: the first current slot of the column layout, kHist in the fused kernel)
template <int cur = kHist>
__device__ __forceinline__ void window_exact(const float* RA, const float* RB, int k, f2 acc2[9]) {
#pragma clang fp contract(off)
  float dw[16];
#pragma unroll
  for (int j = 0; j < 16; j++) dw[j] = vtab(&g_fast.dwin[0][0])[16 * k + j];
#pragma unroll
  for (int ss = 0; ss < 18; ss++) {
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; j++) sum = sum + ((j & 1) ? RB : RA)[cur + ss - j] * dw[j];
    const float t = sum * 32767.0f;
    if (ss & 1) acc2[ss >> 1].y = t;
    else acc2[ss >> 1].x = t;
  }
}

// ---- per-granule stages shared by the fast loop and the exact zone ----------
__device__ __forceinline__ bool is_short_blk(uint32_t d1) { return (d1 & 0x00ffff00u) == 0x00020100u; }

// The granule's wave-uniform parameters (SGPRs) and this lane's channel's.
struct GranParams {
  uint32_t h;
  int nch, combo;
  // the channels' scalar parameters (one 8-B LDS read each):
  // cp0 = count1 | global_gain << 16 | scalefac_scale << 24,
  // cp1 = preflag | win_switch_flag << 8 | block_type << 16 | mixed_block_flag << 24
  uint32_t cp0[2], cp1[2];
  bool all_long;  // every channel of this granule is a long block (no reorder)
  // this lane's channel (lanes of an absent channel mirror channel 0's block
  // layout: no extra divergence)
  uint32_t d1;
  int count1;
  bool shortblk, mixed;
};

// Reads the descriptor in s.desc and fills the band exponents s.expo (long
// bands only when no channel has short blocks).
template <class WS>
__device__ __forceinline__ GranParams granule_params(WS& s, int ch) {
  GranParams P;
  // wave-uniform (SGPR): the per-combo tables become scalar loads
  P.h = __builtin_amdgcn_readfirstlane(s.desc.header);
  P.nch = hdr_nch(P.h);
  P.combo = hdr_combo(P.h);
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint2 v = *reinterpret_cast<const uint2*>(&s.desc.ch[c]);
    P.cp0[c] = __builtin_amdgcn_readfirstlane(v.x);
    P.cp1[c] = __builtin_amdgcn_readfirstlane(v.y);
  }
  P.all_long = !is_short_blk(P.cp1[0]) && (P.nch == 1 || !is_short_blk(P.cp1[1]));
  const bool act = ch < P.nch;
  const uint32_t d0 = (act && ch) ? P.cp0[1] : P.cp0[0];
  P.d1 = (act && ch) ? P.cp1[1] : P.cp1[0];
  {
    // long bands: lane = (c, sfb), 44 lanes
    const int e = lane_fresh();
    if (e < 44) {
      const int c = e >= 22, sfb = e - 22 * c;
      const uint32_t a0 = c ? P.cp0[1] : P.cp0[0], a1 = c ? P.cp1[1] : P.cp1[0];
      const int v = (int)((a0 >> 16) & 0xffu) - 210 -
                    ((a0 >> 24) ? 4 : 2) * ((int)s.desc.ch[c].scalefac_l[sfb] + (int)(a1 & 0xffu) * kPretab(sfb));
      s.expo[e] = (_Float16)(0.25f * (float)v);
    }
    if (!P.all_long) {
      // short bands: (c, sfb, win), 78 entries
      for (int r0 = e; r0 < 2 * 39; r0 += kLanes) {
        const int c = r0 >= 39, r = r0 - 39 * c, sfb = r / 3, win = r - 3 * sfb;
        const uint32_t a0 = c ? P.cp0[1] : P.cp0[0];
        const mp3g_channel& D = s.desc.ch[c];
        const int v = (int)((a0 >> 16) & 0xffu) - 210 - 8 * (int)D.subblock_gain[win] -
                      ((a0 >> 24) ? 4 : 2) * (int)D.scalefac_s[sfb][win];
        s.expo[44 + r0] = (_Float16)(0.25f * (float)v);
      }
    }
  }
  P.count1 = (int)(d0 & 0xffffu);
  P.shortblk = is_short_blk(P.d1);
  P.mixed = (P.d1 >> 24) != 0;
  wave_sync();
  return P;
}

// Requantization of long-block granules, lane = (ch, sb = k), from the raw
// lines in registers.
template <class WS>
__device__ __forceinline__ void front_long_fast(float x[18], const uint32_t cw[9], const WS& s,
                                                const SharedSmem& sh, const GranParams& P, int ch, int k) {
  int xi[18];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    xi[2 * q] = (int)(int16_t)(cw[q] & 0xffffu);
    xi[2 * q + 1] = (int)(int16_t)(cw[q] >> 16);
  }
  // long band of line j: first band of the subband + band starts among
  // lines 1..j.  Every long band starts at an even line (consts.go:68-97
  // SfBandIndices; dsp_tables.cpp checks it), so lines 2q and 2q + 1
  // share one band: one exponent read per line pair.
  const uint32_t lb = sh.lband_at(P.combo, k);
  _Float16 ex[9];
#pragma unroll
  for (int q = 0; q < 9; q++)
    ex[q] = s.expo[22 * ch + (int)(lb & 31u) + __builtin_popcount((lb >> 5) & ((2u << (2 * q)) - 1u))];
  // Lines >= count1 hold zeros (the bitstream parse's guarantee,
  // maindata/huffman.go:130-134; mp3g_validate checks it), and requantizing
  // 0 gives 0, so long blocks need no per-line count1 test here.
  // (absent-channel lanes compute garbage that nothing reads)
#pragma unroll
  for (int j = 0; j < 18; j++) x[j] = requant_fast(xi[j], ex[j >> 1]);
}

// Requantization in gather form (any block type; the reorder of short
// blocks, frame.go:184-302): the channel's raw lines staged in the current
// slots of the ring, lane (ch, sb) gathering its 18 output lines.
template <bool kExact, class WS>
__device__ __forceinline__ void front_gather(float x[18], const uint32_t cw[9], WS& s, const GranParams& P,
                                             int ch, int k) {
  int nsfs = 0;  // short bands whose first line lies below count1 (frame.go:229-255 loop bound)
#pragma unroll
  for (int b = 0; b < 13; b++) nsfs += 3 * (int)g_fast.sfb_short[P.combo][b] < P.count1;
  {
    uint32_t* col = reinterpret_cast<uint32_t*>(&s.ring[ch][k][kHist]);
#pragma unroll
    for (int q = 0; q < 9; q++) col[q] = cw[q];
  }
  wave_sync();
  const int16_t* rch = reinterpret_cast<const int16_t*>(&s.ring[ch][0][kHist]);
  // line info through a buffer resource (SGPR base, 32-bit lane offset) and
  // the lane's first line recomputed here: nothing of this rare path stays
  // live (in VGPRs) across the granule loop
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(&g_fast.linfo[P.combo][0]), (short)0, 576 * 4, 0x00020000);
  const int L0 = 18 * (lane_fresh() & 31);
#pragma unroll
  for (int j = 0; j < 18; j++) {
    const int L = L0 + j;
    const uint32_t inf = __builtin_amdgcn_raw_buffer_load_b32(rl, 4 * L, 0, 0);
    const int sfl = inf & 31, sfs = (inf >> 5) & 15, wsrc = (inf >> 9) & 3, wown = (inf >> 11) & 3;
    const int srcr = inf >> 13;
    const bool longlike = !P.shortblk || (P.mixed && L < 36);
    const bool started = sfs < nsfs;
    const bool reord = sfs == (P.mixed ? 3 : 0) || started;
    const int src = seli(longlike || !reord, L, srcr);
    const int win = seli(reord, wsrc, wown);
    const int eidx = seli(longlike, 22 * ch + sfl, 44 + 39 * ch + 3 * sfs + win);
    const bool process = longlike ? (P.shortblk || L < P.count1) : started;
    const int sk = (src * 3641) >> 16;  // src / 18 for src < 576
    const int xi = rch[2 * kSlots * sk + (src - 18 * sk)];
    const float v = kExact ? requant_exact(xi, s.expo[eidx]) : requant_fast(xi, s.expo[eidx]);
    x[j] = self(process, v, (float)xi);
  }
  wave_sync();  // staged lines read before the slots are reused
}

// MS / intensity stereo with the partner channel's lane (frame.go:304-420):
// single roundings in the reference's order, exact in both modes.
template <class WS, class SH>
__device__ __forceinline__ void stereo_stage(float x[18], const WS& s, const SH& sh,
                                             const GranParams& P, int ch) {
  if (!(P.nch == 2 && hdr_mode(P.h) == 1 && (P.h & 0x30u))) return;
  const mp3g_channel& C0 = s.desc.ch[0];
  const int c1r = (int)(P.cp0[1] & 0xffffu);
  const int msmax = max((int)(P.cp0[0] & 0xffffu), c1r);
  const bool ms = P.h & 0x20u, is = P.h & 0x10u;
  const bool short0 = is_short_blk(P.cp1[0]);
  const bool mixed0 = (P.cp1[0] >> 24) != 0;
  const float inv_sqrt2 = 0.70710678118654752440f;
  if (ms) {
    // MS: L' = (l + r)c, R' = (l - r)c for lines below max(count1)
    // (frame.go:362-377).  Two lines per step: one swap gives lanes < 32
    // (l, r) of line j and lanes >= 32 those of line j + 1, (l + r)c,
    // (l - r)c in one packed pair, a second swap hands back L' / R' of
    // both lines to their channels' lanes.  Long blocks without intensity
    // stereo transform every line: at or above max(count1) both channels
    // are 0, where (l +- r)c is 0 too.  Otherwise lines >= max(count1) keep
    // their values (the reorder can move values past count1; IS follows).
    auto ms_pair = [&](float& u, float& v) {
      const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(u), __float_as_int(v), false, false);
      const float a = __int_as_float(r[0]), b = __int_as_float(r[1]);
      const f2 pq = (f2){a + b, a - b} * bcast(inv_sqrt2);
      const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_int(pq.x), __float_as_int(pq.y), false, false);
      u = __int_as_float(r2[0]);
      v = __int_as_float(r2[1]);
    };
    if (P.all_long && !is) {  // wave-uniform
#pragma unroll
      for (int j = 0; j < 18; j += 2) ms_pair(x[j], x[j + 1]);
    } else {
      const int left = msmax - 18 * (lane_fresh() & 31);  // lines of this subband below msmax
#pragma unroll
      for (int j = 0; j < 18; j += 2) {
        float n0 = x[j], n1 = x[j + 1];
        ms_pair(n0, n1);
        x[j] = j < left ? n0 : x[j];
        x[j + 1] = j + 1 < left ? n1 : x[j + 1];
      }
    }
  }
  if (is) {
    // Intensity stereo per line of this lane (frame.go:308-359, :379-419):
    // bands at or above channel 1's count1, ratio index from CHANNEL 0's
    // scale factors, each channel scaled by its own ratio (is_pos 7 = no
    // change: isr[7] = (1, 1)).  Long blocks: the line's band from the
    // subband's band-start mask (as in the requantization); short / mixed
    // blocks: the line info table.
    const int k0 = lane_fresh() & 31;
    int nl_is = 0, ns_is = 0;  // first long / short band starting at or above channel 1's count1
#pragma unroll
    for (int b = 0; b < 23; b++) nl_is += (int)g_fast.sfb_long[P.combo][b] < c1r;
#pragma unroll
    for (int b = 0; b < 14; b++) ns_is += 3 * (int)g_fast.sfb_short[P.combo][b] < c1r;
    if (!short0) {
      const uint32_t lb = sh.lband_at(P.combo, k0);
#pragma unroll
      for (int j = 0; j < 18; j++) {
        const int sfl = (int)(lb & 31u) + __builtin_popcount((lb >> 5) & ((2u << j) - 1u));
        const int pos = min((int)C0.scalefac_l[min(sfl, 21)], 7);
        const float rr = sh.isr[pos][ch];
        x[j] = (sfl < 21 && sfl >= nl_is) ? x[j] * rr : x[j];
      }
    } else {
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint32_t*>(&g_fast.linfo[P.combo][0]), (short)0, 576 * 4, 0x00020000);
#pragma unroll
      for (int j = 0; j < 18; j++) {
        const uint32_t info = __builtin_amdgcn_raw_buffer_load_b32(rl, 4 * (18 * k0 + j), 0, 0);
        const int sfl = info & 31, sfs = (info >> 5) & 15, wown = (info >> 11) & 3;
        const bool lp = mixed0 && sfl < 8 && sfl >= nl_is;
        const bool sp = sfs < 12 && (!mixed0 || sfs >= 3) && sfs >= ns_is;
        const int pl = lp ? min((int)C0.scalefac_l[min(sfl, 21)], 7) : 7;
        const int ps = sp ? min((int)C0.scalefac_s[min(sfs, 12)][min(wown, 2)], 7) : 7;
        x[j] = x[j] * sh.isr[pl][ch] * sh.isr[ps][ch];
      }
    }
  }
}

// Antialias butterflies with the neighbouring subbands' lanes (DPP wave
// shifts; frame.go:427-452).  kExact: the reference's two products and one
// sum per output, each rounded.
template <bool kExact>
__device__ __forceinline__ void antialias_stage(float x[18], const GranParams& P, bool act, int k) {
  const bool sw = P.shortblk;
  const bool skip = !act || (sw && !P.mixed);
  const int sblim = (sw && P.mixed) ? 2 : 32;
  const bool lower = !skip && k >= 1 && k < sblim;     // butterfly with subband k-1
  const bool upper = !skip && k < 31 && k + 1 < sblim;  // butterfly with subband k+1
  float up[8], dn[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    up[i] = xl::from_prev(x[17 - i]);  // x_{k-1}[17-i]
    dn[i] = xl::from_next(x[i]);       // x_{k+1}[i]
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const float cs = g_fast.aa_cs[i], ca = g_fast.aa_ca[i];  // (16 SGPRs, as in the fast loop)
    const float ui = x[i], li = x[17 - i];
    if (kExact) {
      x[i] = self(lower, radd(rmul(ui, cs), rmul(up[i], ca)), ui);
      x[17 - i] = self(upper, rsub(rmul(li, cs), rmul(dn[i], ca)), li);
    } else {
      x[i] = self(lower, ui * cs + up[i] * ca, ui);
      x[17 - i] = self(upper, li * cs - dn[i] * ca, li);
    }
  }
}

// Block type of subband k's IMDCT: long windows for subbands 0, 1 whenever
// win_switch && mixed (frame.go:462-466)
__device__ __forceinline__ int imdct_block_type(uint32_t d1, int k) {
  int bt = (int)((d1 >> 16) & 3u);
  if ((d1 & 0xff00ff00u) == 0x01000100u && k < 2) bt = 0;
  return bt;
}

// IMDCT + overlap + frequency inversion in fast order: raw[0..17] + old
// overlap -> o[], raw[18..35] -> new overlap, frequency inversion riding on
// the signs of the windows and of stp.
__device__ __forceinline__ void imdct_fast(const float x[18], int bt, int nch, bool act, float sodd,
                                           const SharedSmem& sh, f2 stp[9], float o[18]) {
  if (bt == 2) {
    float st[18];
#pragma unroll
    for (int q = 0; q < 9; q++) {
      st[q] = stp[q].x;
      st[17 - q] = stp[q].y;
    }
    // raw[pos] = sum over the windows wi with 0 <= pos-6-6wi < 12 of
    // (sum_m x[wi+3m] cosN12[m][p]) * win[2][p], p = pos-6-6wi (imdct.go:88-94)
#pragma unroll
    for (int pos = 0; pos < 36; pos++) {
      float raw = 0.0f;
#pragma unroll
      for (int wi = 0; wi < 3; wi++) {
        const int p = pos - 6 - 6 * wi;
        if (p < 0 || p >= 12) continue;
        float sum = 0.0f;
#pragma unroll
        for (int m = 0; m < 6; m++) sum += x[wi + 3 * m] * dct4::kCos12[p][m];
        raw += sum * dct4::kWin12[p];
      }
      if (pos & 1) raw *= sodd;  // (pos and pos - 18 have the same parity)
      if (pos < 18) o[pos] = raw + st[pos];
      else st[pos - 18] = self(act, raw, st[pos - 18]);
    }
#pragma unroll
    for (int q = 0; q < 9; q++) stp[q] = (f2){st[q], st[17 - q]};
  } else {
    // the 18 distinct sums are a DCT-IV of size 18 (dct4_18.h):
    // sum_m x[m] cosN36[m][q] = X[9+q], sum_m x[m] cosN36[m][18+q] = -X[8-q];
    // packed, pair k = (X[2k], X[17-2k]) holds X[9+q] and X[8-q] of one q
    f2 P[9];
    dct4::dct4_18_pk(x, P);
    const float4* Wq = sh.winp[bt][lane_fresh() & 1];
    // (the overlap of an absent channel stays frozen: frame.go Decode
    // touches ch < nch only; stereo granules need no per-lane select)
    auto overlap = [&](auto frozen) {
#pragma unroll
      for (int kk = 0; kk < 9; kk++) {
        const int q = kk <= 4 ? 8 - 2 * kk : 2 * kk - 9;
        const float za = kk <= 4 ? P[kk].y : P[kk].x;  // X[9+q]
        const float zb = kk <= 4 ? P[kk].x : P[kk].y;  // X[8-q]
        const float4 w = Wq[q];
        // (o[q], o[17-q]) = X[9+q] (W[q], -W[17-q]) + stp[q];
        // new stp[q] = X[8-q] (-W[18+q], -W[35-q])   (signs folded in w)
        const f2 oq = pfma(bcast(za), (f2){w.x, w.y}, stp[q]);
        o[q] = oq.x;
        o[17 - q] = oq.y;
        const f2 ns = bcast(zb) * (f2){w.z, w.w};
        if constexpr (decltype(frozen)::value)
          stp[q] = (f2){self(act, ns.x, stp[q].x), self(act, ns.y, stp[q].y)};
        else
          stp[q] = ns;
      }
    };
    if (nch == 2) overlap(std::false_type{});
    else overlap(std::true_type{});
  }
}

// (L, R) sample pairs without LDS staging: one v_permlane32_swap per slot
// pair hands lane i slot 2p's (L, R) and lane 32 + i slot 2p + 1's, so every
// lane stores one dword per slot pair and the wave 2 x 128 contiguous bytes.
// Mono: the swap hands lane i channel 0's slot 2p and lane 32 + i its slot
// 2p + 1, stored in both halves (frame.go:671-678).  acc2 holds sum * 32767.
__device__ __forceinline__ void pack_pcm(const f2 acc2[9], int nch, uint32_t pk[9]) {
  auto pack = [&](auto mono) {
#pragma unroll
    for (int p = 0; p < 9; p++) {
      // int(sum * 32767) clamped to +-32767 (frame.go:663-669); no decodable
      // input gets near NaN or |t| >= 2^63 (|sum| < 1e12)
      const int a = (int)__builtin_amdgcn_fmed3f(acc2[p].x, -32767.0f, 32767.0f);
      const int b = (int)__builtin_amdgcn_fmed3f(acc2[p].y, -32767.0f, 32767.0f);
      const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
      // low halves of (r[0], r[1]) -> one dword: L | R << 16 (R = L for mono)
      pk[p] = __builtin_amdgcn_perm((uint32_t)(decltype(mono)::value ? r[0] : r[1]), (uint32_t)r[0], 0x05040100u);
    }
  };
  if (nch == 2) pack(std::false_type{});
  else pack(std::true_type{});
}

// PCM of granule g: one dword per lane and slot pair, non-temporal (c2
// -1.9 %, c3 -0.8 %).  Issued for replayed granules too, through a resource
// with no records (straight-line vmcnt accounting).
__device__ __forceinline__ void store_pcm(int16_t* pcm, uint32_t g, bool out, const uint32_t pk[9], int hi, int k) {
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      pcm + (size_t)g * 1152, (short)0, out ? MP3G_PCM_BYTES_PER_GRANULE : 0, 0x00020000);
#pragma unroll
  for (int p = 0; p < 9; p++)
    __builtin_amdgcn_raw_buffer_store_b32(pk[p], rp, 4 * (32 * (2 * p + hi) + k), 0, MP3G_PCM_STORE_AUX);
}

// Entry state of a replay start: overlap store in registers, V history as X
// vectors, from the stream's state_in (init_in) or zero.  stp[q] =
// (store[q], store[17-q]), each element times the frequency-inversion sign of
// its line (odd line of an odd subband: -1), so the overlap-add yields
// frequency-inverted output directly.
__device__ __forceinline__ void init_state(WaveSmem& s, const mp3g_state* sin, const int init_in[2], int lane,
                                           f2 stp[9]) {
  const int ch = lane >> 5, k = lane & 31;
  const float sodd = (k & 1) ? -1.0f : 1.0f;
  // (no dynamic indexing of init_in[]: a private array would be promoted to LDS)
  const bool in0 = init_in[0] && sin, in1 = init_in[1] && sin;
  const bool from_in = ch ? in1 : in0;
#pragma unroll
  for (int q = 0; q < 9; q++) {
    const float a = from_in ? sin->store[ch][k][q] : 0.0f, b = from_in ? sin->store[ch][k][17 - q] : 0.0f;
    stp[q] = (f2){(q & 1) ? a * sodd : a, (q & 1) ? b : b * sodd};
  }
  for (int e = lane; e < 2 * 15 * 32; e += kLanes) {
    const int c = e / (15 * 32), blk = (e >> 5) % 15, m = e & 31;
    const bool in = c ? in1 : in0;
    s.ring[c][dct32::kPosOfM[m]][kHist - 1 - blk] = in ? x_from_v(&sin->vvec[c][64 * blk], m) : 0.0f;
  }
}

// The granule's descriptor into s.desc and its lines into cw (direct loads).
__device__ __forceinline__ void load_granule(const mp3g_granule* gran, const int16_t* coef, uint32_t g, int lane,
                                             WaveSmem& s, uint32_t cw[9]) {
  load_lines_lim(coef, g, lane, cw, (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t)), count1_lim(gran, g, lane));
  if (lane < 10) reinterpret_cast<uint4*>(&s.desc)[lane] = reinterpret_cast<const uint4*>(gran + g)[lane];
}

// Does replayed granule g (< out_from) produce V a later granule reads? Only
// the last replayed one, or one followed by a granule with fewer channels
// (see v2 / DESIGN.md halo).  Both channel counts come from the headers in
// memory: it is called before exact_granule has loaded g's descriptor into
// s.desc, which still holds whatever granule the wave handled last.
__device__ __forceinline__ bool replay_needs_v(const mp3g_granule* gran, uint32_t g, uint32_t out_from) {
  if (g >= out_from || g + 1 >= out_from) return true;
  return hdr_nch(gran[g + 1].header) < hdr_nch(gran[g].header);
}

// One granule in the reference's operation order (the hot-zone fixup):
// descriptor and lines loaded directly, every stage exact, PCM stored when
// `out`.  Returns whether the granule is hot by its exact hybrid output.
__device__ __forceinline__ bool exact_granule(const mp3g_granule* __restrict__ gran, const int16_t* __restrict__ coef,
                                              int16_t* __restrict__ pcm, WaveSmem& s, const SharedSmem& sh,
                                              uint32_t g, bool out, bool need_v, f2 stp[9]) {
  const int lane = lane_fresh();
  const int ch = lane >> 5, k = lane & 31, hi = lane >> 5;
  uint32_t cw[9];
  load_granule(gran, coef, g, lane, s, cw);
  wave_sync();
  const GranParams P = granule_params(s, ch);
  const bool act = ch < P.nch;
  float x[18];
  front_gather<true>(x, cw, s, P, ch, k);
  stereo_stage(x, s, sh, P, ch);
  antialias_stage<true>(x, P, act, k);
  float o[18];
  imdct_exact(x, imdct_block_type(P.d1, k), k, act, stp, o);
  const bool hot1 = __builtin_amdgcn_ballot_w64((act ? max_abs18(o) : 0.0f) > kHotS) != 0;
  if (act) {
#pragma unroll
    for (int j = 0; j < 18; j++) s.ring[ch][k][kHist + j] = o[j];
  }
  wave_sync();
  const bool hot = hot1 && slot_sums_hot(s.ring, P.nch);
  if (need_v && act && (lane & 31) < 18) matrix_exact(&s.ring[ch][0][kHist + (lane & 31)]);
  wave_sync();
  uint32_t pk[9] = {};
  if (out) {
    const int pa = dct32::kPosOfM[k < 16 ? 16 + k : (k == 16 ? 0 : 48 - k)];
    const int pb = dct32::kPosOfM[k < 16 ? 16 - k : k - 16];
    f2 acc2[9];
    window_exact(&s.ring[ch][pa][0], &s.ring[ch][pb][0], k, acc2);
    pack_pcm(acc2, P.nch, pk);
  }
  store_pcm(pcm, g, out, pk, hi, k);
  wave_sync();
  if (ch < P.nch && need_v) {
    f2* col = reinterpret_cast<f2*>(&s.ring[ch][k][0]);
#pragma unroll
    for (int q = 0; q < 8; q++) col[q] = col[9 + q];
  }
  wave_sync();
  return hot;
}

// End (exclusive, clipped to the chunk) of the granules whose PCM reads a
// hot granule g's V blocks.  Channel 0's V of g feeds the windows of g and
// g + 1.  Channel 1's -- g stereo -- feeds g's window and that of the next
// STEREO granule: a mono granule leaves channel 1's FIFO alone (Decode works
// on ch < nch, frame.go:125-133), so across a mono run the zone reaches the
// first stereo granule after it.  (Rare path: scalar header loads.)
__device__ __forceinline__ uint32_t zone_end(const mp3g_granule* __restrict__ gran, uint32_t g, uint32_t end) {
  uint32_t e = g + 2;
  if (hdr_nch(__builtin_amdgcn_readfirstlane(gran[g].header)) == 2) {
    uint32_t n = g + 1;
    while (n < end && hdr_nch(__builtin_amdgcn_readfirstlane(gran[n].header)) == 1) n++;
    if (n + 1 > e) e = n + 1;
  }
  return e < end ? e : end;
}

// Zones recorded by the fast pass (WaveSmem::zone): a hot granule g opens
// (or extends) the zone [max(g, out_first), zone_end(g)) of granules whose
// PCM depends on its hybrid output (a replayed granule g < out_first whose V
// reaches an output only across a mono run included); the in-wave zone pass
// also extends a zone when its exact arithmetic meets a hot granule.  When
// the list is full the last zone runs to the chunk end.
template <class Smem>
__device__ __forceinline__ void record_hot(Smem& s, uint32_t& nz, const mp3g_granule* __restrict__ gran, uint32_t g,
                                           uint32_t out_first, uint32_t end) {
  // (wave-uniform throughout: every lane stores the same values)
  // (zone_end here, not only in the in-wave pass: a zone deferred to the zone
  // list gets no exact re-detection to extend it across a mono run)
  const uint32_t zs = g > out_first ? g : out_first;
  const uint32_t ze = zone_end(gran, g, end);
  if (zs >= ze) return;  // a replayed granule whose V no output reads
  const uint32_t last_end = nz ? __builtin_amdgcn_readfirstlane(s.zone[nz - 1][1]) : 0u;
  if (nz > 0 && zs <= last_end) {
    s.zone[nz - 1][1] = ze > last_end ? ze : last_end;
  } else if (nz < kZones) {
    s.zone[nz][0] = zs;
    s.zone[nz][1] = ze;
    nz = __builtin_amdgcn_readfirstlane(nz + 1);
  } else {
    s.zone[kZones - 1][1] = end;
  }
  wave_sync();
}

}  // namespace

// kStamp: diagnostic build -- per-phase s_memtime cycle sums of every wave go
// to `stamps` (kPhases per workgroup); never used for output.
constexpr int kPhases = 8;
// kHotCount: the build of MP3G_FLAG_HOT_STATS plans -- the hot-zone pass adds
// its work to the counters in aux (kHotCounters); a separate instantiation
// because the counting alone cost the production kernel ~1.5 % (register
// allocation).
template <bool kStamp, bool kHotCount = false>
__global__ void __launch_bounds__(kLanes * kWaves, MP3G_FAST_WAVES_PER_SIMD)
granule_fast_kernel(const ChunkDesc* __restrict__ chunks, uint32_t n_chunks, const mp3g_granule* __restrict__ gran,
                    const int16_t* __restrict__ coef, const mp3g_state* __restrict__ state_in,
                    mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm,
                    void* __restrict__ aux_arg) {
  // one pointer argument for both: kStamp builds' stamp array, the zone
  // scratch otherwise (an argument more cost the granule loop SGPRs)
  unsigned long long* const stamps = kStamp ? static_cast<unsigned long long*>(aux_arg) : nullptr;
  uint32_t* const aux = kStamp ? nullptr : static_cast<uint32_t*>(aux_arg);
  unsigned long long ph[kPhases] = {}, tprev = 0, rt[4] = {};
  if constexpr (kStamp) rt[0] = __builtin_amdgcn_s_memrealtime();
  auto stamp = [&](int p) {
    if constexpr (kStamp) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[p] += t - tprev;
      tprev = t;
    }
  };
  // one block, the shared tables first: the p43 table then sits below 64 KiB
  // (its address is a ds_read's immediate offset) and every offset its
  // discarded reads can form stays inside the workgroup's LDS
  __shared__ struct {
    SharedSmem sh;
    WaveSmem w[kWaves];
  } lds;
  SharedSmem& sh = lds.sh;
  WaveSmem* const wsm = lds.w;
  // the workgroup's tables, filled after each wave has issued its first
  // loads: their latencies overlap
  auto shared_init = [&]() {
    const int t = threadIdx.x;
    for (int e = t; e < 4 * 2 * 9; e += kLanes * kWaves) {
      const int bt = e / 18, par = (e / 9) & 1, q = e % 9;
      const float* W = g_fast.win[bt];
      // frequency inversion: line j of an odd subband is negated when j is odd
      const float sq = par && (q & 1) ? -1.0f : 1.0f, sr = par && !(q & 1) ? -1.0f : 1.0f;  // j = q, 17 - q
      sh.winp[bt][par][q] = make_float4(W[q] * sq, -W[17 - q] * sr, -W[18 + q] * sq, -W[35 - q] * sr);
    }
    // is_pos 0..6 -> isRatios (frame.go:304-306); 7 -> (1, 1): no change
    for (int e = t; e < 16; e += kLanes * kWaves) (&sh.isr[0][0])[e] = e < 14 ? (&g_fast.is_ratio[0][0])[e] : 1.0f;
    for (int e = t; e < 32 * 16; e += kLanes * kWaves) sh.dwin[e >> 4][e & 15] = (&g_fast.dwin[0][0])[e] * 32767.0f;
    for (int e = t; e < kCombos * 32; e += kLanes * kWaves) {
      const uint32_t lb = (&g_fast.lband[0][0])[e];
      uint32_t d = 0;
      // (bit 5 + j of lb: line j = 1..17 starts a band; line 2i = 2..16 into
      // bits 4 (i - 1) .. 4 i - 1 -- odd lines never start one)
      for (int i = 1; i <= 8; i++) d |= ((lb >> (5 + 2 * i)) & 1u) * (15u << (4 * (i - 1)));
      (&sh.lbd[0][0])[e] = make_uint2(lb, d);
    }
    for (int e = t; e < kFastP43; e += kLanes * kWaves) sh.p43[e] = g_fast.p43[e];
  };
  const int lane = threadIdx.x & (kLanes - 1);
  // wave-uniform in an SGPR: the chunk descriptor then comes in by scalar
  // loads and its fields (pointers, counts) stay out of the VGPR budget
  const uint32_t ci = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
  if (ci >= n_chunks) {  // (wave-uniform: one barrier per wave either way)
    shared_init();
    __syncthreads();
    return;
  }
  WaveSmem& s = wsm[threadIdx.x >> 6];
  const ChunkDesc cd = chunks[ci];
  const int ch = lane >> 5, k = lane & 31;
  // ring positions of the two X values the window of output i = k reads
  const int pa = dct32::kPosOfM[k < 16 ? 16 + k : (k == 16 ? 0 : 48 - k)];
  const int pb = dct32::kPosOfM[k < 16 ? 16 - k : k - 16];

  uint64_t w64;
  int init_in[2];
  prologue(cd, gran, &w64, init_in, lane);
  // loop state as wave-uniform 32-bit scalars (plans are limited to < 2^32
  // granules): keeps it in SGPRs, so per-granule header reads are scalar loads
  // (lgkmcnt) that never wait behind the prefetch loads or PCM stores (vmcnt)
  const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)w64);
  const uint32_t out_first = __builtin_amdgcn_readfirstlane((uint32_t)cd.out_first);
  const uint32_t end = __builtin_amdgcn_readfirstlane((uint32_t)(cd.out_first + cd.n_out));
  const mp3g_state* sin = state_in ? state_in + cd.stream : nullptr;


  // entry state: overlap store in registers, V history as X vectors
  // IMDCT overlap `store` (frame.go:473-476) in registers as pairs
  // stp[q] = (store[q], store[17-q]), each element times the frequency-inversion
  // sign of its line (odd line of an odd subband: -1), so the overlap-add
  // yields frequency-inverted output directly
  const float sodd = (k & 1) ? -1.0f : 1.0f;  // sign of the odd lines of this subband
  f2 stp[9];
  {
    // (no dynamic indexing of init_in[]: a private array would be promoted to LDS)
    const bool in0 = init_in[0] && sin, in1 = init_in[1] && sin;
    const bool from_in = ch ? in1 : in0;
#pragma unroll
    for (int q = 0; q < 9; q++) {
      const float a = from_in ? sin->store[ch][k][q] : 0.0f, b = from_in ? sin->store[ch][k][17 - q] : 0.0f;
      stp[q] = (f2){(q & 1) ? a * sodd : a, (q & 1) ? b : b * sodd};
    }
    for (int e = lane; e < 2 * 15 * 32; e += kLanes) {
      const int c = e / (15 * 32), blk = (e >> 5) % 15, m = e & 31;
      const bool in = c ? in1 : in0;
      s.ring[c][dct32::kPosOfM[m]][kHist - 1 - blk] = in ? x_from_v(&sin->vvec[c][64 * blk], m) : 0.0f;
    }
  }

  uint32_t cw[9] = {};  // the current granule's raw coefficients (lane's 18 lines)
#if MP3G_FAST_DESC_VGPR
  // the descriptors of the current and the next granule, one dword per lane
  uint32_t dv = 0, dvn = 0;
  if (w < end) {
    load_lines_lim(coef, w, lane, cw, (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t)), count1_lim(gran, w, lane));
    dv = load_desc_dword(gran, w, lane, true);
    dvn = load_desc_dword(gran, w + 1, lane, w + 1 < end);
  }
#else
  if (w < end) {
    load_lines_lim(coef, w, lane, cw, (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t)), count1_lim(gran, w, lane));
    if (lane < 10) reinterpret_cast<uint4*>(&s.desc)[lane] = reinterpret_cast<const uint4*>(gran + w)[lane];
    if (lane < 10 && w + 1 < end)
      reinterpret_cast<uint4*>(&s.descn)[lane] = reinterpret_cast<const uint4*>(gran + w + 1)[lane];
  }
#endif
  shared_init();
  __syncthreads();  // the only workgroup barrier: the waves are independent from here on

  // PCM of a granule: one dword (L, R) per lane and slot pair
  uint32_t pk[9] = {};
  const int hi = lane >> 5;

  // ---- 16-tap window over the X ring -> s16 PCM, stored straight to HBM ----
  // (lanes of an absent channel compute values that are never stored; the
  // PCM stores are issued for replayed granules too, through a resource with
  // no records)
  auto window_store = [&](uint32_t g, bool out, int nch) {
    if (out) {
      float dw[16];
      {
        const float4* d4 = reinterpret_cast<const float4*>(&sh.dwin[k][0]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const float4 v = d4[q];
          dw[4 * q] = v.x;
          dw[4 * q + 1] = v.y;
          dw[4 * q + 2] = v.z;
          dw[4 * q + 3] = v.w;
        }
      }
      // accumulator pair p = output slots (2p, 2p+1).  Tap 2t of the pair reads
      // column a of rows (v, v+1) and tap 2t+1 column b of rows (v-1, v),
      // v = 2p - 2t: every operand pair is two rows of one column, i.e. one
      // ds_read2_b32 that lands as the packed operand, and each feeds up to 8
      // accumulator pairs.
      const f2* RA = reinterpret_cast<const f2*>(&s.ring[ch][pa][0]);
      const float* RB = &s.ring[ch][pb][0];
      f2 acc2[9];
#pragma unroll
      for (int p = 0; p < 9; p++) acc2[p] = bcast(0.0f);
#pragma unroll
      for (int v = -14; v <= 16; v += 2) {
        const f2 A = RA[(kHist + v) / 2];  // slots (16+v, 17+v): 8-B aligned
        const f2 B = {RB[kHist + v - 1], RB[kHist + v]};
#pragma unroll
        for (int t = 0; t < 8; t++) {
          const int p = v / 2 + t;
          if (p >= 0 && p < 9) {
            acc2[p] = pfma(bcast(dw[2 * t]), A, acc2[p]);
            acc2[p] = pfma(bcast(dw[2 * t + 1]), B, acc2[p]);
          }
        }
      }
      // (L, R) sample pairs without LDS staging: one v_permlane32_swap per slot
      // pair hands lane i slot 2p's (L, R) and lane 32 + i slot 2p + 1's, so
      // every lane stores one dword per slot pair and the wave 2 x 128
      // contiguous bytes.  Mono: the swap hands lane i channel 0's slot 2p and
      // lane 32 + i its slot 2p + 1, stored in both halves (frame.go:671-678).
      auto pack = [&](auto mono) {
#pragma unroll
        for (int p = 0; p < 9; p++) {
          const int a = (int)__builtin_amdgcn_fmed3f(acc2[p].x, -32767.0f, 32767.0f);
          const int b = (int)__builtin_amdgcn_fmed3f(acc2[p].y, -32767.0f, 32767.0f);
          const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
          // low halves of (r[0], r[1]) -> one dword: L | R << 16 (R = L for mono)
          pk[p] = __builtin_amdgcn_perm((uint32_t)(decltype(mono)::value ? r[0] : r[1]), (uint32_t)r[0], 0x05040100u);
        }
      };
#if MP3G_FAST_PCM_D16
      // (A/B) each lane stores its own channel's samples as 16-bit stores, no
      // swap and no merge: per slot the wave writes 128 contiguous bytes; mono:
      // the channel-0 lanes store (s, s) dwords, the others nothing
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          pcm + (size_t)g * 1152, (short)0, MP3G_PCM_BYTES_PER_GRANULE, 0x00020000);
      if (nch == 2) {
#pragma unroll
        for (int p = 0; p < 9; p++) {
          const int a = (int)__builtin_amdgcn_fmed3f(acc2[p].x, -32767.0f, 32767.0f);
          const int b = (int)__builtin_amdgcn_fmed3f(acc2[p].y, -32767.0f, 32767.0f);
          __builtin_amdgcn_raw_buffer_store_b16((unsigned short)a, rp, 4 * (32 * (2 * p) + k) + 2 * ch, 0, 2);
          __builtin_amdgcn_raw_buffer_store_b16((unsigned short)b, rp, 4 * (32 * (2 * p + 1) + k) + 2 * ch, 0, 2);
        }
      } else {
        const int off = ch ? kNoRecord : 0;
#pragma unroll
        for (int p = 0; p < 9; p++) {
          const int a = (int)__builtin_amdgcn_fmed3f(acc2[p].x, -32767.0f, 32767.0f);
          const int b = (int)__builtin_amdgcn_fmed3f(acc2[p].y, -32767.0f, 32767.0f);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm((uint32_t)a, (uint32_t)a, 0x05040100u), rp,
                                                off + 4 * (32 * (2 * p) + k), 0, 2);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm((uint32_t)b, (uint32_t)b, 0x05040100u), rp,
                                                off + 4 * (32 * (2 * p + 1) + k), 0, 2);
        }
      }
    } else {
      // as many stores as the output path, through a resource with no
      // records: straight-line vmcnt accounting at the join
      const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(pcm, (short)0, 0, 0x00020000);
#pragma unroll
      for (int p = 0; p < 18; p++) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)0, r0, 4 * p, 0, 2);
    }
#else
      if (nch == 2) pack(std::false_type{});
      else pack(std::true_type{});
      // stored right away: a store's data registers are free again once it
      // has issued (no s_waitcnt before their reuse on gfx950), and the loads
      // this wave waits for next were issued before these stores
    }
    {
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          pcm + (size_t)g * 1152, (short)0, out ? MP3G_PCM_BYTES_PER_GRANULE : 0, 0x00020000);
#pragma unroll
      for (int p = 0; p < 9; p++)
        __builtin_amdgcn_raw_buffer_store_b32(pk[p], rp, 4 * (32 * (2 * p + hi) + k), 0, 2);  // non-temporal: c2 -1.9 %, c3 -0.8 %
    }
#endif
  };

  if constexpr (kStamp) {
    tprev = __builtin_amdgcn_s_memtime();
    rt[1] = __builtin_amdgcn_s_memrealtime();
  }
  // Progress-balanced issue priority.  The SIMD arbitrates VALU issue by
  // priority, then age (MI355X_MICROARCH.md, two waves per SIMD), so at equal
  // priority the oldest of the ~3 waves sharing a SIMD runs ahead and the
  // youngest finishes last, alone and latency-bound (c2 timeline: loop spans
  // 34 .. 101 us for identical chunks).  A wave with more of its chunk left
  // takes a higher priority, which keeps the co-resident waves abreast.
  const uint32_t span = end - w, span2 = 2 * span, span3 = 3 * span;
  uint32_t nz = 0;  // hot zones recorded (s.zone)
  uint32_t n_flagged = 0;  // hot granules the pass flagged (kHotCount builds)
  // priority = #{L in 1..3 : 4 (end - g) > L span}: 3 from the start, one
  // less from granule tL = end - floor(L span / 4) on (three compares per
  // granule instead of recomputing the level)
  const uint32_t t3 = end - (span3 >> 2), t2 = end - (span2 >> 2), t1 = end - (span >> 2);
  if (MP3G_FAST_PRIO) __builtin_amdgcn_s_setprio(3);
  for (uint32_t g = w; g < end; g++) {
    if (MP3G_FAST_PRIO) {
      if (g == t1) __builtin_amdgcn_s_setprio(0);
      else if (g == t2) __builtin_amdgcn_s_setprio(1);
      else if (g == t3) __builtin_amdgcn_s_setprio(2);
    }
    const bool out = g >= out_first;
    // the header and both channels' parameters in one LDS round trip, before
    // anything branches on them (read under the halo test first, the header
    // took a round trip of its own: c3 +0.7 %)
#if MP3G_FAST_DESC_VGPR
    // header (dword 0) and the channels' first two dwords (2, 3 and 20, 21)
    // straight from the lanes that hold them
    const uint32_t h = desc_word(dv, 0);
#else
    const uint32_t hv = s.desc.header;
    const uint2 cv0 = *reinterpret_cast<const uint2*>(&s.desc.ch[0]);
    const uint2 cv1 = *reinterpret_cast<const uint2*>(&s.desc.ch[1]);
    const uint32_t h = __builtin_amdgcn_readfirstlane(hv);
#endif
    // does a replayed granule's V feed anything? (see v2 / DESIGN.md halo)
    bool need_v = true;
    if (!out && g + 1 < out_first) need_v = hdr_nch(gran[g + 1].header) < hdr_nch(h);
    const int nch = hdr_nch(h), combo = hdr_combo(h);
    const bool act = ch < nch;
    // the channels' scalar parameters in SGPRs:
    // dword 0 = count1 | global_gain << 16 | scalefac_scale << 24,
    // dword 1 = preflag | win_switch_flag << 8 | block_type << 16 | mixed_block_flag << 24
#if MP3G_FAST_DESC_VGPR
    const uint32_t cp0[2] = {desc_word(dv, 2), desc_word(dv, 20)};
    const uint32_t cp1[2] = {desc_word(dv, 3), desc_word(dv, 21)};
#else
    const uint32_t cp0[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(cv0.x), (uint32_t)__builtin_amdgcn_readfirstlane(cv1.x)};
    const uint32_t cp1[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(cv0.y), (uint32_t)__builtin_amdgcn_readfirstlane(cv1.y)};
#endif
    auto is_short = [](uint32_t d1) { return (d1 & 0x00ffff00u) == 0x00020100u; };  // win_switch 1, block_type 2
    // wave-uniform: every channel of this granule is a long block (no reorder)
    const bool all_long = !is_short(cp1[0]) && (nch == 1 || !is_short(cp1[1]));
#if MP3G_FAST_DESC_VGPR
    // the rare paths that index scale factors per line read the descriptor
    // from the wave's LDS slot: short blocks and intensity stereo
    if (!all_long || (nch == 2 && hdr_mode(h) == 1 && (h & 0x10u))) {
      const int l = lane_fresh();
      if (l < 40) reinterpret_cast<uint32_t*>(&s.desc)[l] = dv;
      wave_sync();
    }
#endif
    // this lane's channel (lanes of an absent channel mirror channel 0's block
    // layout: no extra divergence)
    const uint32_t d0 = (act && ch) ? cp0[1] : cp0[0], d1 = (act && ch) ? cp1[1] : cp1[0];

    // ---- per-granule front-end parameters: band exponents (long bands only
    //      when no channel has short blocks) ----
    {
      // long bands: lane = (ch, sfb = k), k < 22 -- the lane's own channel
      // parameters d0 / d1 (an absent channel's lanes write values nothing reads)
      const int e = lane_fresh();
#if MP3G_FAST_DESC_VGPR
      // scalefac_l[sfb] of channel ch: descriptor byte 19 + 72 ch + sfb
      // (every lane takes part in the permute: lanes >= 22 read bytes they drop)
      const int sfl_byte = (int)desc_byte(dv, 19 + 72 * ch + (e & 31));
#else
      const int sfl_byte = (int)s.desc.ch[ch].scalefac_l[e & 31];
#endif
      if ((e & 31) < 22) {
        const int sfb = e & 31;
        const int v = (int)((d0 >> 16) & 0xffu) - 210 -
                      ((d0 >> 24) ? 4 : 2) * (sfl_byte + (int)(d1 & 0xffu) * kPretab(sfb));
        if (all_long) s.expo_gain()[22 * ch + sfb] = __builtin_amdgcn_exp2f(0.25f * (float)v);
        else s.expo[22 * ch + sfb] = (_Float16)(0.25f * (float)v);
      }
      if (!all_long) {
        // short bands: (c, sfb, win), 78 entries
        for (int r0 = e; r0 < 2 * 39; r0 += kLanes) {
          const int c = r0 >= 39, r = r0 - 39 * c, sfb = r / 3, win = r - 3 * sfb;
          const uint32_t a0 = c ? cp0[1] : cp0[0];
          const mp3g_channel& D = s.desc.ch[c];
          const int v = (int)((a0 >> 16) & 0xffu) - 210 - 8 * (int)D.subblock_gain[win] -
                        ((a0 >> 24) ? 4 : 2) * (int)D.scalefac_s[sfb][win];
          s.expo[44 + r0] = (_Float16)(0.25f * (float)v);
        }
      }
    }
    const int count1 = (int)(d0 & 0xffffu);
    const bool shortblk = is_short(d1);
    const bool mixed = (d1 >> 24) != 0;
    wave_sync();
    stamp(0);

    // ---- front end: requantize (gather through the reorder), lane = (ch, sb = k) ----
    // the lane's 18 line-info words and raw integers are loaded in bulk first
    float x[18];
    if (all_long) {
      // long band of line j: first band of the subband + band starts among
      // lines 1..j.  Every long band starts at an even line (consts.go:68-97
      // SfBandIndices; dsp_tables.cpp checks it), so lines 2q and 2q + 1
      // share one band: one gain read per line pair.
      const int kl = lane_fresh() & 31;  // (lane recomputed: no spilled address)
      const uint2 lbd = sh.lbd[combo][kl];
      const uint32_t lb = lbd.x, d4 = lbd.y;
      const char* eb = reinterpret_cast<const char*>(&s.expo_gain()[22 * ch + (int)(lb & 31u)]);
      float gq[9];
#pragma unroll
      for (int q = 0; q < 9; q++)  // band starts among lines 2..2q (bits 0..4q-1 of d4)
        gq[q] = *reinterpret_cast<const float*>(eb + __builtin_popcount(d4 & (q == 8 ? ~0u : (1u << (4 * q)) - 1u)));
      // x^(4/3) 2^(n4/4) (frame.go:187-200) as p43[x] times the band gain.
      // Both lines of a dword at once: 4 x + 512 per 16-bit half (one
      // v_pk_mad_u16) is the table's byte offset for x = -128..127 and >= 1024
      // for every other |x| <= 8206 (mp3g_validate's bound); lanes holding such
      // a line (c3: ~0.2 % of lanes, 12 % of granules have one) redo their 18
      // lines arithmetically below, and their table reads stay inside the
      // workgroup's LDS (offsets < 64 KiB) and are discarded.
      // Lines >= count1 hold zeros (the bitstream parse's guarantee,
      // maindata/huffman.go:130-134; mp3g_validate checks it), and requantizing
      // 0 gives 0, so long blocks need no per-line count1 test here.
      // (absent-channel lanes compute garbage that nothing reads)
#if MP3G_FAST_P43
      const char* tb = reinterpret_cast<const char*>(&sh.p43[0]);
      uint32_t big = 0;
#pragma unroll
      for (int q = 0; q < 9; q++) {
        // (v_pk_mad_u16 by hand: the compiler splits it into a shift and an
        // add; op_sel_hi 0 on the inline constant: its high half would be 0)
        uint32_t t;
        asm("v_pk_mad_u16 %0, %1, 4, %2 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(cw[q]), "s"(0x00010001u * 2u * kFastP43));
        big |= t;
        x[2 * q] = *reinterpret_cast<const float*>(tb + (t & 0xffffu));
        x[2 * q + 1] = *reinterpret_cast<const float*>(tb + (t >> 16));
      }
#if MP3G_P43_SCHED
      __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
      for (int j = 0; j < 18; j++) x[j] *= gq[j >> 1];
      // (an offset at or past the table's 4 kFastP43 bytes: some |x| >= kFastP43 / 2)
      if (big & (0x00010001u * (0x10000u - 4u * kFastP43))) {
#pragma unroll
        for (int q = 0; q < 9; q++) {
          x[2 * q] = requant_gain(cw[q] & 0xffffu, gq[q]);
          x[2 * q + 1] = requant_gain(cw[q] >> 16, gq[q]);
        }
      }
#else  // (A/B: every long-block line arithmetically, the round-5 path before the table)
#pragma unroll
      for (int q = 0; q < 9; q++) {
        x[2 * q] = requant_gain(cw[q] & 0xffffu, gq[q]);
        x[2 * q + 1] = requant_gain(cw[q] >> 16, gq[q]);
      }
#endif
    } else {
      int nsfs = 0;  // short bands whose first line lies below count1 (frame.go:229-255 loop bound)
#pragma unroll
      for (int b = 0; b < 13; b++) nsfs += 3 * (int)g_fast.sfb_short[combo][b] < count1;
      // reorder gather: the channel's raw lines staged in the current slots of
      // the ring, lane (ch, sb) writing its 9 dwords to column sb
      {
        uint32_t* col = reinterpret_cast<uint32_t*>(&s.ring[ch][k][kHist]);
#pragma unroll
        for (int q = 0; q < 9; q++) col[q] = cw[q];
      }
      wave_sync();
      const int16_t* rch = reinterpret_cast<const int16_t*>(&s.ring[ch][0][kHist]);
      // line info through a buffer resource (SGPR base, 32-bit lane offset) and
      // the lane's first line recomputed here: nothing of this rare path stays
      // live (in VGPRs) across the granule loop.  Short, non-mixed blocks in
      // every channel (wave-uniform) take the pre-resolved table sinfo.
      auto plain = [&](uint32_t d) { return is_short(d) && !(d >> 24); };
      const bool plain_short = plain(cp1[0]) && (nch == 1 || plain(cp1[1]));
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint32_t*>(plain_short ? &g_fast.sinfo[combo][0] : &g_fast.linfo[combo][0]), (short)0,
          576 * 4, 0x00020000);
      const int L0 = 18 * (lane_fresh() & 31);
      // all 18 words first, as 9 8-B loads: one wait, not one per line
      uint32_t infw[18];
#pragma unroll
      for (int q = 0; q < 9; q++) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rl, 4 * L0 + 8 * q, 0, 0);
        infw[2 * q] = v[0];
        infw[2 * q + 1] = v[1];
      }
      if (plain_short) {
        // (the general loop of the else branch with longlike = false, mixed = false)
        const int ebase = 44 + 39 * ch;
#pragma unroll
        for (int j = 0; j < 18; j++) {
          const uint32_t inf = infw[j];
          const int sfs = inf & 15u;
          const bool started = sfs < nsfs;
          const bool reord = sfs == 0 || started;
          const int xi = rch[seli(reord, (int)(inf >> 16), 2 * kSlots * (lane_fresh() & 31) + j)];
          const int e = seli(reord, (int)((inf >> 4) & 63u), (int)((inf >> 10) & 63u));
          x[j] = self(started, requant_fast(xi, s.expo[ebase + e]), (float)xi);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 18; j++) {
          const int L = L0 + j;
          const uint32_t inf = infw[j];
          const int sfl = inf & 31, sfs = (inf >> 5) & 15, wsrc = (inf >> 9) & 3, wown = (inf >> 11) & 3;
          const int srcr = inf >> 13;
          const bool longlike = !shortblk || (mixed && L < 36);
          const bool started = sfs < nsfs;
          const bool reord = sfs == (mixed ? 3 : 0) || started;
          const int src = seli(longlike || !reord, L, srcr);
          const int win = seli(reord, wsrc, wown);
          const int eidx = seli(longlike, 22 * ch + sfl, 44 + 39 * ch + 3 * sfs + win);
          const bool process = longlike ? (shortblk || L < count1) : started;
          const int sk = (src * 3641) >> 16;  // src / 18 for src < 576
          const int xi = rch[2 * kSlots * sk + (src - 18 * sk)];
          x[j] = self(process, requant_fast(xi, s.expo[eidx]), (float)xi);
        }
      }
      wave_sync();  // staged lines read before the slots are reused
    }
    stamp(1);
    // ---- MS / intensity stereo with the partner channel's lane (frame.go:304-420) ----
    if (nch == 2 && hdr_mode(h) == 1 && (h & 0x30u)) {
      const mp3g_channel& C0 = s.desc.ch[0];
      const int c1r = (int)(cp0[1] & 0xffffu);
      const int msmax = max((int)(cp0[0] & 0xffffu), c1r);
      const bool ms = h & 0x20u, is = h & 0x10u;
      const bool short0 = is_short(cp1[0]);
      const bool mixed0 = (cp1[0] >> 24) != 0;
      const float inv_sqrt2 = 0.70710678118654752440f;
      if (ms) {
        // MS: L' = (l + r)c, R' = (l - r)c for lines below max(count1)
        // (frame.go:362-377).  Two lines per step: one swap gives lanes < 32
        // (l, r) of line j and lanes >= 32 those of line j + 1, (l + r)c,
        // (l - r)c in one packed pair, a second swap hands back L' / R' of
        // both lines to their channels' lanes.  Long blocks without intensity
        // stereo transform every line: at or above max(count1) both channels
        // are 0, where (l +- r)c is 0 too.  Otherwise lines >= max(count1) keep
        // their values (the reorder can move values past count1; IS follows).
        auto ms_pair = [&](float& u, float& v) {
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(u), __float_as_int(v), false, false);
          const float a = __int_as_float(r[0]), b = __int_as_float(r[1]);
          const f2 pq = (f2){a + b, a - b} * bcast(inv_sqrt2);
          const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_int(pq.x), __float_as_int(pq.y), false, false);
          u = __int_as_float(r2[0]);
          v = __int_as_float(r2[1]);
        };
        if (all_long && !is) {  // wave-uniform
#pragma unroll
          for (int j = 0; j < 18; j += 2) ms_pair(x[j], x[j + 1]);
        } else {
          const int left = msmax - 18 * (lane_fresh() & 31);  // lines of this subband below msmax
#pragma unroll
          for (int j = 0; j < 18; j += 2) {
            float n0 = x[j], n1 = x[j + 1];
            ms_pair(n0, n1);
            x[j] = j < left ? n0 : x[j];
            x[j + 1] = j + 1 < left ? n1 : x[j + 1];
          }
        }
      }
      if (is) {
        // Intensity stereo per line of this lane (frame.go:308-359, :379-419):
        // bands at or above channel 1's count1, ratio index from CHANNEL 0's
        // scale factors, each channel scaled by its own ratio (is_pos 7 = no
        // change: isr[7] = (1, 1)).  Long blocks: the line's band from the
        // subband's band-start mask (as in the requantization); short / mixed
        // blocks: the line info table.
        const int k0 = lane_fresh() & 31;
        int nl_is = 0, ns_is = 0;  // first long / short band starting at or above channel 1's count1
#pragma unroll
        for (int b = 0; b < 23; b++) nl_is += (int)g_fast.sfb_long[combo][b] < c1r;
#pragma unroll
        for (int b = 0; b < 14; b++) ns_is += 3 * (int)g_fast.sfb_short[combo][b] < c1r;
        if (!short0) {
          const uint32_t lb = sh.lbd[combo][k0].x;
#pragma unroll
          for (int j = 0; j < 18; j++) {
            const int sfl = (int)(lb & 31u) + __builtin_popcount((lb >> 5) & ((2u << j) - 1u));
            const int pos = min((int)C0.scalefac_l[min(sfl, 21)], 7);
            const float rr = sh.isr[pos][ch];
            x[j] = (sfl < 21 && sfl >= nl_is) ? x[j] * rr : x[j];
          }
        } else {
          const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<uint32_t*>(&g_fast.linfo[combo][0]), (short)0, 576 * 4, 0x00020000);
          uint32_t infw[18];  // (9 8-B loads, one wait)
#pragma unroll
          for (int q = 0; q < 9; q++) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rl, 4 * 18 * k0 + 8 * q, 0, 0);
            infw[2 * q] = v[0];
            infw[2 * q + 1] = v[1];
          }
#pragma unroll
          for (int j = 0; j < 18; j++) {
            const uint32_t info = infw[j];
            const int sfl = info & 31, sfs = (info >> 5) & 15, wown = (info >> 11) & 3;
            const bool lp = mixed0 && sfl < 8 && sfl >= nl_is;
            const bool sp = sfs < 12 && (!mixed0 || sfs >= 3) && sfs >= ns_is;
            const int pl = lp ? min((int)C0.scalefac_l[min(sfl, 21)], 7) : 7;
            const int ps = sp ? min((int)C0.scalefac_s[min(sfs, 12)][min(wown, 2)], 7) : 7;
            x[j] = x[j] * sh.isr[pl][ch] * sh.isr[ps][ch];
          }
        }
      }
    }
    {
      const bool sw = shortblk;
      const bool skip = !act || (sw && !mixed);
      const int sblim = (sw && mixed) ? 2 : 32;
      const bool lower = !skip && k >= 1 && k < sblim;     // butterfly with subband k-1
      const bool upper = !skip && k < 31 && k + 1 < sblim;  // butterfly with subband k+1
      float up[8], dn[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        up[i] = xl::from_prev(x[17 - i]);  // x_{k-1}[17-i]
        dn[i] = xl::from_next(x[i]);       // x_{k+1}[i]
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const float cs = g_fast.aa_cs[i], ca = g_fast.aa_ca[i];
        const float ui = x[i], li = x[17 - i];
        x[i] = self(lower, ui * cs + up[i] * ca, ui);
        x[17 - i] = self(upper, li * cs - dn[i] * ca, li);
      }
    }

    stamp(2);
    // ---- IMDCT + overlap + frequency inversion ----
    float o[18];
    {
      // mixed blocks: long windows for subbands 0, 1 whenever win_switch && mixed (frame.go:462-466)
      int bt = (int)((d1 >> 16) & 3u);
      if ((d1 & 0xff00ff00u) == 0x01000100u && k < 2) bt = 0;
      // raw[0..17] + old overlap -> o[], raw[18..35] -> new overlap, written as
      // each raw value is produced (no 36-entry temporary); frequency
      // inversion rides on the signs of the windows and of stp
      if (bt == 2) {
        float st[18];
#pragma unroll
        for (int q = 0; q < 9; q++) {
          st[q] = stp[q].x;
          st[17 - q] = stp[q].y;
        }
        // raw[pos] = sum over the windows wi with 0 <= pos-6-6wi < 12 of
        // (sum_m x[wi+3m] cosN12[m][p]) * win[2][p], p = pos-6-6wi (imdct.go:88-94)
#pragma unroll
        for (int pos = 0; pos < 36; pos++) {
          float raw = 0.0f;
#pragma unroll
          for (int wi = 0; wi < 3; wi++) {
            const int p = pos - 6 - 6 * wi;
            if (p < 0 || p >= 12) continue;
            float sum = 0.0f;
#pragma unroll
            for (int m = 0; m < 6; m++) sum += x[wi + 3 * m] * dct4::kCos12[p][m];
            raw += sum * dct4::kWin12[p];
          }
          if (pos & 1) raw *= sodd;  // (pos and pos - 18 have the same parity)
          if (pos < 18) o[pos] = raw + st[pos];
          else st[pos - 18] = self(act, raw, st[pos - 18]);
        }
#pragma unroll
        for (int q = 0; q < 9; q++) stp[q] = (f2){st[q], st[17 - q]};
      } else {
        // the 18 distinct sums are a DCT-IV of size 18 (dct4_18.h):
        // sum_m x[m] cosN36[m][q] = X[9+q], sum_m x[m] cosN36[m][18+q] = -X[8-q];
        // packed, pair k = (X[2k], X[17-2k]) holds X[9+q] and X[8-q] of one q
        f2 P[9];
        dct4::dct4_18_pk(x, P);
        const float4* Wq = sh.winp[bt][lane_fresh() & 1];
        // (the overlap of an absent channel stays frozen: frame.go Decode
        // touches ch < nch only; stereo granules need no per-lane select)
        auto overlap = [&](auto frozen) {
#pragma unroll
          for (int kk = 0; kk < 9; kk++) {
            const int q = kk <= 4 ? 8 - 2 * kk : 2 * kk - 9;
            const float za = kk <= 4 ? P[kk].y : P[kk].x;  // X[9+q]
            const float zb = kk <= 4 ? P[kk].x : P[kk].y;  // X[8-q]
            const float4 w = Wq[q];
            // (o[q], o[17-q]) = X[9+q] (W[q], -W[17-q]) + stp[q];
            // new stp[q] = X[8-q] (-W[18+q], -W[35-q])   (signs folded in w)
            const f2 oq = pfma(bcast(za), (f2){w.x, w.y}, stp[q]);
            o[q] = oq.x;
            o[17 - q] = oq.y;
            const f2 ns = bcast(zb) * (f2){w.z, w.w};
            if constexpr (decltype(frozen)::value)
              stp[q] = (f2){self(act, ns.x, stp[q].x), self(act, ns.y, stp[q].y)};
            else
              stp[q] = ns;
          }
        };
        if (nch == 2) overlap(std::false_type{});
        else overlap(std::true_type{});
      }
    }
    // ---- a hot granule? the first test (every granule) ----
#if MP3G_HOT_CHECK
    const bool hot1 = __builtin_amdgcn_ballot_w64((act ? max_abs18(o) : 0.0f) > kHotS) != 0;
#endif
    stamp(3);
    // prefetch the next granule: lands during the matrixing and window phases
    // (issued here, not at the top, so its 13 VGPRs are not live across the
    // front end and IMDCT); buffer resources with SGPR bases and 32-bit lane
    // offsets: no 64-bit pointer is kept (and spilled) in VGPRs -- a spill
    // reload costs an s_waitcnt vmcnt(0), which would also wait for this
    // prefetch
    const bool more = g + 1 < end;
#if MP3G_FAST_DESC_VGPR
    uint32_t pdw;  // the descriptor two granules ahead, one dword per lane
#else
    uint4 pd = {0, 0, 0, 0};
#endif
    // issued unconditionally (straight-line vmcnt accounting, as the PCM
    // stores below): past the chunk the resources have no records
    {
      // the next granule's descriptor is already in LDS (loaded one granule
      // earlier): its count1s bound this prefetch; the descriptor two ahead
      // is loaded with it
      {
#if MP3G_FAST_DESC_VGPR
        const uint32_t nh = desc_word(dvn, 0);
        const int c0 = (int)(desc_word(dvn, 2) & 0xffffu);
        const int c1 = (int)(desc_word(dvn, 20) & 0xffffu);
#else
        const uint32_t nh = __builtin_amdgcn_readfirstlane(s.descn.header);
        const uint2 n0 = *reinterpret_cast<const uint2*>(&s.descn.ch[0]);
        const uint2 n1 = *reinterpret_cast<const uint2*>(&s.descn.ch[1]);
        const int c0 = (int)(__builtin_amdgcn_readfirstlane(n0.x) & 0xffffu);
        const int c1 = (int)(__builtin_amdgcn_readfirstlane(n1.x) & 0xffffu);
#endif
        const int lim = ch ? (hdr_nch(nh) == 2 ? c1 : 0) : c0;
        load_lines_lim(coef, g + 1, lane, cw, more ? (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t)) : 0, lim);
      }
#if MP3G_FAST_DESC_VGPR
      pdw = load_desc_dword(gran, g + 2, lane_fresh(), g + 2 < end);
#else
      if (lane < 10) {
        const bool more2 = g + 2 < end;
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<mp3g_granule*>(gran + g + 2), (short)0, more2 ? (int)sizeof(mp3g_granule) : 0, 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, lane * 16, 0, 0);
        pd = make_uint4(v[0], v[1], v[2], v[3]);
      }
#endif
    }

    // ---- matrixing (frame.go:642-648): S rows into the ring (lane (ch, sb)
    //      writes its 18 slots), then one lane per (ch, slot) turns its row into
    //      the 32 distinct values X of V = synthNWin * S with an in-lane fast
    //      DCT-II-32 on float pairs (dct32.h), in place ----
    if (need_v && act) {
#pragma unroll
      for (int j = 0; j < 18; j++) s.ring[ch][k][kHist + j] = o[j];
    }
    wave_sync();
#if MP3G_HOT_CHECK
    // the second test (rare) on S in the ring: the granule's zone is redone
    // in the reference's order after the pass (a granule whose V feeds no
    // output needs no zone)
    if (hot1 && need_v && slot_sums_hot(s.ring, nch)) {
      record_hot(s, nz, gran, g, out_first, end);
      if constexpr (kHotCount) n_flagged++;
    }
#endif
    stamp(4);
    {
      const int slot = lane & 31;  // lane = (ch, slot), slots 0..17
      if (need_v && act && slot < 18) {
        float* colu = &s.ring[ch][0][kHist + slot];  // S[k] / X at colu[kSlots * k]
        dct32::f2 sp[16];
#pragma unroll
        for (int q = 0; q < 16; q++) sp[q] = (dct32::f2){colu[kSlots * 2 * q], colu[kSlots * (2 * q + 1)]};
        dct32::dct2_32_to(sp, [&](int t, dct32::f2 v) {
          colu[kSlots * dct32::kColX[t]] = v.x;
          colu[kSlots * dct32::kColY[t]] = v.y;
        });
      }
    }
    stamp(5);
    wave_sync();  // ring slots of this granule written before the window reads them

    // ---- next granule in: raw/eo (dead after the matrixing) and the
    //      descriptor (not read again this granule) take the prefetch now,
    //      before the PCM stores are issued -- vmcnt counts loads and stores in
    //      issue order, so a wait for the prefetch after the stores would wait
    //      for the stores too ----
    // (lane recomputed: the two LDS addresses kept live across the granule
    // were spilled, and a scratch reload here waits for the PCM stores)
#if MP3G_FAST_DESC_VGPR
    dv = dvn;
    dvn = pdw;
#else
    if (more) {
      const int l = lane_fresh();
      if (l < 10) {
        reinterpret_cast<uint4*>(&s.desc)[l] = reinterpret_cast<const uint4*>(&s.descn)[l];
        reinterpret_cast<uint4*>(&s.descn)[l] = pd;
      }
    }
#endif

    window_store(g, out, nch);
    wave_sync();  // ring reads done
    stamp(6);

    // ---- history shift (channels this granule touched): lane = (c, column),
    //      slots 18..33 -> 0..15 as 8-B moves; not after a replayed granule
    //      whose V feeds nothing (its slots hold no X; the next granule is a
    //      replay too and rewrites the history before any window reads it) ----
    if (ch < nch && need_v) {
      f2* col = reinterpret_cast<f2*>(&s.ring[ch][k][0]);
#pragma unroll
      for (int q = 0; q < 8; q++) col[q] = col[9 + q];
    }
    wave_sync();
    stamp(7);
  }
  if constexpr (kStamp) rt[2] = __builtin_amdgcn_s_memrealtime();

  // Frame.store / vVec after the chunk's last granule (frame.go:48-49)
  auto export_state = [&](const f2 (&st)[9]) {
    if (!(cd.flags & kChunkStateOut)) return;
    mp3g_state* so = state_out + cd.stream;
    const int c = lane_fresh() >> 5, kk = lane_fresh() & 31;
    const float sg = (kk & 1) ? -1.0f : 1.0f;
#pragma unroll
    for (int q = 0; q < 9; q++) {
      so->store[c][kk][q] = (q & 1) ? st[q].x * sg : st[q].x;
      so->store[c][kk][17 - q] = (q & 1) ? st[q].y : st[q].y * sg;
    }
    for (int e = lane_fresh(); e < 2 * 1024; e += kLanes) {
      const int cc = e >> 10, blk = (e >> 6) & 15, i = e & 63;
      so->vvec[cc][64 * blk + i] = blk < 15 ? v_from_x(&s.ring[cc][0][kHist - 1 - blk], i) : 0.0f;
    }
  };
  export_state(stp);

  // ---- hot zones (rare): redo their granules in the reference's order from
  //      their replay start (exact entry state) and overwrite their PCM; a
  //      zone ends two granules after the last hot granule it meets.  Past
  //      a zone the fast pass's own output stands: it depends on no hot
  //      granule's hybrid output.  A zone reaching the chunk end also rewrites
  //      the exported state.  (The zones' stages mirror the fast loop's, in
  //      the reference's operation order: exact_granule.) ----
  // ---- hot zones (rare), deferred: appended to the launch's zone list as
  //      chunks of their own, which the exact v4 kernel then decodes in the
  //      reference's order over many waves (launch_fast: the zone launch).
  //      The list has room for every zone of every chunk (kZoneListPerChunk),
  //      so the production builds carry no in-wave pass (and no scratch: its
  //      registers spilled 1.9 KB per lane); the in-wave pass below runs in
  //      the diagnostic (kStamp) builds only, which pass no list. ----
  // aux (kernels.h ZoneScratch): [0] zones listed, [2] the list's capacity,
  // [4..7] the hot-granule counters (kHotCount builds), the list from byte 32
  // (one pointer: the three fields as arguments of their own cost the granule
  // loop SGPRs, 26 spilled instead of 15, +1 % at c3)
  uint32_t* const hot_count = aux ? aux + 4 : nullptr;
  if (!kStamp && nz) {
    uint32_t* const zone_count = aux;
    ChunkDesc* const zone_list = reinterpret_cast<ChunkDesc*>(aux + 8);
    const uint32_t zone_cap = __builtin_amdgcn_readfirstlane(aux[2]);
    // every zone as pieces of at most kZonePiece granules (kernels.h), one
    // atomic for all of them
    uint32_t n_pieces = 0;
    for (uint32_t i = 0; i < nz; i++) {
      const uint32_t zs = __builtin_amdgcn_readfirstlane(s.zone[i][0]), ze = __builtin_amdgcn_readfirstlane(s.zone[i][1]);
      n_pieces += (ze - zs + kZonePiece - 1) / kZonePiece;
    }
    uint32_t base = 0;
    if (lane_fresh() == 0) base = atomicAdd(zone_count, n_pieces);
    base = __builtin_amdgcn_readfirstlane(base);  // lane 0 is the first active lane
    for (uint32_t i = 0; i < nz; i++) {
      const uint32_t zs = __builtin_amdgcn_readfirstlane(s.zone[i][0]), ze = __builtin_amdgcn_readfirstlane(s.zone[i][1]);
      const uint32_t np = (ze - zs + kZonePiece - 1) / kZonePiece;
      const uint32_t l = (uint32_t)lane_fresh();
      // (always below the capacity: zone_list_capacity counts every piece)
      if (l < np && base + l < zone_cap) {
        const uint32_t ps = zs + l * kZonePiece, pe = min(ps + kZonePiece, ze);
        ChunkDesc z;
        z.out_first = ps;
        z.stream_first = cd.stream_first;
        z.n_out = pe - ps;
        z.stream = cd.stream;
        // entry state as the chunk's (the zone launch replays the piece's halo
        // from it or from zero, as for any chunk); the exported state when
        // the piece ends the chunk (it then overwrites this pass's export)
        z.flags = (cd.flags & kChunkStateIn) | (pe == end ? (cd.flags & kChunkStateOut) : 0u);
        z.reserved = 0;
        zone_list[base + l] = z;
      }
      base += np;
    }
  }
  // (counting build) a chunk counts its flagged granules even when none of
  // them recorded a zone -- a replayed granule whose V feeds no output is
  // hot all the same (counter [2] is every hot granule the fast pass met)
  if constexpr (!kStamp && kHotCount) {
    if (nz || n_flagged) {
      uint32_t n_out = 0;
      for (uint32_t i = 0; i < nz; i++)
        n_out += __builtin_amdgcn_readfirstlane(s.zone[i][1]) - __builtin_amdgcn_readfirstlane(s.zone[i][0]);
      if (lane_fresh() == 0) {
        atomicAdd(hot_count + 0, n_out);
        atomicAdd(hot_count + 1, nz);
        atomicAdd(hot_count + 2, n_flagged);
      }
    }
  }
  if (kStamp && nz) {
    f2 zst[9];  // the zones' own overlap state (nothing flows in from the fast pass)
    uint32_t done = 0;  // the exact state in zst / the ring is valid for granules < done
    bool have = false;
    uint32_t n_out = 0, n_run = 0;  // for hot_count (kernels.h kHotCounters)
    for (uint32_t i = 0; i < nz; i++) {
      const uint32_t zs = __builtin_amdgcn_readfirstlane(s.zone[i][0]);
      uint32_t ze = __builtin_amdgcn_readfirstlane(s.zone[i][1]);
      if (have && ze <= done) continue;
      uint32_t gz = done;
      if (!have || zs > done) {  // a fresh zone: replay from its start's replay start
        ChunkDesc cr = cd;
        cr.out_first = zs;
        cr.n_out = end - zs;
        uint64_t wz;
        int zin[2];
        prologue(cr, gran, &wz, zin, lane_fresh());
        init_state(s, sin, zin, lane_fresh(), zst);
        gz = __builtin_amdgcn_readfirstlane((uint32_t)wz);
        have = true;
      }
      for (; gz < ze; gz++) {
        const bool nv = replay_needs_v(gran, gz, zs);
        n_run++;
        n_out += gz >= zs ? 1u : 0u;
        if (exact_granule(gran, coef, pcm, s, sh, gz, gz >= zs, nv, zst)) {
          const uint32_t e = zone_end(gran, gz, end);
          ze = e > ze ? e : ze;
        }
      }
      done = gz;
    }
    if (done >= end) export_state(zst);
    // (rare: one vector atomic per counter from lane 0 of a chunk with zones)
    if (kHotCount && hot_count && lane_fresh() == 0) {
      atomicAdd(hot_count + 0, n_out);
      atomicAdd(hot_count + 1, nz);
      atomicAdd(hot_count + 2, n_flagged);
      atomicAdd(hot_count + 3, n_run);
    }
  }
  if constexpr (kStamp) {
    rt[3] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      for (int p = 0; p < kPhases; p++) stamps[(size_t)ci * kFastStampSlots + p] = ph[p];
      for (int p = 0; p < 4; p++) stamps[(size_t)ci * kFastStampSlots + kPhases + p] = rt[p];
    }
  }
}

}  // namespace v3
}  // namespace mp3g
