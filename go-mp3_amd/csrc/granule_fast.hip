// granule_fast.hip -- MP3G_MODE_FAST granule decode, v3 (gfx950).
//
// Same contract, chunk/halo decomposition and front end as the exact kernels
// (reference internal/frame/frame.go:121-688), but the three transforms are
// evaluated in reassociated, FMA-contracted float32, so PCM is within +-1 LSB
// of the reference instead of bit-identical (north star tolerance; measured
// by tests/test_gpu_parity.py::test_fast_mode_*).
//
// Work decomposition: ONE WAVE PER CHUNK.  A 64-lane workgroup walks its chunk
// granule by granule with no s_barrier-level cross-wave traffic:
//   front end   lane = (ch, sb): the 18 lines of its subband -- requantize
//               (gather through the reorder table), MS/IS with the partner
//               channel via a lane^32 shuffle, antialias butterflies with the
//               neighbouring subbands via lane+-1 shuffles;
//   IMDCT       lane = (ch, sb): 36-point (or 3 x 12-point) IMDCT in registers,
//               the overlap `store` lives in the lane's VGPRs for the whole
//               chunk, frequency inversion;
//   matrixing   V = synthNWin * S has 32 distinct values X (DSP identity,
//               dsp_tables.h FastTables); the lane pair (sb, 31-sb) folds
//               S into even/odd halves (lane^31 shuffle), then lane = (ch, m)
//               computes X_m for all 18 time slots: 16 FMAs per value against
//               its coefficient row held in VGPRs;
//   window      lane = (ch, i): 16-tap window over the X ring with the V->X
//               signs folded into the taps (VGPRs), 18 outputs per lane, s16
//               packed (L,R) with one lane^32 exchange per slot pair.
// LDS per wave ~14 KB (raw/eo union, X ring 2 x 34 x 32, descriptor, IMDCT
// windows) -> 11 resident waves per CU.
// (compiled as part of kernels.hip, after granule_common.hip)
#pragma clang fp contract(fast)
#include <type_traits>

#include "dct32.h"
#include "dct4_18.h"
#include "xlane.h"

namespace mp3g {
namespace v3 {
// Independent chunks (one per wave) per workgroup, sharing the read-only
// tables.  8 waves: 2 workgroups (16 waves) per CU, the shared tables held
// twice per CU instead of four times (2-3 % faster than 4-wave workgroups on
// c2 and c3, tools/gpu_ab.sh; 16 waves measured the same).
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
#ifndef MP3G_FAST_STRAIGHT
#define MP3G_FAST_STRAIGHT 1
#endif
#ifndef MP3G_FAST_NT_STORE
#define MP3G_FAST_NT_STORE 1  // non-temporal PCM stores: c2 -1.9 %, c3 -0.8 % (tools/gpu_ab.sh)
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
  uint32_t lband[kCombos][32];
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
  // requantization exponents n4 / 4 (float16, exact) of the long bands
  // [ch][sfb] and short bands [ch][sfb][win]
  _Float16 expo[2 * 22 + 2 * 39];
};

// Raw coefficients of lane (ch, sb) of granule g: its 18 lines, 36 B at
// coef[g][ch][18 sb], as 9 dwords (two int16 each) by three 12-B buffer loads
// through a per-granule resource (SGPR base, 32-bit lane offset).
// (nbytes = 0: a resource without records -- the loads return 0 and touch no memory)
__device__ __forceinline__ void load_lines(const int16_t* coef, uint32_t g, int lane, uint32_t cw[9],
                                           int nbytes = (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t))) {
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int16_t*>(coef + (size_t)g * MP3G_COEF_PER_GRANULE), (short)0, nbytes, 0x00020000);
  const int off = (lane >> 5) * 1152 + (lane & 31) * 36;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(rc, off + 12 * i, 0, 0);
    cw[3 * i] = v[0];
    cw[3 * i + 1] = v[1];
    cw[3 * i + 2] = v[2];
  }
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
// x: one slot of the column-major ring (X[m] at x[kSlots * kPosOfM[m]]).
__device__ __forceinline__ float v_from_x(const float* x, int i) {
  if (i < 16) return x[kSlots * dct32::kPosOfM[16 + i]];
  if (i == 16) return 0.0f;
  if (i < 48) return -x[kSlots * dct32::kPosOfM[48 - i]];
  return -x[kSlots * dct32::kPosOfM[i - 48]];
}

}  // namespace

// kStamp: diagnostic build -- per-phase s_memtime cycle sums of every wave go
// to `stamps` (kPhases per workgroup); never used for output.
constexpr int kPhases = 8;
template <bool kStamp>
__global__ void __launch_bounds__(kLanes * kWaves, MP3G_FAST_WAVES_PER_SIMD)
granule_fast_kernel(const ChunkDesc* __restrict__ chunks, uint32_t n_chunks, const mp3g_granule* __restrict__ gran,
                    const int16_t* __restrict__ coef, const mp3g_state* __restrict__ state_in,
                    mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm,
                    unsigned long long* __restrict__ stamps) {
  unsigned long long ph[kPhases] = {}, tprev = 0, rt[4] = {};
  if constexpr (kStamp) rt[0] = __builtin_amdgcn_s_memrealtime();
  auto stamp = [&](int p) {
    if constexpr (kStamp) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[p] += t - tprev;
      tprev = t;
    }
  };
  __shared__ SharedSmem sh;
  __shared__ WaveSmem wsm[kWaves];
#ifdef MP3G_FAST_LDS_PAD
  // diagnostic builds only (tools/build_variant.sh): extra LDS per workgroup
  // to lower the resident workgroups per CU (occupancy sensitivity)
  __shared__ char ldspad[MP3G_FAST_LDS_PAD];
  if (n_chunks == 0xffffffffu) reinterpret_cast<volatile char*>(ldspad)[threadIdx.x] = 0;
#endif
  {
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
    for (int e = t; e < kCombos * 32; e += kLanes * kWaves) (&sh.lband[0][0])[e] = (&g_fast.lband[0][0])[e];
  }
  __syncthreads();  // the only workgroup barrier: the waves are independent from here on
  const int lane = threadIdx.x & (kLanes - 1);
  // wave-uniform in an SGPR: the chunk descriptor then comes in by scalar
  // loads and its fields (pointers, counts) stay out of the VGPR budget
  const uint32_t ci = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
  if (ci >= n_chunks) return;
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
#ifdef MP3G_EXP_NOHALO
  const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)cd.out_first);  // timing experiment only: wrong PCM
#else
  const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)w64);
#endif
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
  if (w < end) {
    load_lines(coef, w, lane, cw);
    if (lane < 10) reinterpret_cast<uint4*>(&s.desc)[lane] = reinterpret_cast<const uint4*>(gran + w)[lane];
  }
  wave_sync();

  // PCM of a granule: one dword (L, R) per lane and slot pair
  uint32_t pk[9] = {};
  const int hi = lane >> 5;

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
  for (uint32_t g = w; g < end; g++) {
#ifdef MP3G_EXP_SALU
    // timing experiment only (tools/build_variant.sh): extra scalar ALU work
    {
      uint32_t d = g;
#pragma unroll
      for (int i = 0; i < MP3G_EXP_SALU; i++) asm volatile("s_add_u32 %0, %0, 1" : "+s"(d));
    }
#endif
#ifndef MP3G_EXP_NOPRIO
    {
      const uint32_t left4 = 4u * (end - g);  // priority floor(4 * left / span), 3 .. 0
      if (left4 > span3) __builtin_amdgcn_s_setprio(3);
      else if (left4 > span2) __builtin_amdgcn_s_setprio(2);
      else if (left4 > span) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
    const bool out = g >= out_first;
    // does a replayed granule's V feed anything? (see v2 / DESIGN.md halo)
    bool need_v = true;
    if (!out && g + 1 < out_first) need_v = hdr_nch(gran[g + 1].header) < hdr_nch(s.desc.header);
    // wave-uniform (SGPR): the per-combo tables below become scalar loads
    const uint32_t h = __builtin_amdgcn_readfirstlane(s.desc.header);
    const int nch = hdr_nch(h), combo = hdr_combo(h);
    const bool act = ch < nch;
    // the channels' scalar parameters in SGPRs (one 8-B LDS read each):
    // dword 0 = count1 | global_gain << 16 | scalefac_scale << 24,
    // dword 1 = preflag | win_switch_flag << 8 | block_type << 16 | mixed_block_flag << 24
    uint32_t cp0[2], cp1[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const uint2 v = *reinterpret_cast<const uint2*>(&s.desc.ch[c]);
      cp0[c] = __builtin_amdgcn_readfirstlane(v.x);
      cp1[c] = __builtin_amdgcn_readfirstlane(v.y);
    }
    auto is_short = [](uint32_t d1) { return (d1 & 0x00ffff00u) == 0x00020100u; };  // win_switch 1, block_type 2
    // wave-uniform: every channel of this granule is a long block (no reorder)
    const bool all_long = !is_short(cp1[0]) && (nch == 1 || !is_short(cp1[1]));
    // this lane's channel (lanes of an absent channel mirror channel 0's block
    // layout: no extra divergence)
    const uint32_t d0 = (act && ch) ? cp0[1] : cp0[0], d1 = (act && ch) ? cp1[1] : cp1[0];

    // ---- per-granule front-end parameters: band exponents (long bands only
    //      when no channel has short blocks) ----
    {
      // long bands: lane = (c, sfb), 44 lanes
      const int e = lane_fresh();
      if (e < 44) {
        const int c = e >= 22, sfb = e - 22 * c;
        const uint32_t a0 = c ? cp0[1] : cp0[0], a1 = c ? cp1[1] : cp1[0];
        const int v = (int)((a0 >> 16) & 0xffu) - 210 -
                      ((a0 >> 24) ? 4 : 2) * ((int)s.desc.ch[c].scalefac_l[sfb] + (int)(a1 & 0xffu) * kPretab(sfb));
        s.expo[e] = (_Float16)(0.25f * (float)v);
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
      const uint32_t lb = sh.lband[combo][k];
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
      // live (in VGPRs) across the granule loop
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint32_t*>(&g_fast.linfo[combo][0]), (short)0, 576 * 4, 0x00020000);
      const int L0 = 18 * (lane_fresh() & 31);
#pragma unroll
      for (int j = 0; j < 18; j++) {
        const int L = L0 + j;
        const uint32_t inf = __builtin_amdgcn_raw_buffer_load_b32(rl, 4 * L, 0, 0);
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
      wave_sync();  // staged lines read before the slots are reused
    }
    stamp(1);
    // ---- MS / intensity stereo with the partner channel's lane (frame.go:304-420) ----
    if (nch == 2 && hdr_mode(h) == 1 && (h & 0x30u)) {
      const mp3g_channel& C0 = s.desc.ch[0];
      const int c1r = (int)(cp0[1] & 0xffffu);
      const int msmax = max((int)(cp0[0] & 0xffffu), c1r);
#ifdef MP3G_EXP_NOIS
      const bool ms = h & 0x20u, is = false;  // timing experiment only: wrong PCM
#else
      const bool ms = h & 0x20u, is = h & 0x10u;
#endif
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
          const uint32_t lb = sh.lband[combo][k0];
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
    stamp(3);
    // prefetch the next granule: lands during the matrixing and window phases
    // (issued here, not at the top, so its 13 VGPRs are not live across the
    // front end and IMDCT); buffer resources with SGPR bases and 32-bit lane
    // offsets: no 64-bit pointer is kept (and spilled) in VGPRs -- a spill
    // reload costs an s_waitcnt vmcnt(0), which would also wait for this
    // prefetch
    const bool more = g + 1 < end;
    uint4 pd = {0, 0, 0, 0};
#if MP3G_FAST_STRAIGHT
    // issued unconditionally (straight-line vmcnt accounting, as the PCM
    // stores below): past the chunk the resources have no records
    {
      load_lines(coef, g + 1, lane, cw, more ? (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t)) : 0);
      if (lane < 10) {
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<mp3g_granule*>(gran + g + 1), (short)0, more ? (int)sizeof(mp3g_granule) : 0, 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, lane * 16, 0, 0);
        pd = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
#else
    if (more) {
      load_lines(coef, g + 1, lane, cw);
      if (lane < 10) {
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<mp3g_granule*>(gran + g + 1), (short)0, (int)sizeof(mp3g_granule), 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, lane * 16, 0, 0);
        pd = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
#endif

    // ---- matrixing (frame.go:642-648): S rows into the ring (lane (ch, sb)
    //      writes its 18 slots), then one lane per (ch, slot) turns its row into
    //      the 32 distinct values X of V = synthNWin * S with an in-lane fast
    //      DCT-II-32 on float pairs (dct32.h), in place ----
    if (need_v && act) {
#pragma unroll
      for (int j = 0; j < 18; j++) s.ring[ch][k][kHist + j] = o[j];
    }
    wave_sync();
    stamp(4);
    {
      const int slot = lane & 31;  // lane = (ch, slot), slots 0..17
      if (need_v && act && slot < 18) {
        float* colu = &s.ring[ch][0][kHist + slot];  // S[k] / X at colu[kSlots * k]
        dct32::f2 sp[16];
#pragma unroll
        for (int q = 0; q < 16; q++) sp[q] = (dct32::f2){colu[kSlots * 2 * q], colu[kSlots * (2 * q + 1)]};
#ifdef MP3G_EXP_NODCT
        // timing experiment only: X = S (wrong PCM)
#pragma unroll
        for (int t = 0; t < 16; t++) {
          colu[kSlots * dct32::kColX[t]] = sp[t].x;
          colu[kSlots * dct32::kColY[t]] = sp[t].y;
        }
        if (false)
#endif
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
    if (more && lane < 10) reinterpret_cast<uint4*>(&s.desc)[lane] = pd;

    // ---- 16-tap window over the X ring -> s16 PCM, stored straight to HBM ----
    // (lanes of an absent channel compute values that are never stored)
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
#ifdef MP3G_EXP_HALFWIN
          if (t & 1) continue;  // timing experiment only: half the taps (wrong PCM)
#endif
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
      if (nch == 2) pack(std::false_type{});
      else pack(std::true_type{});
      // stored right away: a store's data registers are free again once it
      // has issued (no s_waitcnt before their reuse on gfx950), and the loads
      // this wave waits for next were issued before these stores
#if !MP3G_FAST_STRAIGHT
      uint32_t* P = reinterpret_cast<uint32_t*>(pcm + (size_t)g * 1152);
#pragma unroll
      for (int p = 0; p < 9; p++) {
#if MP3G_FAST_NT_STORE
        __builtin_nontemporal_store(pk[p], &P[32 * (2 * p + hi) + k]);
#else
        P[32 * (2 * p + hi) + k] = pk[p];
#endif
      }
#endif
    }
#if MP3G_FAST_STRAIGHT
    {
      // issued for replayed granules too, through a resource with no records
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          pcm + (size_t)g * 1152, (short)0, out ? MP3G_PCM_BYTES_PER_GRANULE : 0, 0x00020000);
#pragma unroll
      for (int p = 0; p < 9; p++)
        __builtin_amdgcn_raw_buffer_store_b32(pk[p], rp, 4 * (32 * (2 * p + hi) + k), 0, MP3G_FAST_NT_STORE ? 2 : 0);
    }
#endif
#ifndef MP3G_EXP_NOSYNC_SHIFT
    wave_sync();  // ring reads done
#endif
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
#ifndef MP3G_EXP_NOSYNC_SHIFT2
    wave_sync();
#endif
    stamp(7);
  }
  if constexpr (kStamp) rt[2] = __builtin_amdgcn_s_memrealtime();

  if (cd.flags & kChunkStateOut) {
    mp3g_state* so = state_out + cd.stream;
#pragma unroll
    for (int q = 0; q < 9; q++) {
      so->store[ch][k][q] = (q & 1) ? stp[q].x * sodd : stp[q].x;
      so->store[ch][k][17 - q] = (q & 1) ? stp[q].y : stp[q].y * sodd;
    }
    for (int e = lane; e < 2 * 1024; e += kLanes) {
      const int c = e >> 10, blk = (e >> 6) & 15, i = e & 63;
      so->vvec[c][64 * blk + i] = blk < 15 ? v_from_x(&s.ring[c][0][kHist - 1 - blk], i) : 0.0f;
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
