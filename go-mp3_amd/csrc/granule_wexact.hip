// granule_wexact.hip -- MP3G_MODE_EXACT granule decode, v4 (gfx950): the
// reference's Frame.Decode (internal/frame/frame.go:121-688) bit for bit, in
// the fast kernel's work decomposition.
//
// v2 (granule_fused.hip) decodes a chunk with a 256-thread workgroup and four
// barriers per granule; its waves spend most of their time at those barriers
// and in LDS round trips.  v4 gives a chunk to ONE wave, eight independent
// waves per workgroup, 16 per CU, as the fast kernel v3 does, and runs every
// stage in the reference's operation order (one rounding per product and per
// sum, sums from 0.0 in the reference's index order):
//   front end   lane = (ch, sb): requantization through the proven table
//               ldexp(req[n4 & 3][|x|], n4 >> 2) (long blocks straight from
//               the lane's registers, short / mixed blocks through the reorder
//               gather), MS / IS stereo and antialias butterflies as in v3's
//               exact stages;
//   IMDCT       lane = (ch, sb): imdctWin's sums in order (imdct_exact);
//   matrixing   lane = (ch, slot): the 32 distinct V values X[m] (rows
//               synthNWin[m-16] / -synthNWin[48-m]: bit-negated sums) and
//               V[16], the residue of the ~1e-16 row 16, each a 32-term sum
//               in order, into the X ring (column 32 holds V[16]);
//   window      lane = (ch, i): U * D rounded, summed j = 0..15 from 0.0,
//               times 32767, truncated and clamped (frame.go:649-669); V[16]
//               enters output 16's even taps.
// The exported vVec is rebuilt from X with 0 - x for the negated rows (the
// reference's sums from +0 never give -0).  Tested bit-exact against the
// oracle's PCM and state (tests/test_gpu_parity.py, exact mode).
// (compiled in kernels_fast.hip after granule_fast.hip: shares its stages)
#pragma clang fp contract(off)

namespace mp3g {
namespace v4 {

using namespace v3;

constexpr int kXWaves = 8;
constexpr int kCols = 33;     // 32 X columns + V[16]
constexpr int kColV16 = 32;

// read-only tables, one copy per workgroup
struct __align__(16) XSharedSmem {
  float isr[8][2];            // as v3's SharedSmem (stereo_stage)
  uint32_t lband[kCombos][32];
  __device__ uint32_t lband_at(int c, int k) const { return lband[c][k]; }
  float dwin[32][20];         // window taps (below), rows padded to 20 floats
  float win[4][36];           // imdctWinData (imdct.go:21-57)
};

struct __align__(16) XWaveSmem {
  float ring[2][kCols][kSlots];
  mp3g_granule desc;
  mp3g_granule descn;  // the next granule's descriptor (its count1s bound its prefetch)
  _Float16 expo[2 * 22 + 2 * 39];
};

namespace {

// Long-block requantization from the lane's registers in the reference's
// rounding (every line of a long block is processed or zero).
__device__ __forceinline__ void front_long_exact(float x[18], const uint32_t cw[9], const XWaveSmem& s,
                                                 const XSharedSmem& sh, const GranParams& P, int ch, int k) {
  int xi[18];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    xi[2 * q] = (int)(int16_t)(cw[q] & 0xffffu);
    xi[2 * q + 1] = (int)(int16_t)(cw[q] >> 16);
  }
  const uint32_t lb = sh.lband[P.combo][k];
  _Float16 ex[9];
#pragma unroll
  for (int q = 0; q < 9; q++)
    ex[q] = s.expo[22 * ch + (int)(lb & 31u) + __builtin_popcount((lb >> 5) & ((2u << (2 * q)) - 1u))];
  // lines >= count1 are zero (the parse's guarantee) and requantize to +0,
  // the value the reference leaves there
#pragma unroll
  for (int j = 0; j < 18; j++) x[j] = requant_exact(xi[j], ex[j >> 1]);
}

// +0.0 the compiler cannot see: every reference sum starts from +0 (`sum :=
// float32(0)`), and with a literal 0 and literal negative constants the AMDGPU
// backend folds (0 - a) + b into b - a, which is -0 where the reference has
// +0 (an all-zero subband's overlap `store` came out -0).  Starting each sum
// from this register keeps the reference's zeros.
__device__ __forceinline__ float ozero() {
  float z = 0.0f;
  asm volatile("" : "+v"(z));
  return z;
}

// The reference's float32 constants of the IMDCT and matrixing sums as
// instruction literals (every lane multiplies by the same entry): no table
// loads, no registers (generated from dsp_tables.cpp, tests/test_tables.py).
#include "exact_consts.inc"

// imdct.Win + overlap-add + frequency inversion of subband k in the
// reference's order (imdct.go:83-108, frame.go:454-486), as v3's imdct_exact
// with literal cosines and the window row from LDS.  stp holds the overlap with the
// frequency-inversion signs folded in; negation commutes with rounding.
__device__ __forceinline__ void imdct_exact_s(const float x[18], int bt, const float* win, int k, bool act,
                                              f2 stp[9], float o[18]) {
#pragma clang fp contract(off)
  const float sodd = (k & 1) ? -1.0f : 1.0f;
  float st[18];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    st[q] = stp[q].x;
    st[17 - q] = stp[q].y;
  }
  const float z0 = ozero();
  if (bt == 2) {
    // out[6 wi + p + 6] += (sum_m in[wi + 3m] cosN12[m][p]) win[2][p], wi ascending
#pragma unroll
    for (int pos = 0; pos < 36; pos++) {
      float raw = z0;
#pragma unroll
      for (int wi = 0; wi < 3; wi++) {
        const int p = pos - 6 - 6 * wi;
        if (p < 0 || p >= 12) continue;
        float sum = z0;
#pragma unroll
        for (int m = 0; m < 6; m++) sum = sum + x[wi + 3 * m] * kXC12[m][p];
        raw = raw + sum * win[p];
      }
      const float f = (pos & 1) ? raw * sodd : raw;
      if (pos < 18) o[pos] = f + st[pos];
      else if (act) st[pos - 18] = f;
    }
  } else {
    // the 18 distinct columns of cosN36 (DspTables::cos36_distinct):
    // col(17 - p) = -col(p), col(53 - p) = col(p) bit for bit
    // the 18 sums, each over m ascending (the cosines are instruction literals)
    float sum[18];
#pragma unroll
    for (int q = 0; q < 18; q++) sum[q] = z0;
#pragma unroll
    for (int m = 0; m < 18; m++) {
#pragma unroll
      for (int q = 0; q < 18; q++) sum[q] = sum[q] + x[m] * kXC36[m][q];
    }
#pragma unroll
    for (int q = 0; q < 9; q++) {
      const float sa = sum[q], sb = sum[9 + q];
      // raw[q] = sa, raw[17-q] = -sa, raw[18+q] = raw[35-q] = sb (times the window)
      const int p0 = q, p1 = 17 - q, p2 = 18 + q, p3 = 35 - q;
      const float r0 = sa * win[p0], r1 = (z0 - sa) * win[p1];
      const float r2 = sb * win[p2], r3 = sb * win[p3];
      o[p0] = ((p0 & 1) ? r0 * sodd : r0) + st[p0];
      o[p1] = ((p1 & 1) ? r1 * sodd : r1) + st[p1];
      if (act) {
        st[p2 - 18] = (p2 & 1) ? r2 * sodd : r2;
        st[p3 - 18] = (p3 & 1) ? r3 * sodd : r3;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 9; q++) stp[q] = (f2){st[q], st[17 - q]};
}

// V = synthNWin * S of one time slot in the reference's order: the 32
// distinct values X[m] to their ring columns and V[16] to column 32.
// J (wave-uniform): every subband j >= J has S = +-0 in every slot of both
// channels.  Its terms c * S[j] are +-0, and adding +-0 to a sum that started
// from +0 leaves it unchanged bit for bit (such a sum is never -0, and
// +0 + -0 = +0), so the 33 sums stop after the last block of four subbands
// below J: the zero subbands above the coded bandwidth (count1, the encoder's
// lowpass) cost nothing.  The sums advance together, four subbands at a time.
__device__ __forceinline__ void matrix_exact_v16(float* colu, int J) {
#pragma clang fp contract(off)
  const float z0 = ozero();
  float acc[33];
#pragma unroll
  for (int m = 0; m < 33; m++) acc[m] = z0;
#pragma unroll
  for (int jb = 0; jb < 32; jb += 4) {
    if (jb >= J) break;  // wave-uniform
    float S[4];
#pragma unroll
    for (int i = 0; i < 4; i++) S[i] = colu[kSlots * (jb + i)];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int m = 0; m < 33; m++) acc[m] = acc[m] + kXNrow[m][jb + i] * S[i];
  }
#pragma unroll
  for (int m = 0; m < 33; m++) colu[kSlots * (m < 32 ? dct32::kPosOfM[m] : kColV16)] = acc[m];
}

// V[i] of the slot at x (the reference's value, bit for bit: 0 - x, not -x,
// for the negated rows, since a sum from +0 is never -0).
__device__ __forceinline__ float v_from_x_exact(const float* x, int i) {
  if (i < 16) return x[kSlots * dct32::kPosOfM[16 + i]];
  if (i == 16) return x[kSlots * kColV16];
  if (i < 48) return ozero() - x[kSlots * dct32::kPosOfM[48 - i]];
  return ozero() - x[kSlots * dct32::kPosOfM[i - 48]];
}

// Entry state: overlap store in registers (frequency-inversion signs folded,
// as in v3) and all 16 V blocks of vVec as X vectors + V[16].
__device__ __forceinline__ void init_state_exact(XWaveSmem& s, const mp3g_state* sin, const int init_in[2], int lane,
                                                 f2 stp[9]) {
  const int ch = lane >> 5, k = lane & 31;
  const float sodd = (k & 1) ? -1.0f : 1.0f;
  const bool in0 = init_in[0] && sin, in1 = init_in[1] && sin;
  const bool from_in = ch ? in1 : in0;
#pragma unroll
  for (int q = 0; q < 9; q++) {
    const float a = from_in ? sin->store[ch][k][q] : 0.0f, b = from_in ? sin->store[ch][k][17 - q] : 0.0f;
    stp[q] = (f2){(q & 1) ? a * sodd : a, (q & 1) ? b : b * sodd};
  }
  for (int e = lane; e < 2 * 16 * 33; e += kLanes) {
    const int c = e / (16 * 33), r = e % (16 * 33), blk = r / 33, m = r % 33;
    const bool in = c ? in1 : in0;
    const float* v = in ? &sin->vvec[c][64 * blk] : nullptr;
    const float val = !in ? 0.0f : m < 32 ? x_from_v(v, m) : v[16];
    s.ring[c][m < 32 ? dct32::kPosOfM[m] : kColV16][kHist - 1 - blk] = val;
  }
}

}  // namespace

__device__ __forceinline__ void wexact_chunk(const ChunkDesc& cd, const mp3g_granule* __restrict__ gran,
                                             const int16_t* __restrict__ coef, const mp3g_state* __restrict__ state_in,
                                             mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm,
                                             XWaveSmem& s, const XSharedSmem& sh);

// kZones: the zone launch of a fast-mode plan (kernels_fast.hip launch_fast):
// `chunks` is the zone list the fast kernel filled -- hot zones as chunks of
// their own, to be decoded in the reference's order -- with its length in
// zone_counts[0] (n_chunks = the list's capacity; kernels.h ZoneScratch).
// The waves take zone after zone; the last workgroup to finish
// (zone_counts[1] counts them) empties the list for the next launch, after
// every workgroup has read its length.  An
// empty list ends every workgroup at once and leaves the counters alone, so
// the launch pair needs no host-side state (graph replays included).
template <bool kZones = false>
__global__ void __launch_bounds__(kLanes * kXWaves, 4)
granule_wexact_kernel(const ChunkDesc* __restrict__ chunks, uint32_t n_chunks, const mp3g_granule* __restrict__ gran,
                      const int16_t* __restrict__ coef, const mp3g_state* __restrict__ state_in,
                      mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm,
                      uint32_t* __restrict__ zone_counts = nullptr) {
  __shared__ XSharedSmem sh;
  __shared__ XWaveSmem wsm[kXWaves];
  uint32_t live = n_chunks;
  bool work = true;
  if constexpr (kZones) {
    const uint32_t c = __builtin_amdgcn_readfirstlane(__hip_atomic_load(zone_counts, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_AGENT));
    if (c == 0) return;  // (grid-uniform)
    live = c < n_chunks ? c : n_chunks;
    work = blockIdx.x * kXWaves < live;  // (workgroup-uniform)
  }
  if (work) {
    const int t = threadIdx.x;
    for (int e = t; e < 16; e += kLanes * kXWaves) (&sh.isr[0][0])[e] = e < 14 ? (&g_fast.is_ratio[0][0])[e] : 1.0f;
    for (int e = t; e < kCombos * 32; e += kLanes * kXWaves) (&sh.lband[0][0])[e] = (&g_fast.lband[0][0])[e];
    // the window taps D[32 j + i] of output i with the V -> X signs folded in
    // (exact: a sign flip commutes with rounding), NOT scaled by 32767 as in
    // the fast kernel; output 16's even taps read V[16] itself
    for (int e = t; e < 32 * 16; e += kLanes * kXWaves) {
      const int i = e >> 4, j = e & 15;
      sh.dwin[i][j] = (i == 16 && !(j & 1)) ? g_fast.dwin16[j >> 1] : g_fast.dwin[i][j];
    }
    for (int e = t; e < 4 * 36; e += kLanes * kXWaves) (&sh.win[0][0])[e] = (&g_fast.win[0][0])[e];
  }
  __syncthreads();  // the table fill (the only workgroup barrier of a plan launch)
  XWaveSmem& s = wsm[threadIdx.x >> 6];
  if constexpr (kZones) {
    if (work) {
      for (uint32_t ci = __builtin_amdgcn_readfirstlane(blockIdx.x * kXWaves + (threadIdx.x >> 6)); ci < live;
           ci += gridDim.x * kXWaves) {
        const ChunkDesc cd = chunks[ci];
        wexact_chunk(cd, gran, coef, state_in, state_out, pcm, s, sh);
      }
    }
    __syncthreads();  // the workgroup is done with the list
    if (threadIdx.x == 0) {
      const uint32_t done = __hip_atomic_fetch_add(zone_counts + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (done == gridDim.x - 1) {  // the last workgroup: every one has read the length
        __hip_atomic_store(zone_counts, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(zone_counts + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    const uint32_t ci = __builtin_amdgcn_readfirstlane(blockIdx.x * kXWaves + (threadIdx.x >> 6));
    if (ci >= live) return;
    const ChunkDesc cd = chunks[ci];
    wexact_chunk(cd, gran, coef, state_in, state_out, pcm, s, sh);
  }
}

// One chunk in the reference's order (one wave).
__device__ __forceinline__ void wexact_chunk(const ChunkDesc& cd, const mp3g_granule* __restrict__ gran,
                                             const int16_t* __restrict__ coef, const mp3g_state* __restrict__ state_in,
                                             mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm,
                                             XWaveSmem& s, const XSharedSmem& sh) {
  const int lane = threadIdx.x & (kLanes - 1);
  const int ch = lane >> 5, k = lane & 31;

  uint64_t w64;
  int init_in[2];
  prologue(cd, gran, &w64, init_in, lane);
  const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)w64);
  const uint32_t out_first = __builtin_amdgcn_readfirstlane((uint32_t)cd.out_first);
  const uint32_t end = __builtin_amdgcn_readfirstlane((uint32_t)(cd.out_first + cd.n_out));
  const mp3g_state* sin = state_in ? state_in + cd.stream : nullptr;
  f2 stp[9];
  init_state_exact(s, sin, init_in, lane, stp);

  uint32_t cw[9] = {};
  if (w < end) {
    load_lines_lim(coef, w, lane, cw, (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t)), count1_lim(gran, w, lane));
    if (lane < 10) reinterpret_cast<uint4*>(&s.desc)[lane] = reinterpret_cast<const uint4*>(gran + w)[lane];
    if (lane < 10 && w + 1 < end)
      reinterpret_cast<uint4*>(&s.descn)[lane] = reinterpret_cast<const uint4*>(gran + w + 1)[lane];
  }
  wave_sync();
  const uint32_t span = end - w, span2 = 2 * span, span3 = 3 * span;
  for (uint32_t g = w; g < end; g++) {
    {
      const uint32_t left4 = 4u * (end - g);  // progress-balanced priority (as v3)
      if (left4 > span3) __builtin_amdgcn_s_setprio(3);
      else if (left4 > span2) __builtin_amdgcn_s_setprio(2);
      else if (left4 > span) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    const bool out = g >= out_first;
    bool need_v = true;
    if (!out && g + 1 < out_first) need_v = hdr_nch(gran[g + 1].header) < hdr_nch(s.desc.header);
    const GranParams P = granule_params(s, ch);
    const bool act = ch < P.nch;

    // ---- front end (frame.go:140-452) ----
    float x[18];
    if (P.all_long) front_long_exact(x, cw, s, sh, P, ch, k);
    else front_gather<true>(x, cw, s, P, ch, k);
    stereo_stage(x, s, sh, P, ch);
    antialias_stage<true>(x, P, act, k);
    // ---- IMDCT + overlap + frequency inversion (frame.go:454-486) ----
    float o[18];
    const int bt = imdct_block_type(P.d1, k);
    imdct_exact_s(x, bt, &sh.win[bt][0], k, act, stp, o);

    // prefetch the next granule (lands during the matrixing and window)
    const bool more = g + 1 < end;
    uint4 pd = {0, 0, 0, 0};
    {
      // lines below the next granule's count1s only (its descriptor is in
      // LDS since the previous granule; lines at and above count1 are zero,
      // maindata/huffman.go:127-134, and need not be written by the Huffman
      // kernel), the descriptor two granules ahead with them
      {
        const uint32_t nh = __builtin_amdgcn_readfirstlane(s.descn.header);
        const uint2 n0 = *reinterpret_cast<const uint2*>(&s.descn.ch[0]);
        const uint2 n1 = *reinterpret_cast<const uint2*>(&s.descn.ch[1]);
        const int c0 = (int)(__builtin_amdgcn_readfirstlane(n0.x) & 0xffffu);
        const int c1 = (int)(__builtin_amdgcn_readfirstlane(n1.x) & 0xffffu);
        const int lim = lane_fresh() >> 5 ? (hdr_nch(nh) == 2 ? c1 : 0) : c0;
        load_lines_lim(coef, g + 1, lane, cw, more ? (int)(MP3G_COEF_PER_GRANULE * sizeof(int16_t)) : 0, lim);
      }
      if (lane < 10) {
        const bool more2 = g + 2 < end;
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<mp3g_granule*>(gran + g + 2), (short)0, more2 ? (int)sizeof(mp3g_granule) : 0, 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, lane * 16, 0, 0);
        pd = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
    // ---- matrixing (frame.go:642-648) ----
    if (need_v && act) {
#pragma unroll
      for (int j = 0; j < 18; j++) s.ring[ch][k][kHist + j] = o[j];
    }
    // J = 1 + the highest subband with a non-zero S in either channel
    int J;
    {
      bool nz = false;
#pragma unroll
      for (int j = 0; j < 18; j++) nz |= o[j] != 0.0f;
      const uint64_t b = __builtin_amdgcn_ballot_w64(act && nz);
      const uint32_t m = (uint32_t)b | (uint32_t)(b >> 32);
      J = m ? 32 - __builtin_clz(m) : 0;
    }
    wave_sync();
    if (need_v && act && (lane & 31) < 18) matrix_exact_v16(&s.ring[ch][0][kHist + (lane & 31)], J);
    wave_sync();
    if (more && lane < 10) {
      reinterpret_cast<uint4*>(&s.desc)[lane] = reinterpret_cast<const uint4*>(&s.descn)[lane];
      reinterpret_cast<uint4*>(&s.descn)[lane] = pd;
    }

    // ---- window -> s16 PCM (frame.go:649-678) ----
    uint32_t pk[9] = {};  // (replayed granules: stored to no records)
    if (out) {
      // ring columns of output i = k's operands: V_j[i] (j even; V[16] has a
      // column of its own) and V_j[32 + i] (j odd); lane values recomputed
      // here, not kept across the loop
      const int ko = lane_fresh() & 31, co = lane_fresh() >> 5;
      const int pa = ko == 16 ? kColV16 : dct32::kPosOfM[ko < 16 ? 16 + ko : 48 - ko];
      const int pb = dct32::kPosOfM[ko < 16 ? 16 - ko : ko - 16];
      float dw[16];
      {
        const float4* d4 = reinterpret_cast<const float4*>(&sh.dwin[ko][0]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const float4 v = d4[q];
          dw[4 * q] = v.x;
          dw[4 * q + 1] = v.y;
          dw[4 * q + 2] = v.z;
          dw[4 * q + 3] = v.w;
        }
      }
      // slot ss sums tap j from slot r = 16 + ss - j: walking r downwards
      // feeds every slot's sum its taps in ascending j (the reference's
      // order) while each operand is read from LDS once
      const float* RA = &s.ring[co][pa][0];
      const float* RB = &s.ring[co][pb][0];
      float acc[18];
      const float z0 = ozero();
#pragma unroll
      for (int ss = 0; ss < 18; ss++) acc[ss] = z0;
#pragma unroll
      for (int r = kHist + 17; r >= kHist - 15; r--) {
        const float a = RA[r], b = RB[r];
#pragma unroll
        for (int ss = 0; ss < 18; ss++) {
          const int j = kHist + ss - r;
          if (j < 0 || j > 15) continue;
          acc[ss] = acc[ss] + ((j & 1) ? b : a) * dw[j];
        }
      }
      f2 acc2[9];
#pragma unroll
      for (int p = 0; p < 9; p++) acc2[p] = (f2){acc[2 * p] * 32767.0f, acc[2 * p + 1] * 32767.0f};
      pack_pcm(acc2, P.nch, pk);
    }
    store_pcm(pcm, g, out, pk, lane_fresh() >> 5, lane_fresh() & 31);
    wave_sync();
    // ---- history shift of the channels this granule touched: slots 18..33
    //      -> 0..15 of the 33 columns (lane (c, k): column k; k = 0 also V[16]) ----
    if (act && need_v) {
      f2* col = reinterpret_cast<f2*>(&s.ring[ch][k][0]);
#pragma unroll
      for (int q = 0; q < 8; q++) col[q] = col[9 + q];
      if (k == 0) {
        f2* c16 = reinterpret_cast<f2*>(&s.ring[ch][kColV16][0]);
#pragma unroll
        for (int q = 0; q < 8; q++) c16[q] = c16[9 + q];
      }
    }
    wave_sync();
  }

  // Frame.store / vVec after the chunk's last granule (frame.go:48-49)
  if (cd.flags & kChunkStateOut) {
    mp3g_state* so = state_out + cd.stream;
    const float sg = (k & 1) ? -1.0f : 1.0f;
#pragma unroll
    for (int q = 0; q < 9; q++) {
      so->store[ch][k][q] = (q & 1) ? stp[q].x * sg : stp[q].x;
      so->store[ch][k][17 - q] = (q & 1) ? stp[q].y : stp[q].y * sg;
    }
    for (int e = lane_fresh(); e < 2 * 1024; e += kLanes) {
      const int c = e >> 10, blk = (e >> 6) & 15, i = e & 63;
      so->vvec[c][64 * blk + i] = v_from_x_exact(&s.ring[c][0][kHist - 1 - blk], i);
    }
  }
}

}  // namespace v4
}  // namespace mp3g
