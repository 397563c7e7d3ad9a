// granule_fused.hip -- exact-mode fused granule decode, v2 (gfx950).
//
// Same contract and halo decomposition as granule_exact.hip (bit-exact
// Frame.Decode, reference internal/frame/frame.go:121-688), restructured for
// CDNA4 issue efficiency:
//
//  * 4 barriers per granule; the next granule's descriptor + coefficients are
//    prefetched into registers during the current one (global latency hidden
//    behind the IMDCT and matrixing phases) and the PCM of a granule leaves
//    through an LDS staging area as 16-B coalesced stores.
//  * front end in GATHER form: each thread owns output lines (an antialias
//    butterfly pair or one of the 80 untouched lines) for both channels and
//    computes requantize (source line through the inverse reorder table) ->
//    MS/IS -> butterfly in registers; no scatter, no extra barrier.
//  * IMDCT-36 uses the bitwise symmetries of cosN36 (col 17-p = -col p,
//    col 53-p = col p; tests/test_tables.py): 18 sequential-order sums per
//    subband instead of 36, every product/sum still rounded as the reference.
//  * matrixing V = N*S as a register-blocked GEMM in sequential k order:
//    each lane keeps its synthNWin row(s) in VGPRs, S vectors are read as
//    16-B LDS broadcasts, 5 independent accumulation chains per lane; only the
//    34 distinct rows are computed (rows 16+k = -rows 16-k, rows 48+k =
//    rows 48-k, k = 1..15, exact by RNE sign symmetry).
//  * window/sum: synthesis-window taps of the lane's output index live in
//    VGPRs for the whole kernel.
// (compiled as part of kernels.hip)
namespace mp3g {
namespace v2 {
namespace {

constexpr int kThreads = 256;
// V-block window per channel: slots 0..15 hold the previous 16 blocks (slot 15
// newest, = Frame.vVec blocks 0..15 reversed), slots 16..33 the current
// granule's 18 blocks; after a granule slots 18..33 move to 0..15.  Static
// slots give immediate-offset LDS addressing in the window sum.
constexpr int kRing = 34;
constexpr int kNStride = 36;
constexpr int kSStride = 36;  // 16 different time slots read by one b128 group -> distinct bank quads

struct PcmRaw {
  int16_t pcm[576 * 2];   // staged s16 stereo output of the last decoded granule
  int16_t raw[2][576];    // staged coefficients of the next granule
};

struct __align__(16) Smem {
  union {
    float xr[2][576];     // front-end output (requantized, stereo, antialiased)
    int flags[256];       // prologue scratch
  } a;
  union {
    float xt[2][18][kSStride];  // hybrid output, transposed: [ch][time slot][subband] (padded rows)
    PcmRaw io;            // (dead while xt is live)
  } b;
  float store[2][576];    // IMDCT overlap == Frame.store[ch][sb][i]
  float ring[2][kRing][64];
  float nrow[34][kNStride];  // row stride 36: the 16 rows a ds_read_b128 group reads hit 16 distinct bank quads
  float c36[18][18];
  float win[4][36];
  float cos12[6][12];
  float dwin[512];
  mp3g_granule desc;
};

using common::hdr_combo;
using common::hdr_mode;
using common::hdr_nch;
using common::pcm_sample;

__device__ __forceinline__ float requant_line(const Smem& s, const mp3g_channel& C, int ch, int L,
                                              int combo) {
  return common::requant_line(s.b.io.raw[ch], C, L, combo);
}
__device__ __forceinline__ void stereo_line(const Smem& s, uint32_t h, int combo, int L, float& l,
                                            float& r) {
  common::stereo_line(s.desc, h, combo, L, l, r);
}

// Phase 1: front end.  Items 0..247: butterfly pairs (sb = 1..31, i = 0..7);
// items 248..327: the 80 lines no butterfly touches.
__device__ void phase_front(Smem& s, uint32_t h, int nch, int combo) {
  for (int it = threadIdx.x; it < 328; it += kThreads) {
    if (it < 248) {
      const int sb = 1 + (it >> 3), i = it & 7;
      const int li = 18 * sb - 1 - i, ui = 18 * sb + i;
      float a0 = requant_line(s, s.desc.ch[0], 0, li, combo);
      float b0 = requant_line(s, s.desc.ch[0], 0, ui, combo);
      float a1 = 0.0f, b1 = 0.0f;
      if (nch == 2) {
        a1 = requant_line(s, s.desc.ch[1], 1, li, combo);
        b1 = requant_line(s, s.desc.ch[1], 1, ui, combo);
        stereo_line(s, h, combo, li, a0, a1);
        stereo_line(s, h, combo, ui, b0, b1);
      }
      const float cs = g_tab.aa_cs[i], ca = g_tab.aa_ca[i];
#pragma unroll
      for (int ch = 0; ch < 2; ch++) {
        if (ch >= nch) break;
        float& lv = ch ? a1 : a0;
        float& uv = ch ? b1 : b0;
        const mp3g_channel& C = s.desc.ch[ch];
        const bool sw = C.win_switch_flag == 1 && C.block_type == 2;
        const bool skip = sw && C.mixed_block_flag == 0;
        const int sblim = (sw && C.mixed_block_flag == 1) ? 2 : 32;
        if (!skip && sb < sblim) {  // antialias (frame.go:427-452)
          const float lb = lv * cs - uv * ca;
          const float ub = uv * cs + lv * ca;
          lv = lb;
          uv = ub;
        }
        s.a.xr[ch][li] = lv;
        s.a.xr[ch][ui] = uv;
      }
    } else {
      const int L = g_tab.aa_singles[it - 248];
      float v0 = requant_line(s, s.desc.ch[0], 0, L, combo);
      if (nch == 2) {
        float v1 = requant_line(s, s.desc.ch[1], 1, L, combo);
        stereo_line(s, h, combo, L, v0, v1);
        s.a.xr[1][L] = v1;
      }
      s.a.xr[0][L] = v0;
    }
  }
}

// ---- Phase 2: IMDCT + overlap + frequency inversion ------------------------
// Item (ch, sb, q), q = 0..8, produces raw[q], raw[17-q], raw[18+q], raw[35-q].
__device__ __forceinline__ float short_raw(const Smem& s, const float* in, int Q) {
  float acc = 0.0f;
#pragma unroll
  for (int w = 0; w < 3; w++) {
    const int p = Q - 6 * w - 6;
    if (p >= 0 && p < 12) {
      float sum = 0.0f;
#pragma unroll
      for (int m = 0; m < 6; m++) sum = sum + in[w + 3 * m] * s.cos12[m][p];
      acc = acc + sum * s.win[2][p];
    }
  }
  return acc;
}

__device__ void phase_imdct(Smem& s, int nch) {
  for (int it = threadIdx.x; it < nch * 288; it += kThreads) {
    const int ch = it / 288;
    const int sb = (it % 288) / 9;
    const int q = it % 9;
    const mp3g_channel& C = s.desc.ch[ch];
    int bt = C.block_type & 3;
    if (C.win_switch_flag == 1 && C.mixed_block_flag == 1 && sb < 2) bt = 0;
    const float* in = &s.a.xr[ch][sb * 18];
    float r0, r1, r2, r3;  // raw[q], raw[17-q], raw[18+q], raw[35-q]
    if (bt == 2) {
      r0 = short_raw(s, in, q);
      r1 = short_raw(s, in, 17 - q);
      r2 = short_raw(s, in, 18 + q);
      r3 = short_raw(s, in, 35 - q);
    } else {
      float sa = 0.0f, sbb = 0.0f;
#pragma unroll
      for (int m = 0; m < 18; m++) {
        const float x = in[m];
        sa = sa + x * s.c36[m][q];
        sbb = sbb + x * s.c36[m][9 + q];
      }
      r0 = sa * s.win[bt][q];
      r1 = (0.0f - sa) * s.win[bt][17 - q];  // sum[17-q] == 0 - sum[q] bitwise
      r2 = sbb * s.win[bt][18 + q];
      r3 = sbb * s.win[bt][35 - q];
    }
    float* st = &s.store[ch][sb * 18];
    float o0 = r0 + st[q];
    float o1 = r1 + st[17 - q];
    st[q] = r2;
    st[17 - q] = r3;
    if (sb & 1) {  // frequency inversion: odd time slots of odd subbands
      if (q & 1) o0 = -o0;
      else o1 = -o1;  // 17 - q is odd when q is even
    }
    s.b.xt[ch][q][sb] = o0;
    s.b.xt[ch][17 - q][sb] = o1;
  }
}

// ---- Phase 3: matrixing V = N * S ------------------------------------------
struct VLane {
  int ch, rbase, row, row5, ss5;  // main row / fifth-chain row and slot
  bool store5;
};

__device__ __forceinline__ void ring_store(Smem& s, int ch, int slot, int row, float v) {
  slot += 16;
  s.ring[ch][slot][row] = v;
  // the reference's sequential sums never yield -0: mirror as 0 - v, not -v
  if (row >= 1 && row <= 15) s.ring[ch][slot][32 - row] = 0.0f - v;
  else if (row >= 33 && row <= 47) s.ring[ch][slot][96 - row] = v;
}

__device__ void phase_matrix(Smem& s, const VLane& L, int nch) {
  if (L.ch >= nch) return;
  const int q4 = (threadIdx.x & 63) >> 4;
  const float* S = &s.b.xt[L.ch][0][0];
  const float* Nm = &s.nrow[L.row < 17 ? L.row : L.row - 15][0];
  const float* N5 = &s.nrow[L.row5 < 17 ? L.row5 : L.row5 - 15][0];
  float acc[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  // k-blocks of 4 in a runtime loop: bounded live ranges, every operand an LDS
  // 16-B read (S rows broadcast across the 16 lanes sharing a time slot)
#pragma unroll 1
  for (int j = 0; j < 32; j += 4) {
    const float4 nv = *reinterpret_cast<const float4*>(Nm + j);
    const float4 n5 = *reinterpret_cast<const float4*>(N5 + j);
    float4 sv[5];
#pragma unroll
    for (int k = 0; k < 4; k++) sv[k] = *reinterpret_cast<const float4*>(S + (q4 + 4 * k) * kSStride + j);
    sv[4] = *reinterpret_cast<const float4*>(S + L.ss5 * kSStride + j);
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = acc[k] + nv.x * sv[k].x;
    acc[4] = acc[4] + n5.x * sv[4].x;
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = acc[k] + nv.y * sv[k].y;
    acc[4] = acc[4] + n5.y * sv[4].y;
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = acc[k] + nv.z * sv[k].z;
    acc[4] = acc[4] + n5.z * sv[4].z;
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = acc[k] + nv.w * sv[k].w;
    acc[4] = acc[4] + n5.w * sv[4].w;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) ring_store(s, L.ch, q4 + 4 * k, L.row, acc[k]);
  if (L.store5) ring_store(s, L.ch, L.ss5, L.row5, acc[4]);
}

// After a granule: its 16 newest V blocks (slots 18..33) become the history
// (slots 0..15) of every channel it processed; a channel skipped by a mono
// granule keeps its frozen history (Decode only touches ch < nch).
__device__ void shift_history(Smem& s, int nch_prev) {
  for (int k = threadIdx.x; k < nch_prev * 16 * 16; k += kThreads) {  // float4 units
    const int ch = k >> 8, e = k & 255;
    float4* dst = reinterpret_cast<float4*>(&s.ring[ch][0][0]);
    const float4* src = reinterpret_cast<const float4*>(&s.ring[ch][18][0]);
    dst[e] = src[e];
  }
}

// ---- Phase 4: 16-tap window sum -> s16 into the LDS staging area -------------
__device__ void phase_pcm(Smem& s, int nch) {
  const int i = threadIdx.x & 31;
  const int p0 = threadIdx.x >> 5;  // items p = p0 + 8k, p < nch*18, (ch, ss) = (p / 18, p % 18)
  const int np = nch * 18;
  float acc[5];
  int base[5];  // float index of (slot 16 + ss, lane i) in ring; block j is at slot 16 + ss - j
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const int p = min(p0 + 8 * k, np - 1);
    base[k] = ((p / 18) * kRing + 16 + p % 18) * 64 + i;
    acc[k] = 0.0f;
  }
  const float* R = &s.ring[0][0][0];
#pragma unroll 1
  for (int j = 0; j < 16; j += 2) {
    const float d0 = s.dwin[32 * j + i], d1 = s.dwin[32 * j + 32 + i];
    float u0[5], u1[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
      u0[k] = R[base[k] - 64 * j];            // j even: first half of the block
      u1[k] = R[base[k] - 64 * j - 64 + 32];  // j+1 odd: second half
    }
#pragma unroll
    for (int k = 0; k < 5; k++) acc[k] = acc[k] + u0[k] * d0;
#pragma unroll
    for (int k = 0; k < 5; k++) acc[k] = acc[k] + u1[k] * d1;
  }
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const int p = p0 + 8 * k;
    if (p < np) {
      const int ch = p / 18, ss = p % 18;
      const int smp = pcm_sample(acc[k]);
      const int o = (32 * ss + i) * 2;
      if (nch == 1) {
        s.b.io.pcm[o] = (int16_t)smp;
        s.b.io.pcm[o + 1] = (int16_t)smp;
      } else {
        s.b.io.pcm[o + ch] = (int16_t)smp;
      }
    }
  }
}

__device__ void load_state(Smem& s, const mp3g_state* st, int ch) {
  for (int k = threadIdx.x; k < 576; k += kThreads) s.store[ch][k] = st ? (&st->store[ch][0][0])[k] : 0.0f;
  for (int k = threadIdx.x; k < kRing * 64; k += kThreads) {
    const int slot = k / 64, e = k % 64;
    const int blk = 15 - slot;  // slot 15 <- newest block vVec[0:64]
    s.ring[ch][slot][e] = (st && blk >= 0) ? st->vvec[ch][64 * blk + e] : 0.0f;
  }
}

// Called after shift_history of the last granule: history slots hold the state.
__device__ void save_state(const Smem& s, mp3g_state* st) {
  for (int ch = 0; ch < 2; ch++) {
    for (int k = threadIdx.x; k < 576; k += kThreads) (&st->store[ch][0][0])[k] = s.store[ch][k];
    for (int k = threadIdx.x; k < 1024; k += kThreads) st->vvec[ch][k] = s.ring[ch][15 - k / 64][k % 64];
  }
}

// Replay start (see granule_exact.hip: plan_prologue) -- identical logic.
__device__ void plan_prologue(Smem& s, const ChunkDesc& cd, const mp3g_granule* gran, uint64_t* w_out,
                              int init_from_in[2]) {
  const uint64_t c0 = cd.out_first, s0 = cd.stream_first;
  const bool have_in = cd.flags & kChunkStateIn;
  if (c0 == s0) {
    *w_out = c0;
    init_from_in[0] = init_from_in[1] = have_in;
    return;
  }
  const uint64_t start0 = (c0 >= 2 && c0 - 2 > s0) ? c0 - 2 : s0;
  const bool st1 = hdr_nch(gran[c0 - 1].header) == 2;
  const bool st2 = (c0 >= 2 && c0 - 2 >= s0) ? hdr_nch(gran[c0 - 2].header) == 2 : false;
  if (st1 && st2) {
    *w_out = start0;
    init_from_in[0] = init_from_in[1] = (start0 == s0) && have_in;
    return;
  }
  int any = 0;
  for (uint32_t k = threadIdx.x; k < cd.n_out; k += kThreads) any |= hdr_nch(gran[c0 + k].header) == 2;
  const bool need1 = __syncthreads_or(any) || (cd.flags & kChunkStateOut);
  uint64_t start1 = c0;
  bool ch1_from_in = false;
  if (need1) {
    int found = 0;
    uint64_t p2 = 0;
    for (uint64_t hi = c0; hi > s0 && found < 2;) {
      const uint64_t lo = hi - s0 > kThreads ? hi - kThreads : s0;
      const uint64_t g = hi - 1 - threadIdx.x;
      __syncthreads();
      s.a.flags[threadIdx.x] = (g >= lo && g < hi) ? (hdr_nch(gran[g].header) == 2) : 0;
      __syncthreads();
      for (uint64_t k = 0; k < hi - lo && found < 2; k++)
        if (s.a.flags[k]) {
          found++;
          if (found == 2) p2 = hi - 1 - k;
        }
      hi = lo;
    }
    if (found == 2) start1 = p2;
    else if (found == 1) start1 = s0;
    else ch1_from_in = true;
  }
  const uint64_t w = start0 < start1 ? start0 : start1;
  *w_out = w;
  init_from_in[0] = (w == s0) && have_in;
  init_from_in[1] = ch1_from_in ? have_in : ((w == s0) && have_in);
}

}  // namespace

__global__ void __launch_bounds__(kThreads, 4)
granule_fused_kernel(const ChunkDesc* __restrict__ chunks, const mp3g_granule* __restrict__ gran,
                     const int16_t* __restrict__ coef, const mp3g_state* __restrict__ state_in,
                     mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm) {
  __shared__ Smem s;
  const ChunkDesc cd = chunks[blockIdx.x];
  const int t = threadIdx.x;

  for (int k = t; k < 34 * 32; k += kThreads) s.nrow[k >> 5][k & 31] = (&g_tab.nwin_distinct[0][0])[k];
  for (int k = t; k < 18 * 18; k += kThreads) (&s.c36[0][0])[k] = (&g_tab.cos36_distinct[0][0])[k];
  for (int k = t; k < 4 * 36; k += kThreads) (&s.win[0][0])[k] = (&g_tab.imdct_win[0][0])[k];
  for (int k = t; k < 6 * 12; k += kThreads) (&s.cos12[0][0])[k] = (&g_tab.cos12[0][0])[k];
  for (int k = t; k < 512; k += kThreads) s.dwin[k] = g_tab.synth_d[k];

  uint64_t w;
  int init_in[2];
  plan_prologue(s, cd, gran, &w, init_in);
  const mp3g_state* sin = state_in ? state_in + cd.stream : nullptr;
  load_state(s, init_in[0] ? sin : nullptr, 0);
  load_state(s, init_in[1] ? sin : nullptr, 1);
  const uint64_t end = cd.out_first + cd.n_out;
  if (w < end) {  // first granule straight into the staging area
    if (t < 144) reinterpret_cast<uint4*>(&s.b.io.raw[0][0])[t] =
        reinterpret_cast<const uint4*>(coef + w * MP3G_COEF_PER_GRANULE)[t];
    if (t < 10) reinterpret_cast<uint4*>(&s.desc)[t] = reinterpret_cast<const uint4*>(gran + w)[t];
  }
  __syncthreads();

  // per-lane constants of the matrixing and window phases (registers for the whole kernel)
  VLane vl;
  {
    const int wv = t >> 6, l = t & 63, q4 = l >> 4;
    vl.ch = wv >> 1;
    vl.rbase = (wv & 1) ? 32 : 0;
    vl.row = vl.rbase + (l & 15);
    if (q4 < 2) {
      vl.row5 = vl.row;
      vl.ss5 = 16 + q4;
      vl.store5 = true;
    } else {
      const int idx = l - 32;
      vl.row5 = vl.rbase + 16;
      vl.ss5 = idx < 18 ? idx : 0;
      vl.store5 = idx < 18;
    }
  }
  int nch_prev = 0;            // channels processed by the previous granule (history shift)
  int16_t* pending = nullptr;  // PCM of the previous granule waiting in LDS staging
  for (uint64_t g = w; g < end; g++) {
    const bool out = g >= cd.out_first;
    const uint32_t h = s.desc.header;
    const int nch = hdr_nch(h), combo = hdr_combo(h);
    shift_history(s, nch_prev);
    // flush the previous granule's PCM (16-B stores) and prefetch the next granule
    if (pending && t < 144)
      reinterpret_cast<uint4*>(pending)[t] = reinterpret_cast<const uint4*>(s.b.io.pcm)[t];
    uint4 nraw = {0, 0, 0, 0}, ndesc = {0, 0, 0, 0};
    const bool more = g + 1 < end;
    if (more) {
      if (t < 144) nraw = reinterpret_cast<const uint4*>(coef + (g + 1) * MP3G_COEF_PER_GRANULE)[t];
      if (t < 10) ndesc = reinterpret_cast<const uint4*>(gran + g + 1)[t];
    }
    phase_front(s, h, nch, combo);
    __syncthreads();
    phase_imdct(s, nch);
    __syncthreads();
    bool need_v = true;
    if (!out && g + 1 < cd.out_first) need_v = hdr_nch(gran[g + 1].header) < nch;
    if (need_v) phase_matrix(s, vl, nch);
    __syncthreads();
    if (out) phase_pcm(s, nch);
    pending = out ? pcm + g * 1152 : nullptr;
    if (more) {
      if (t < 144) reinterpret_cast<uint4*>(&s.b.io.raw[0][0])[t] = nraw;
      if (t < 10) reinterpret_cast<uint4*>(&s.desc)[t] = ndesc;
    }
    nch_prev = nch;
    __syncthreads();
  }
  if (pending && t < 144)
    reinterpret_cast<uint4*>(pending)[t] = reinterpret_cast<const uint4*>(s.b.io.pcm)[t];
  if (cd.flags & kChunkStateOut) {
    shift_history(s, nch_prev);
    __syncthreads();
    save_state(s, state_out + cd.stream);
  }
}

}  // namespace v2
}  // namespace mp3g
