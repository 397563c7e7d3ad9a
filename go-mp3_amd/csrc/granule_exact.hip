// granule_exact.hip -- exact-mode fused granule decode for gfx950 (CDNA4).
//
// Replaces Frame.Decode (reference internal/frame/frame.go:121-138) for a
// batch of granules: requantize (:140-255) -> reorder (:257-302) -> stereo
// (:304-420) -> antialias (:422-452) -> hybrid IMDCT + overlap (:454-478,
// imdct.go:83-108) -> frequency inversion (:480-486) -> polyphase synthesis
// (:630-688) -> s16 PCM.
//
// Bit-exact with the reference (linux/amd64 float semantics): every float32
// product and sum is rounded individually and in the reference's order
// (file compiled with -ffp-contract=off, plus the pragma below); sums keep
// the sequential order; requantization uses float64-derived tables.
//
// Work decomposition: one 256-thread workgroup per CHUNK of consecutive
// granules of one stream.  Cross-granule state (IMDCT overlap `store`,
// polyphase FIFO `vVec`) stays in LDS while the workgroup walks its chunk.
// A chunk that does not start its stream first replays the granules its
// state depends on (normally the two preceding ones; see plan_prologue) with
// PCM output disabled -- the state is a pure function of those granules, so
// the result is bit-identical to a serial decode.
// (compiled as part of kernels.hip)

namespace mp3g {
namespace v1 {
namespace {

constexpr int kThreads = 256;
constexpr int kRing = 36;  // V-block ring per channel: two granules of 18 blocks

struct __align__(16) Smem {
  float xr[2][576];       // spectrum (requantized / reordered / stereo / antialiased)
  float xt[2][576];       // hybrid output: 32 subbands x 18 time samples
  float store[2][576];    // IMDCT overlap, [ch][sb*18+i] == Frame.store[ch][sb][i]
  float ring[2][kRing][64];
  float nwin[64][33];     // synthNWin, padded row (conflict-free column reads)
  float cos36[18][36];
  float synth_d[512];
  float win[4][36];
  float cos12[6][12];
  mp3g_granule desc;
  int flags[256];
};

__device__ __forceinline__ int hdr_mode(uint32_t h) { return (int)((h >> 6) & 3u); }
__device__ __forceinline__ int hdr_nch(uint32_t h) { return hdr_mode(h) == 3 ? 1 : 2; }
__device__ __forceinline__ int hdr_combo(uint32_t h) {
  const int lsf = ((h >> 19) & 3u) == 3u ? 0 : 1;
  int sf = (int)((h >> 10) & 3u);
  sf = sf > 2 ? 2 : sf;  // reserved index never passes header validation
  return lsf * 3 + sf;
}

// Go: int(float32) (CVTTSS2SQ; NaN / overflow -> MinInt64) then clamp to
// [-32767, 32767] (frame.go:663-669).
__device__ __forceinline__ int pcm_sample(float sum) {
  const float t = sum * 32767.0f;
  if (!(t == t) || fabsf(t) >= 9.2233720368547758e18f) return -32767;
  const float c = fminf(fmaxf(t, -32767.0f), 32767.0f);
  return (int)c;  // v_cvt_i32_f32 truncates toward zero
}

// ---- phase A: requantize + reorder (frame.go:140-302) ---------------------
__device__ void phase_requantize(Smem& s, const uint4* coef16, int nch, int combo) {
  const int t = threadIdx.x;
  if (t >= nch * 72) return;
  const int ch = t / 72;
  const int base = 8 * (t % 72);
  const uint4 raw = coef16[t];
  const short* xs = reinterpret_cast<const short*>(&raw);
  const mp3g_channel& C = s.desc.ch[ch];
  const bool shortblk = C.win_switch_flag == 1 && C.block_type == 2;
  const bool mixed = C.mixed_block_flag != 0;
  const int count1 = C.count1;
  const int sfmul = C.scalefac_scale != 0 ? 4 : 2;  // 4 * sfMult
  const int gg = C.global_gain;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int i = base + k;
    const int x = xs[k];
    bool process, is_long;
    int sfb = 0, win = 0, dest = i;
    if (!shortblk) {
      process = i < count1;
      is_long = true;
      sfb = g_tab.line_long_sfb[combo][i];
    } else if (mixed && i < 36) {
      process = true;  // the 36 long lines are always requantized (frame.go:194)
      is_long = true;
      sfb = g_tab.line_long_sfb[combo][i];
    } else {
      const int info = g_tab.line_short[combo][i];
      sfb = info & 15;
      win = (info >> 4) & 3;
      const int bstart = 3 * (int)g_tab.sfb_short[combo][sfb];
      process = bstart < count1;                       // band-granular loop (frame.go:207-222)
      const bool first_band = sfb == (mixed ? 3 : 0);
      if (first_band || bstart < count1) dest = info >> 6;  // reorder (frame.go:277-296)
      is_long = false;
    }
    float v;
    if (process) {
      int n4;
      if (is_long)
        n4 = gg - 210 - sfmul * ((int)C.scalefac_l[sfb] + (int)C.preflag * (int)g_tab.pretab[sfb]);
      else
        n4 = gg - 210 - 8 * (int)C.subblock_gain[win] - sfmul * (int)C.scalefac_s[sfb][win];
      const int a = min(abs(x), 8206);
      v = ldexpf(g_tab.req[n4 & 3][a], n4 >> 2);
      if (x < 0) v = -v;
    } else {
      v = (float)x;
    }
    s.xr[ch][dest] = v;
  }
}

// ---- phase B: MS / intensity stereo (frame.go:304-420) --------------------
__device__ void phase_stereo(Smem& s, uint32_t h, int combo) {
  const bool ms = hdr_mode(h) == 1 && (h & 0x20u);
  const bool is = hdr_mode(h) == 1 && (h & 0x10u);
  if (!ms && !is) return;
  const mp3g_channel& C0 = s.desc.ch[0];
  const int c1r = s.desc.ch[1].count1;
  const int max_pos = max((int)C0.count1, c1r);
  const float inv_sqrt2 = 0.70710678118654752440f;
  const bool short0 = C0.win_switch_flag == 1 && C0.block_type == 2;
  const bool mixed0 = C0.mixed_block_flag != 0;
  for (int i = threadIdx.x; i < 576; i += kThreads) {
    float l = s.xr[0][i], r = s.xr[1][i];
    if (ms && i < max_pos) {
      const float nl = (l + r) * inv_sqrt2;
      const float nr = (l - r) * inv_sqrt2;
      l = nl;
      r = nr;
    }
    if (is) {
      const int sfl = g_tab.line_long_sfb[combo][i];
      const int info = g_tab.line_short[combo][i];
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
    s.xr[0][i] = l;
    s.xr[1][i] = r;
  }
}

// ---- phase C: antialias butterflies (frame.go:427-452) --------------------
__device__ void phase_antialias(Smem& s, int nch) {
  for (int b = threadIdx.x; b < nch * 248; b += kThreads) {
    const int ch = b / 248;
    const int sb = 1 + (b % 248) / 8;
    const int i = b & 7;
    const mp3g_channel& C = s.desc.ch[ch];
    const bool sw = C.win_switch_flag == 1 && C.block_type == 2;
    if (sw && C.mixed_block_flag == 0) continue;
    const int sblim = (sw && C.mixed_block_flag == 1) ? 2 : 32;
    if (sb >= sblim) continue;
    const int li = 18 * sb - 1 - i, ui = 18 * sb + i;
    const float lv = s.xr[ch][li], uv = s.xr[ch][ui];
    const float cs = g_tab.aa_cs[i], ca = g_tab.aa_ca[i];
    const float lb = lv * cs - uv * ca;
    const float ub = uv * cs + lv * ca;
    s.xr[ch][li] = lb;
    s.xr[ch][ui] = ub;
  }
}

// ---- phase D: IMDCT + window + overlap-add + frequency inversion ----------
// (frame.go:454-486, imdct.go:83-108).  Item = (ch, sb, i), computes raw[i]
// and raw[18+i] of subband sb.
__device__ __forceinline__ float imdct_short_at(const Smem& s, const float* in, int q) {
  float acc = 0.0f;  // out[] cleared, then += per window in order 0,1,2
#pragma unroll
  for (int w = 0; w < 3; w++) {
    const int p = q - 6 * w - 6;
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
  for (int it = threadIdx.x; it < nch * 576; it += kThreads) {
    const int ch = it / 576;
    const int sb = (it % 576) / 18;
    const int i = it % 18;
    const mp3g_channel& C = s.desc.ch[ch];
    int bt = C.block_type & 3;
    if (C.win_switch_flag == 1 && C.mixed_block_flag == 1 && sb < 2) bt = 0;
    const float* in = &s.xr[ch][sb * 18];
    float lo, hi;
    if (bt == 2) {
      lo = imdct_short_at(s, in, i);
      hi = imdct_short_at(s, in, 18 + i);
    } else {
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int m = 0; m < 18; m++) {
        const float x = in[m];
        s0 = s0 + x * s.cos36[m][i];
        s1 = s1 + x * s.cos36[m][18 + i];
      }
      lo = s0 * s.win[bt][i];
      hi = s1 * s.win[bt][18 + i];
    }
    float o = lo + s.store[ch][sb * 18 + i];
    s.store[ch][sb * 18 + i] = hi;
    if ((sb & 1) && (i & 1)) o = -o;
    s.xt[ch][sb * 18 + i] = o;
  }
}

// ---- phase E: polyphase matrixing V = N * S (frame.go:636-648) ------------
__device__ void phase_matrix(Smem& s, int nch, const int step[2]) {
  const int row = threadIdx.x & 63;
  for (int p = threadIdx.x >> 6; p < nch * 18; p += kThreads / 64) {
    const int ch = p / 18, ss = p % 18;
    const float* x = &s.xt[ch][ss];
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; j++) sum = sum + s.nwin[row][j] * x[18 * j];
    s.ring[ch][(step[ch] + ss) % kRing][row] = sum;
  }
}

// ---- phase F: window + 16-tap sum + s16 pack (frame.go:649-686) -----------
__device__ void phase_pcm(Smem& s, int nch, const int step[2], uint32_t* pcm32) {
  for (int it = threadIdx.x; it < 576; it += kThreads) {
    const int ss = it >> 5, i = it & 31;
    int smp[2];
    for (int ch = 0; ch < nch; ch++) {
      float sum = 0.0f;
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int slot = (step[ch] + ss - j + kRing) % kRing;
        const float u = s.ring[ch][slot][i + 32 * (j & 1)];
        sum = sum + u * s.synth_d[32 * j + i];
      }
      smp[ch] = pcm_sample(sum);
    }
    if (nch == 1) smp[1] = smp[0];
    pcm32[it] = (uint32_t)(smp[0] & 0xffff) | ((uint32_t)(smp[1] & 0xffff) << 16);
  }
}

__device__ void load_state(Smem& s, const mp3g_state* st, int ch) {
  for (int k = threadIdx.x; k < 576; k += kThreads)
    s.store[ch][k] = st ? (&st->store[ch][0][0])[k] : 0.0f;
  // vVec block k (newest k = 0) -> ring slot for step -1-k
  for (int k = threadIdx.x; k < kRing * 64; k += kThreads) {
    const int slot = k / 64, e = k % 64;
    const int blk = kRing - 1 - slot;  // slot 35 <- block 0
    s.ring[ch][slot][e] = (st && blk < 16) ? st->vvec[ch][64 * blk + e] : 0.0f;
  }
}

__device__ void save_state(const Smem& s, mp3g_state* st, const int step[2]) {
  for (int ch = 0; ch < 2; ch++) {
    for (int k = threadIdx.x; k < 576; k += kThreads) (&st->store[ch][0][0])[k] = s.store[ch][k];
    for (int k = threadIdx.x; k < 1024; k += kThreads) {
      const int blk = k / 64, e = k % 64;
      st->vvec[ch][k] = s.ring[ch][((step[ch] - 1 - blk) % kRing + kRing) % kRing][e];
    }
  }
}

// Decide where the replay (halo) starts and how each channel's state is
// initialised.  Channel 0 is processed in every granule, so its state at c0
// depends on granules c0-2, c0-1 only.  Channel 1 is frozen across mono
// granules (Frame.Decode only touches ch < nch), so its state depends on the
// last two STEREO granules before c0; it matters only if a stereo granule is
// decoded in this chunk or the chunk exports the stream state.
__device__ void plan_prologue(Smem& s, const ChunkDesc& cd, const mp3g_granule* gran,
                              uint64_t* w_out, int init_from_in[2]) {
  const uint64_t c0 = cd.out_first, s0 = cd.stream_first;
  const bool have_in = cd.flags & kChunkStateIn;
  if (c0 == s0) {
    *w_out = c0;
    init_from_in[0] = init_from_in[1] = have_in;
    return;
  }
  const uint64_t start0 = c0 - 2 > s0 && c0 >= 2 ? c0 - 2 : s0;
  // Fast path: both halo granules stereo -> ch1 also needs only them.
  bool st1 = hdr_nch(gran[c0 - 1].header) == 2;
  bool st2 = (c0 - 2 >= s0 && c0 >= 2) ? hdr_nch(gran[c0 - 2].header) == 2 : false;
  if (st1 && st2) {
    *w_out = start0;
    init_from_in[0] = init_from_in[1] = (start0 == s0) && have_in;
    return;
  }
  // need_ch1: any stereo granule decoded in this chunk, or state export.
  int any = 0;
  for (uint32_t k = threadIdx.x; k < cd.n_out; k += kThreads)
    any |= hdr_nch(gran[c0 + k].header) == 2;
  const bool need1 = __syncthreads_or(any) || (cd.flags & kChunkStateOut);
  uint64_t start1 = c0;       // no constraint
  bool ch1_from_in = false;   // ch1 frozen since the stream start
  if (need1) {
    // find the last two stereo granules in [s0, c0), scanning 256 at a time
    int found = 0;
    uint64_t p2 = 0;
    for (uint64_t hi = c0; hi > s0 && found < 2;) {
      const uint64_t lo = hi - s0 > kThreads ? hi - kThreads : s0;
      const uint64_t g = hi - 1 - threadIdx.x;
      __syncthreads();
      s.flags[threadIdx.x] = (g >= lo && g < hi) ? (hdr_nch(gran[g].header) == 2) : 0;
      __syncthreads();
      for (uint64_t k = 0; k < hi - lo && found < 2; k++)
        if (s.flags[k]) {
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

__global__ void __launch_bounds__(kThreads)
granule_exact_kernel(const ChunkDesc* __restrict__ chunks, const mp3g_granule* __restrict__ gran,
                     const int16_t* __restrict__ coef, const mp3g_state* __restrict__ state_in,
                     mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm) {
  __shared__ Smem s;
  const ChunkDesc cd = chunks[blockIdx.x];
  const int t = threadIdx.x;

  // tables -> LDS
  for (int k = t; k < 64 * 32; k += kThreads) s.nwin[k >> 5][k & 31] = g_tab.nwin[k >> 5][k & 31];
  for (int k = t; k < 18 * 36; k += kThreads) (&s.cos36[0][0])[k] = (&g_tab.cos36[0][0])[k];
  for (int k = t; k < 512; k += kThreads) s.synth_d[k] = g_tab.synth_d[k];
  for (int k = t; k < 4 * 36; k += kThreads) (&s.win[0][0])[k] = (&g_tab.imdct_win[0][0])[k];
  for (int k = t; k < 6 * 12; k += kThreads) (&s.cos12[0][0])[k] = (&g_tab.cos12[0][0])[k];

  uint64_t w;
  int init_in[2];
  plan_prologue(s, cd, gran, &w, init_in);
  const mp3g_state* sin = state_in ? state_in + cd.stream : nullptr;
  load_state(s, init_in[0] ? sin : nullptr, 0);
  load_state(s, init_in[1] ? sin : nullptr, 1);
  __syncthreads();

  int step[2] = {0, 0};
  const uint64_t end = cd.out_first + cd.n_out;
  for (uint64_t g = w; g < end; g++) {
    const bool out = g >= cd.out_first;
    // descriptor -> LDS (ten 16-B loads), coefficients -> registers
    if (t < 10) reinterpret_cast<uint4*>(&s.desc)[t] = reinterpret_cast<const uint4*>(gran + g)[t];
    __syncthreads();
    const uint32_t h = s.desc.header;
    const int nch = hdr_nch(h), combo = hdr_combo(h);
    phase_requantize(s, reinterpret_cast<const uint4*>(coef + g * MP3G_COEF_PER_GRANULE), nch, combo);
    __syncthreads();
    if (nch == 2) phase_stereo(s, h, combo);
    __syncthreads();
    phase_antialias(s, nch);
    __syncthreads();
    phase_imdct(s, nch);
    __syncthreads();
    // V blocks of a replayed granule are needed unless the next replayed
    // granule refreshes every FIFO it touches (18 new blocks > 16 kept).
    bool need_v = true;
    if (!out && g + 1 < cd.out_first) need_v = hdr_nch(gran[g + 1].header) < nch;
    if (need_v) phase_matrix(s, nch, step);
    __syncthreads();
    if (out) phase_pcm(s, nch, step, reinterpret_cast<uint32_t*>(pcm + g * 1152));
    step[0] += 18;
    if (nch == 2) step[1] += 18;
    __syncthreads();
  }
  if (cd.flags & kChunkStateOut) save_state(s, state_out + cd.stream, step);
}

}  // namespace v1
}  // namespace mp3g
