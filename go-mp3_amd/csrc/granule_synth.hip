// granule_synth.hip -- the standalone polyphase synthesis kernel (gfx950):
// go-mp3's subbandSynthesis (internal/frame/frame.go:630-688) over a batch of
// granules whose frequency-inverted hybrid output (the float32 lines
// `MainData.Is[gr][ch]` that subbandSynthesis reads, frame.go:133) is already
// in HBM.  Entry point mp3g_plan_synth_execute (include/mp3g.h).
//
// It is the fast kernel's polyphase stage on its own (same in-lane DCT-II-32
// matrixing, same X ring and 16-tap window, +-1 LSB of the reference), with
// the float32 lines streamed from HBM instead of produced by the front end:
// per granule-channel 2,304 B in and 1,152 B of s16 PCM out, the 3,456 B the
// north star's "polyphase kernel at >= 40 % of the HBM roof" is priced on
// (SURVEY.md 8(d)).
//
// Work decomposition: the fused kernel's plans, one wave per chunk.  The
// window of slot ss reads the 15 preceding V blocks, so a chunk replays only
// the granule before it (matrixing, no window) when that granule has both
// channels; otherwise it takes the fused kernel's replay start (a superset).
// Per granule:
//   load      the granule's nch x 576 floats as 8-B pairs, lane + 64 r
//             (coalesced, one granule ahead in registers); the resource is
//             sized to nch x 2,304 B, so a mono granule reads nothing of [1];
//   stage     pair -> its ring slot: line 18 sb + ss of channel c is slot
//             16 + ss of column sb, i.e. S[sb] of time slot ss;
//   matrixing lane (ch, slot < 18): S column -> 32 X values in place;
//   window    lane (ch, i): 16 taps, 18 outputs, s16 (L, R) pairs stored;
//   shift     slots 18..33 -> 0..15.
// (compiled in kernels_fast.hip after granule_fast.hip: shares its helpers)

namespace mp3g {
namespace v3 {

#ifndef MP3G_SYNTH_WG_WAVES
#define MP3G_SYNTH_WG_WAVES 8
#endif
constexpr int kSynthWaves = MP3G_SYNTH_WG_WAVES;
// granules of lines in flight per wave (register buffers of 18 VGPRs)
#ifndef MP3G_SYNTH_DEPTH
#define MP3G_SYNTH_DEPTH 1  // 2 measured the same at c3 and 2 % slower at c2
#endif
#ifndef MP3G_SYNTH_DW_REGS
#define MP3G_SYNTH_DW_REGS 1
#endif
#ifndef MP3G_SYNTH_PRIO
#define MP3G_SYNTH_PRIO 1  // c2 -3.5 %, c3 +-0 (tools/gpu_synthab.sh)
#endif
// cache-policy bits of the line loads / PCM stores (experiments)
#ifndef MP3G_SYNTH_LOAD_AUX
#define MP3G_SYNTH_LOAD_AUX 0
#endif
#ifndef MP3G_SYNTH_STORE_AUX
#define MP3G_SYNTH_STORE_AUX 2  // non-temporal PCM stores: c3 -1.3 %, c2 -2 % (the lines: nt loads +5 %)
#endif

struct __align__(16) SynthWaveSmem {
  float ring[2][32][kSlots];
};

#ifndef MP3G_SYNTH_WAVES_PER_SIMD
#define MP3G_SYNTH_WAVES_PER_SIMD 4
#endif
__global__ void __launch_bounds__(kLanes * kSynthWaves, MP3G_SYNTH_WAVES_PER_SIMD)
granule_synth_kernel(const ChunkDesc* __restrict__ chunks, uint32_t n_chunks, const mp3g_granule* __restrict__ gran,
                     const float* __restrict__ lines, const mp3g_state* __restrict__ state_in,
                     mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm) {
  __shared__ __align__(16) float dwin_s[32][16];  // FastTables::dwin, pre-scaled by 32767
  __shared__ SynthWaveSmem wsm[kSynthWaves];
  for (int e = threadIdx.x; e < 32 * 16; e += kLanes * kSynthWaves)
    (&dwin_s[0][0])[e] = (&g_fast.dwin[0][0])[e] * 32767.0f;
  __syncthreads();  // the only workgroup barrier
  const int lane = threadIdx.x & (kLanes - 1);
  const uint32_t ci = __builtin_amdgcn_readfirstlane(blockIdx.x * kSynthWaves + (threadIdx.x >> 6));
  if (ci >= n_chunks) return;
  SynthWaveSmem& s = wsm[threadIdx.x >> 6];
  const ChunkDesc cd = chunks[ci];
  const int ch = lane >> 5, k = lane & 31;
  const int pa = dct32::kPosOfM[k < 16 ? 16 + k : (k == 16 ? 0 : 48 - k)];
  const int pb = dct32::kPosOfM[k < 16 ? 16 - k : k - 16];

  // replay start: the granule before the chunk when it carries both
  // channels' history, else the fused kernel's decision (a superset)
  uint64_t w64;
  int init_in[2];
  {
    const uint64_t c0 = cd.out_first, s0 = cd.stream_first;
    const bool have_in = cd.flags & kChunkStateIn;
    if (c0 > s0 && hdr_nch(gran[c0 - 1].header) == 2) {
      w64 = c0 - 1;
      init_in[0] = init_in[1] = (w64 == s0) && have_in;
    } else {
      prologue(cd, gran, &w64, init_in, lane);
    }
  }
  const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)w64);
  const uint32_t out_first = __builtin_amdgcn_readfirstlane((uint32_t)cd.out_first);
  const uint32_t end = __builtin_amdgcn_readfirstlane((uint32_t)(cd.out_first + cd.n_out));
  const mp3g_state* sin = state_in ? state_in + cd.stream : nullptr;
  {
    const bool in0 = init_in[0] && sin, in1 = init_in[1] && sin;
    for (int e = lane; e < 2 * 15 * 32; e += kLanes) {
      const int c = e / (15 * 32), blk = (e >> 5) % 15, m = e & 31;
      const bool in = c ? in1 : in0;
      s.ring[c][dct32::kPosOfM[m]][kHist - 1 - blk] = in ? x_from_v(&sin->vvec[c][64 * blk], m) : 0.0f;
    }
  }

  // the granule's lines as 8-B pairs: pair p = lane + 64 r of [nch][576].
  // Issued unconditionally (straight-line vmcnt accounting): past the chunk
  // the resource has no records, so the loads return 0 and touch no memory.
  auto load = [&](uint32_t g, f2 v[9]) {
    const bool in = g < end;
    const uint32_t gg = in ? g : w;
    const uint32_t nch = in ? hdr_nch(__builtin_amdgcn_readfirstlane(gran[gg].header)) : 0u;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(lines + (size_t)gg * MP3G_COEF_PER_GRANULE), (short)0, (int)(nch * 2304u), 0x00020000);
#pragma unroll
    for (int r = 0; r < 9; r++) {
      const auto u = __builtin_amdgcn_raw_buffer_load_b64(rc, 8 * lane + 512 * r, 0, MP3G_SYNTH_LOAD_AUX);
      v[r] = (f2){__uint_as_float(u[0]), __uint_as_float(u[1])};
    }
  };
  const int hi = lane >> 5;
  // the lane's 16 window taps, in registers for the whole chunk (read per
  // granule they were four 4-way bank-conflicted ds_read_b128)
  float dw[16];
#if MP3G_SYNTH_DW_REGS
  {
    const float4* d4 = reinterpret_cast<const float4*>(&dwin_s[k][0]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const float4 v = d4[q];
      dw[4 * q] = v.x;
      dw[4 * q + 1] = v.y;
      dw[4 * q + 2] = v.z;
      dw[4 * q + 3] = v.w;
    }
  }
#endif

  // one granule; its lines in `buf`, which is refilled with granule g + depth
  auto granule = [&](uint32_t g, f2 buf[9]) {
    const uint32_t h = __builtin_amdgcn_readfirstlane(gran[g].header);
    const int nch = hdr_nch(h);
    const bool out = g >= out_first;
    // ---- stage: line 18 sb + ss of channel c -> ring[c][sb][16 + ss] ----
#pragma unroll
    for (int r = 0; r < 9; r++) {
      const int e = 2 * lane_fresh() + 128 * r;  // first line of the pair in [2][576]
      const int c = e >= 576;
      const int l = e - 576 * c;
      const int sb = (l * 3641) >> 16;  // l / 18 for l < 576
      // indexed as 8-B pairs (ds_write_b64, 4 x 16 lanes): as separate dwords
      // the 32 lanes of a write group land on 16 even banks
      f2* colp = reinterpret_cast<f2*>(&s.ring[c][0][0]);
      if (c < nch) colp[17 * sb + kHist / 2 + ((l - 18 * sb) >> 1)] = buf[r];
    }
    // a later granule in flight during the matrixing and window
    load(g + MP3G_SYNTH_DEPTH, buf);
    wave_sync();
    // ---- matrixing (frame.go:642-648): lane (ch, slot) turns its S row into X ----
    {
      const int slot = lane & 31;
      if (ch < nch && slot < 18) {
        float* colu = &s.ring[ch][0][kHist + slot];
        dct32::f2 sp[16];
#pragma unroll
        for (int q = 0; q < 16; q++) sp[q] = (dct32::f2){colu[kSlots * 2 * q], colu[kSlots * (2 * q + 1)]};
        dct32::dct2_32_to(sp, [&](int t, dct32::f2 v) {
          colu[kSlots * dct32::kColX[t]] = v.x;
          colu[kSlots * dct32::kColY[t]] = v.y;
        });
      }
    }
    wave_sync();
    // ---- 16-tap window -> s16 PCM (frame.go:649-678); the stores are issued
    //      for replayed granules too, through a resource with no records ----
    uint32_t pk[9] = {};  // (dropped for replayed granules)
    if (out) {
#if !MP3G_SYNTH_DW_REGS
      {
        const float4* d4 = reinterpret_cast<const float4*>(&dwin_s[k][0]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const float4 v = d4[q];
          dw[4 * q] = v.x;
          dw[4 * q + 1] = v.y;
          dw[4 * q + 2] = v.z;
          dw[4 * q + 3] = v.w;
        }
      }
#endif
      const f2* RA = reinterpret_cast<const f2*>(&s.ring[ch][pa][0]);
      const float* RB = &s.ring[ch][pb][0];
      f2 acc2[9];
#pragma unroll
      for (int p = 0; p < 9; p++) acc2[p] = bcast(0.0f);
#pragma unroll
      for (int v = -14; v <= 16; v += 2) {
        const f2 A = RA[(kHist + v) / 2];
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
      auto pack = [&](auto mono) {
#pragma unroll
        for (int p = 0; p < 9; p++) {
          const int a = (int)__builtin_amdgcn_fmed3f(acc2[p].x, -32767.0f, 32767.0f);
          const int b = (int)__builtin_amdgcn_fmed3f(acc2[p].y, -32767.0f, 32767.0f);
          const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
          pk[p] = __builtin_amdgcn_perm((uint32_t)(decltype(mono)::value ? r[0] : r[1]), (uint32_t)r[0], 0x05040100u);
        }
      };
      if (nch == 2) pack(std::false_type{});
      else pack(std::true_type{});
    }
    {
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          pcm + (size_t)g * 1152, (short)0, out ? MP3G_PCM_BYTES_PER_GRANULE : 0, 0x00020000);
#pragma unroll
      for (int p = 0; p < 9; p++)
        __builtin_amdgcn_raw_buffer_store_b32(pk[p], rp, 4 * (32 * (2 * p + hi) + k), 0, MP3G_SYNTH_STORE_AUX);
    }
    wave_sync();
    // ---- history shift of the channels this granule touched ----
    if (ch < nch) {
      f2* col = reinterpret_cast<f2*>(&s.ring[ch][k][0]);
#pragma unroll
      for (int q = 0; q < 8; q++) col[q] = col[9 + q];
    }
    wave_sync();
  };

#if MP3G_SYNTH_DEPTH == 1
  f2 A[9];
  load(w, A);
  wave_sync();
#if MP3G_SYNTH_PRIO
  const uint32_t span = end - w, span2 = 2 * span, span3 = 3 * span;
#endif
  for (uint32_t g = w; g < end; g++) {
#if MP3G_SYNTH_PRIO
    // progress-balanced issue priority, as in the fused kernel
    const uint32_t left4 = 4u * (end - g);
    if (left4 > span3) __builtin_amdgcn_s_setprio(3);
    else if (left4 > span2) __builtin_amdgcn_s_setprio(2);
    else if (left4 > span) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#endif
    granule(g, A);
  }
#else
  // two granules in flight: ping-pong buffers, the loop unrolled by two
  f2 A[9], B[9];
  load(w, A);
  load(w + 1, B);
  wave_sync();
  for (uint32_t g = w; g < end; g += 2) {
    granule(g, A);
    if (g + 1 < end) granule(g + 1, B);
  }
#endif

  if (cd.flags & kChunkStateOut) {
    // vVec out; the IMDCT overlap `store` is not this stage's: passed through
    mp3g_state* so = state_out + cd.stream;
    const bool have_in = (cd.flags & kChunkStateIn) && sin;
    for (int e = lane; e < 2 * 32 * 18; e += kLanes)
      (&so->store[0][0][0])[e] = have_in ? (&sin->store[0][0][0])[e] : 0.0f;
    for (int e = lane; e < 2 * 1024; e += kLanes) {
      const int c = e >> 10, blk = (e >> 6) & 15, i = e & 63;
      so->vvec[c][64 * blk + i] = blk < 15 ? v_from_x(&s.ring[c][0][kHist - 1 - blk], i) : 0.0f;
    }
  }
}

}  // namespace v3
}  // namespace mp3g
