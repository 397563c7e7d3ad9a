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
// Work decomposition: the fused kernel's plans, one wave per chunk, eight
// chunks per workgroup.  The window of slot ss reads the 15 preceding V
// blocks, so a chunk replays only the granule before it (matrixing, no
// window) when that granule has both channels; otherwise it takes the fused
// kernel's replay start (a superset).  Per granule:
//   load      the granule's nch x 576 floats as 8-B pairs, lane + 64 r
//             (coalesced, one granule ahead in registers); the resource is
//             sized to nch x 2,304 B, so a mono granule reads nothing of [1];
//   stage     pair -> its ring slot: line 18 sb + ss of channel c is slot
//             16 + ss of column sb, i.e. S[sb] of time slot ss;
//   matrixing lane (ch, slot < 18): S column -> 32 X values in place;
//   window    lane (ch, i): 16 taps, 18 outputs, s16 (L, R) pairs stored;
//   shift     slots 18..33 -> 0..15.
// Hot granules (a line above kHotS) and the granule after each are redone in
// the reference's order after the chunk's fast pass (as in the fused kernel).
// (compiled in kernels_fast.hip after granule_fast.hip: shares its helpers)

namespace mp3g {
namespace v3 {

constexpr int kSynthWaves = 8;


// Ping-pong ring: 36 slots per column (stride 38), two halves of 18.  A granule's 18
// slots go to one half while the other half holds the previous granule's,
// whose last 15 are the history its window reads; the next granule writes the
// half just read from.  No history shift (the fused kernel's 34-slot ring
// moves 16 slots per column and granule; leaving that shift out of this
// kernel measured -6 %, tools/gpu_synthlds.sh).  A window operand is named by
// its virtual slot z = 16 + (V block - first block of the current granule),
// z = 1..33, as in the fused kernel; physically
//   even granules (P = 0): current in 18..35, history in 2..17: z + 2
//   odd granules  (P = 1): current in 0..17, history in 20..35:
//                          z - 16 (z >= 16) or z + 20
// The hot-zone fixup (reference order, rare) keeps the even layout and moves
// slots 20..35 to 2..17 after each granule.
// column stride 38 (36 slots used): 38 = 6 mod 32 and 38 = 2 * 19 mod 64 map
// the columns onto the banks exactly as the fused kernel's 34 does (column
// mod 16 for dword reads, mod 32 for 8-B reads); a stride of 36 (4 mod 32)
// folds them onto 8 bank groups (3.1 conflict cycles per LDS op at c3)
constexpr int kSS = 38;
__device__ __forceinline__ constexpr int sphys(int P, int z) { return P ? (z >= 16 ? z - 16 : z + 20) : z + 2; }

struct __align__(16) SynthWaveSmem {
  float ring[2][32][kSS];
  uint32_t zone[kZones][2];  // hot zones of the chunk (record_hot)
};

namespace {

// The granule's lines [nch][576] (1,152 floats): lane's quads lane + 64 r
// (r < 4, floats 0..1023) as 16-B loads and the pair 512 + lane (floats
// 1024..1151) as an 8-B load, held as nine pairs: buf[2 r], buf[2 r + 1] the
// halves of quad r, buf[8] the tail pair.  (Nine 8-B loads before.)
// Issued unconditionally (straight-line vmcnt accounting): past the chunk
// (or with nbytes 0) the resource has no records, so the loads return 0 and
// touch no memory.
// first line in [2][576] of pair i (0..8) of this lane
__device__ __forceinline__ int synth_pair_line(int lane, int i) {
  return i < 8 ? 4 * (lane + 64 * (i >> 1)) + 2 * (i & 1) : 1024 + 2 * lane;
}
__device__ __forceinline__ void synth_load(const float* lines, uint32_t g, uint32_t nbytes, int lane, f2 v[9]) {
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(lines + (size_t)g * MP3G_COEF_PER_GRANULE), (short)0, (int)nbytes,
      0x00020000);
  // non-temporal (cache policy nt): the lines are read once; c3 3.21 -> 3.13 ms
  // (the fused kernel's coefficient loads measured +0.9 % with it,
  // tools/gpu_r03nt.sh)
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b128(rc, 16 * lane + 1024 * r, 0, 2);
    v[2 * r] = (f2){__uint_as_float(u[0]), __uint_as_float(u[1])};
    v[2 * r + 1] = (f2){__uint_as_float(u[2]), __uint_as_float(u[3])};
  }
  const auto u = __builtin_amdgcn_raw_buffer_load_b64(rc, 4096 + 8 * lane, 0, 2);
  v[8] = (f2){__uint_as_float(u[0]), __uint_as_float(u[1])};
}

// stage: line 18 sb + ss of channel c -> ring[c][sb][cur + ss] (cur: the
// first slot of the current half), as 8-B pairs (ds_write_b64)
template <int cur>
__device__ __forceinline__ void synth_stage(SynthWaveSmem& s, const f2 buf[9], int nch) {
#pragma unroll
  for (int r = 0; r < 9; r++) {
    const int e = synth_pair_line(lane_fresh(), r);  // first line of the pair in [2][576]
    const int c = e >= 576;
    const int l = e - 576 * c;
    const int sb = (l * 3641) >> 16;  // l / 18 for l < 576
    f2* colp = reinterpret_cast<f2*>(&s.ring[c][0][0]);
    if (c < nch) colp[(kSS / 2) * sb + cur / 2 + ((l - 18 * sb) >> 1)] = buf[r];
  }
}

__device__ __forceinline__ float max_abs_pairs(const f2 v[9]) {
  float m = 0.0f;
#pragma unroll
  for (int r = 0; r < 9; r++) m = fmaxf(m, fmaxf(fabsf(v[r].x), fabsf(v[r].y)));
  return m;
}

// Replay start of a synthesis chunk beginning at c0: the granule before it
// when that granule carries both channels' history, else the fused kernel's
// decision (a superset).
__device__ __forceinline__ uint32_t synth_replay_start(const ChunkDesc& cd, uint64_t c0, const mp3g_granule* gran,
                                                       int init_in[2], int lane) {
  const uint64_t s0 = cd.stream_first;
  const bool have_in = cd.flags & kChunkStateIn;
  uint64_t w64;
  if (c0 > s0 && hdr_nch(gran[c0 - 1].header) == 2) {
    w64 = c0 - 1;
    init_in[0] = init_in[1] = (w64 == s0) && have_in;
  } else {
    ChunkDesc cr = cd;
    cr.n_out = (uint32_t)(cd.out_first + cd.n_out - c0);
    cr.out_first = c0;
    prologue(cr, gran, &w64, init_in, lane);
  }
  return __builtin_amdgcn_readfirstlane((uint32_t)w64);
}

// V history of a replay start (the even layout: block b at virtual slot
// 15 - b): X vectors from the stream's state_in or zero.
__device__ __forceinline__ void synth_init_ring(SynthWaveSmem& s, const mp3g_state* sin, const int init_in[2],
                                                int lane) {
  const bool in0 = init_in[0] && sin, in1 = init_in[1] && sin;
  for (int e = lane; e < 2 * 15 * 32; e += kLanes) {
    const int c = e / (15 * 32), blk = (e >> 5) % 15, m = e & 31;
    const bool in = c ? in1 : in0;
    s.ring[c][dct32::kPosOfM[m]][sphys(0, 15 - blk)] = in ? x_from_v(&sin->vvec[c][64 * blk], m) : 0.0f;
  }
}

// One granule in the reference's operation order (hot-zone fixup); returns
// whether it is hot.
__device__ __forceinline__ bool synth_exact_granule(const mp3g_granule* __restrict__ gran,
                                                    const float* __restrict__ lines, int16_t* __restrict__ pcm,
                                                    SynthWaveSmem& s, uint32_t g, bool out) {
  const int lane = lane_fresh();
  const int ch = lane >> 5, k = lane & 31, hi = lane >> 5;
  const int nch = hdr_nch(__builtin_amdgcn_readfirstlane(gran[g].header));
  f2 buf[9];
  synth_load(lines, g, nch * 2304u, lane, buf);
  const bool hot1 = __builtin_amdgcn_ballot_w64(max_abs_pairs(buf) > kHotS) != 0;
  synth_stage<18>(s, buf, nch);
  wave_sync();
  const bool hot = hot1 && slot_sums_hot<kSS>(s.ring, nch, 18);
  if (ch < nch && (lane & 31) < 18) matrix_exact<kSS>(&s.ring[ch][0][18 + (lane & 31)]);
  wave_sync();
  uint32_t pk[9] = {};
  if (out) {
    const int pa = dct32::kPosOfM[k < 16 ? 16 + k : (k == 16 ? 0 : 48 - k)];
    const int pb = dct32::kPosOfM[k < 16 ? 16 - k : k - 16];
    f2 acc2[9];
    window_exact<18>(&s.ring[ch][pa][0], &s.ring[ch][pb][0], k, acc2);
    pack_pcm(acc2, nch, pk);
  }
  store_pcm(pcm, g, out, pk, hi, k);
  wave_sync();
  if (ch < nch) {  // slots 20..35 -> 2..17 (the even layout's history)
    f2* col = reinterpret_cast<f2*>(&s.ring[ch][k][0]);
#pragma unroll
    for (int q = 0; q < 8; q++) col[1 + q] = col[10 + q];
  }
  wave_sync();
  return hot;
}

}  // namespace

__global__ void __launch_bounds__(kLanes * kSynthWaves, 4)
granule_synth_kernel(const ChunkDesc* __restrict__ chunks, uint32_t n_chunks, const mp3g_granule* __restrict__ gran,
                     const float* __restrict__ lines, const mp3g_state* __restrict__ state_in,
                     mp3g_state* __restrict__ state_out, int16_t* __restrict__ pcm) {
  // FastTables::dwin, pre-scaled by 32767; rows padded to 20 floats, so the
  // 16 lanes of a ds_read_b128 quad group hit 64 distinct banks
  __shared__ __align__(16) float dwin_s[32][20];
  __shared__ SynthWaveSmem wsm[kSynthWaves];
  for (int e = threadIdx.x; e < 32 * 16; e += kLanes * kSynthWaves)
    dwin_s[e >> 4][e & 15] = (&g_fast.dwin[0][0])[e] * 32767.0f;
  __syncthreads();  // the only workgroup barrier
  const int lane = threadIdx.x & (kLanes - 1);
  const uint32_t ci = __builtin_amdgcn_readfirstlane(blockIdx.x * kSynthWaves + (threadIdx.x >> 6));
  if (ci >= n_chunks) return;
  SynthWaveSmem& s = wsm[threadIdx.x >> 6];
  const ChunkDesc cd = chunks[ci];
  const int ch = lane >> 5, k = lane & 31;
  const int pa = dct32::kPosOfM[k < 16 ? 16 + k : (k == 16 ? 0 : 48 - k)];
  const int pb = dct32::kPosOfM[k < 16 ? 16 - k : k - 16];

  int init_in[2];
  const uint32_t w = synth_replay_start(cd, cd.out_first, gran, init_in, lane);
  const uint32_t out_first = __builtin_amdgcn_readfirstlane((uint32_t)cd.out_first);
  const uint32_t end = __builtin_amdgcn_readfirstlane((uint32_t)(cd.out_first + cd.n_out));
  const mp3g_state* sin = state_in ? state_in + cd.stream : nullptr;
  synth_init_ring(s, sin, init_in, lane);

  // channel counts of the chunk's granules as a stereo bit mask in SGPRs, 64
  // granules per refill (one vector load and a ballot): the per-granule
  // header reads were scalar loads whose wait held up the next granule's
  // line loads
  uint64_t smask = 0;
  uint32_t mbase = 0xffffffffu;  // (no granule yet: the first call fills the mask)
  auto nch_of = [&](uint32_t g) -> int {
    if (g < mbase || g - mbase >= 64u) {
      const uint32_t gi = g + (uint32_t)lane_fresh();
      smask = __builtin_amdgcn_ballot_w64(gi < end && hdr_nch(gran[gi].header) == 2);
      mbase = g;
    }
    return ((smask >> (g - mbase)) & 1u) ? 2 : 1;
  };
  auto load = [&](uint32_t g, f2 v[9]) {
    const bool in = g < end;
    const uint32_t gg = in ? g : w;
    const uint32_t nch = in ? (uint32_t)nch_of(gg) : 0u;
    synth_load(lines, gg, nch * 2304u, lane, v);
  };
  const int hi = lane >> 5;
  // the lane's 16 window taps, in registers for the whole chunk
  float dw[16];
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

  uint32_t nz = 0;  // hot zones recorded (s.zone)
  uint32_t pk[9] = {};  // PCM of a granule (stale for replayed ones: stored to no records)
  const uint32_t span = end - w, span2 = 2 * span, span3 = 3 * span;
  // one granule: stage buf (granule g), refill buf with granule gn, then the
  // matrixing, window, PCM stores and history shift of g.  (A second buffer
  // -- two granules in flight, the taps read from LDS per granule to stay at
  // 116 VGPRs -- measured +1.5 % at c3: the loads are not latency-bound,
  // DESIGN.md "Standalone polyphase kernel")
  // one granule with the ring in layout P (std::integral_constant): stage buf
  // (granule g), refill buf with granule gn, then the matrixing, window and
  // PCM stores of g.  No history shift: the next granule uses the other
  // layout, whose history half this granule's current half is.
  auto step = [&](auto Pc, uint32_t g, f2 (&buf)[9], uint32_t gn) {
    constexpr int P = decltype(Pc)::value;
    constexpr int cur = P ? 0 : 18;  // first slot of the current half
    // progress-balanced issue priority, as in the fused kernel (c2 -3.5 %)
    const uint32_t left4 = 4u * (end - g);
    if (left4 > span3) __builtin_amdgcn_s_setprio(3);
    else if (left4 > span2) __builtin_amdgcn_s_setprio(2);
    else if (left4 > span) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    const int nch = nch_of(g);
    const bool out = g >= out_first;
    // a hot granule: its zone is redone in the reference's order after the pass
#if MP3G_HOT_CHECK
    const bool hot1 = __builtin_amdgcn_ballot_w64(max_abs_pairs(buf) > kHotS) != 0;
#endif
    synth_stage<cur>(s, buf, nch);
    // a later granule in flight during the matrixing and window
    load(gn, buf);
    // a mono granule leaves channel 1 alone (Decode touches ch < nch): its
    // history moves to the other layout's history half (lane (1, k): column k)
    if (nch == 1 && ch == 1) {
      f2* col = reinterpret_cast<f2*>(&s.ring[1][k][0]);
#pragma unroll
      for (int q = 0; q < 8; q++) col[P ? 1 + q : 10 + q] = col[P ? 10 + q : 1 + q];
    }
    wave_sync();
#if MP3G_HOT_CHECK
    // a hot granule (two tests, the second rare and on the staged S): its
    // zone is redone in the reference's order after the pass
    if (hot1 && slot_sums_hot<kSS>(s.ring, nch, cur)) record_hot(s, nz, gran, g, out_first, end);
#endif
    // ---- matrixing (frame.go:642-648): lane (ch, slot) turns its S row into X ----
    {
      const int slot = lane & 31;
      if (ch < nch && slot < 18) {
        float* colu = &s.ring[ch][0][cur + slot];
        dct32::f2 sp[16];
#pragma unroll
        for (int q = 0; q < 16; q++) sp[q] = (dct32::f2){colu[kSS * 2 * q], colu[kSS * (2 * q + 1)]};
        dct32::dct2_32_to(sp, [&](int t, dct32::f2 v) {
          colu[kSS * dct32::kColX[t]] = v.x;
          colu[kSS * dct32::kColY[t]] = v.y;
        });
      }
    }
    wave_sync();
    // ---- 16-tap window -> s16 PCM (frame.go:649-678); the stores are issued
    //      for replayed granules too, through a resource with no records.
    //      Operands by virtual slot z (see SynthWaveSmem): A = the pair
    //      (z, z + 1), z = 16 + v even (8-B aligned in both layouts), B = z - 1
    //      and z (two dwords; in layout 1 the pair (15, 16) wraps) ----
    if (out) {
      const f2* RA = reinterpret_cast<const f2*>(&s.ring[ch][pa][0]);
      const float* RB = &s.ring[ch][pb][0];
      f2 acc2[9];
#pragma unroll
      for (int p = 0; p < 9; p++) acc2[p] = bcast(0.0f);
#pragma unroll
      for (int v = -14; v <= 16; v += 2) {
        const f2 Av = RA[sphys(P, 16 + v) / 2];
        const f2 Bv = {RB[sphys(P, 15 + v)], RB[sphys(P, 16 + v)]};
#pragma unroll
        for (int t = 0; t < 8; t++) {
          const int p = v / 2 + t;
          if (p >= 0 && p < 9) {
            acc2[p] = pfma(bcast(dw[2 * t]), Av, acc2[p]);
            acc2[p] = pfma(bcast(dw[2 * t + 1]), Bv, acc2[p]);
          }
        }
      }
      pack_pcm(acc2, nch, pk);
    }
    store_pcm(pcm, g, out, pk, hi, k);
    wave_sync();  // window reads done before the next granule stages over them
  };
  // Loads are issued right after a granule is staged and waited for when it
  // is staged; the preheader pads each buffer's loads with nine stores to no
  // records, so that the loop is entered with the vector memory counter in the
  // shape of its back edge (loads, then the PCM stores): without them the
  // waits at the loop top are placed for the entry path and also wait for the
  // previous granule's stores, every granule.
  f2 A[9];
  load(w, A);
  store_pcm(pcm, w, false, pk, hi, k);
  wave_sync();
  // granules in pairs: layout 0, then layout 1 (scalar control)
  for (uint32_t g = w; g < end; g += 2) {
    step(std::integral_constant<int, 0>{}, g, A, g + 1);
    if (g + 1 < end) step(std::integral_constant<int, 1>{}, g + 1, A, g + 2);
  }

  // vVec out; the IMDCT overlap `store` is not this stage's: passed through
  // (Pn: the layout the next granule would use, whose history half holds the
  // last 15 V blocks)
  auto export_state = [&](int Pn) {
    if (!(cd.flags & kChunkStateOut)) return;
    mp3g_state* so = state_out + cd.stream;
    const bool have_in = (cd.flags & kChunkStateIn) && sin;
    for (int e = lane_fresh(); e < 2 * 32 * 18; e += kLanes)
      (&so->store[0][0][0])[e] = have_in ? (&sin->store[0][0][0])[e] : 0.0f;
    for (int e = lane_fresh(); e < 2 * 1024; e += kLanes) {
      const int c = e >> 10, blk = (e >> 6) & 15, i = e & 63;
      so->vvec[c][64 * blk + i] =
          blk < 15 ? v_from_x<kSS>(&s.ring[c][0][Pn ? sphys(1, 15 - blk) : sphys(0, 15 - blk)], i) : 0.0f;
    }
  };
  export_state((int)((end - w) & 1u));

  // ---- hot zones (rare): redone in the reference's order from their replay
  //      start, PCM overwritten; a zone reaching the chunk end rewrites the
  //      exported state (see the fused kernel) ----
  if (nz) {
    uint32_t done = 0;
    bool have = false;
    for (uint32_t i = 0; i < nz; i++) {
      const uint32_t zs = __builtin_amdgcn_readfirstlane(s.zone[i][0]);
      uint32_t ze = __builtin_amdgcn_readfirstlane(s.zone[i][1]);
      if (have && ze <= done) continue;
      uint32_t g = done;
      if (!have || zs > done) {
        int zin[2];
        g = synth_replay_start(cd, zs, gran, zin, lane_fresh());
        synth_init_ring(s, sin, zin, lane_fresh());
        wave_sync();
        have = true;
      }
      for (; g < ze; g++)
        if (synth_exact_granule(gran, lines, pcm, s, g, g >= zs)) {
          const uint32_t e = zone_end(gran, g, end);
          ze = e > ze ? e : ze;
        }
      done = g;
    }
    if (done >= end) export_state(0);
  }
}

}  // namespace v3
}  // namespace mp3g
