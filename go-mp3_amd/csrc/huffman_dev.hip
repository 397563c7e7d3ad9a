// huffman_dev.hip -- main-data decode on the GPU.
//
// One lane per (granule, channel) job of the host scan (host_parse.cpp,
// FrameScanner): the lane reads its channel's scale factors and Huffman codes
// straight out of the concatenated main-data buffer, writes the scale factors
// + count1 into the granule descriptor (whose side-info fields the scan
// filled) and the channel's 576 int16 coefficients (huffman_job.h).
// Decoding inside a channel is bit-serial; the parallelism is across jobs
// (two per granule, 64 per wave).  A block's 256 consecutive jobs read one
// contiguous span of the main data: the block ranks them by big_values and
// stages the span in LDS with coalesced 8-byte loads (byte-swapped once), so
// the bit-serial loop never waits on
// global memory (on gfx9 a load's vmcnt wait would also wait for the
// coefficient stores issued before it).  The Huffman tables (huff_lut.h,
// 9 KB) live in LDS too.
// (compiled as part of kernels.hip)
#include "huffman_job.h"

namespace mp3g {
namespace huff {

#ifndef MP3G_HUFF_THREADS
#define MP3G_HUFF_THREADS 256
#endif
constexpr int kThreads = MP3G_HUFF_THREADS;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
  for (int o = 32; o; o >>= 1) {
    const uint64_t u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max(uint64_t v) {
  for (int o = 32; o; o >>= 1) {
    const uint64_t u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

// Block-sorted kernel: the 256 jobs of a block are ranked by big_values
// (counting sort in LDS, bins of 4 pairs) before they are dealt to lanes, so
// each wave's 64 lanes run big-values loops of similar length (the loop of a
// wave lasts as long as its longest job).  The block's main-data span is
// staged once for all four waves (a lane's job can sit anywhere in it).
// 28 KB of staging + 9 KB of tables and <= 128 VGPRs keep 4 blocks (16 waves)
// per CU: c3 3.09 -> 2.78 ms, c2 142 -> 129 us against one lane per job in
// stream order.  The gain is modest because a lane is bound by its own
// dependent chain (window -> LUT lookup in LDS -> shift), not by idle lanes;
// 512-thread blocks (better sort, shared tables) were 3 % faster at c3 and
// 6 % slower at c2.
#ifndef MP3G_HUFF_BLOCK_STAGE_WORDS
#define MP3G_HUFF_BLOCK_STAGE_WORDS kHuffStageWords  // 28 KB: 256 jobs span ~25 KB at 128 kbps
#endif
constexpr int kBlockStage = MP3G_HUFF_BLOCK_STAGE_WORDS;
// the larger instantiations for higher bitrates (tools/huff_time.py, c3's
// shape): MP3G_HUFF_STAGE_MID, 42 KB of stage, 3 blocks per CU -- at 192 kbps
// (no block fits 28 KB) 2.97 ms against 4.58 ms reading global memory at 16
// waves per CU and 3.84 ms with the wide stage; MP3G_HUFF_STAGE_WIDE, 68 KB, 2
// blocks per CU -- at 320 kbps 4.41 ms against 5.19 ms reading global memory.
// At 128 kbps the default is 2.18-2.32 ms, the mid one 2.54, the wide 3.46.
constexpr int kBlockStageMid = kHuffStageWordsMid;
constexpr int kBlockStageWide = kHuffStageWordsWide;
constexpr int kBins = 128;  // bin 0: jobs that read nothing; 1 + big_values / 4 <= 73

#ifndef MP3G_HUFF_MAXVGPR
#define MP3G_HUFF_MAXVGPR 128  // unbounded, the compiler takes 129 (3 waves per SIMD)
#endif
#define MP3G_HUFF_SORTED_ATTR __attribute__((amdgpu_num_vgpr(MP3G_HUFF_MAXVGPR)))
template <int kStage>
__global__ void __launch_bounds__(kThreads) MP3G_HUFF_SORTED_ATTR
huffman_sorted_kernel(const mp3g_hjob* __restrict__ jobs, uint64_t n_jobs, const uint8_t* __restrict__ md,
                      mp3g_granule* __restrict__ gran, int16_t* __restrict__ coef, uint32_t full_rows) {
  static_assert(kThreads <= 1024 && kThreads % 64 == 0, "block shape");
  __shared__ uint32_t T2[kHuffMaxEntries / 2];
  __shared__ uint32_t s_root[34], s_lin[34];
  __shared__ uint64_t stage[kStage + 4];  // + 4: the LDS reader's look-ahead
  __shared__ uint32_t s_bin[kBins];
  __shared__ uint16_t s_order[kThreads];
  __shared__ uint64_t s_lo[kWaves], s_hi[kWaves];
  const uint32_t t = threadIdx.x;
  const int lane = (int)(t & 63u), wv = (int)(t >> 6);
  const uint32_t n_w = (g_huff.n_entries + 1) / 2;
  const uint32_t* src_e = reinterpret_cast<const uint32_t*>(g_huff.e);
  for (uint32_t i = t; i < n_w; i += kThreads) T2[i] = src_e[i];
  const uint16_t* T = reinterpret_cast<const uint16_t*>(T2);
  if (t < 34) {
    s_root[t] = g_huff.root[t];
    s_lin[t] = g_huff.linbits[t];
  }
  for (uint32_t i = t; i < (uint32_t)kBins; i += kThreads) s_bin[i] = 0u;
  const uint64_t j0 = (uint64_t)blockIdx.x * kThreads;
  uint32_t bin = 0u;
  {
    const uint64_t jt = j0 + t;
    mp3g_hjob J{};
    if (jt < n_jobs) J = jobs[jt];
    const bool reads = jt < n_jobs && J.sf_kind != MP3G_SF_NONE;
    const uint64_t base = job_base(J);
    const uint64_t lo = wave_min(reads ? base : ~0ull);
    const uint64_t hi = wave_max(reads ? J.bit_end : 0ull);
    if (lane == 0) {
      s_lo[wv] = lo;
      s_hi[wv] = hi;
    }
    if (reads) bin = 1u + (J.big_values < 288u ? J.big_values : 288u) / 4u;
  }
  __syncthreads();
  const uint32_t rank = atomicAdd(&s_bin[bin], 1u);
  uint64_t lo = ~0ull, hi = 0ull;
#pragma unroll
  for (int w = 0; w < kWaves; w++) {
    lo = s_lo[w] < lo ? s_lo[w] : lo;
    hi = s_hi[w] > hi ? s_hi[w] : hi;
  }
  __syncthreads();
  if (t < 64) {  // exclusive scan of the bins, two per lane
    const uint32_t a = s_bin[2 * t], b = s_bin[2 * t + 1];
    uint32_t inc = a + b;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      inc += lane >= o ? u : 0u;
    }
    const uint32_t ex = inc - (a + b);
    s_bin[2 * t] = ex;
    s_bin[2 * t + 1] = ex + a;
  }
  const uint64_t nwords = hi > lo && lo != ~0ull ? ((hi - lo + 63) >> 6) : 0ull;
  const bool staged = nwords <= (uint64_t)kStage;  // block-uniform
  if (staged) {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(md + (lo >> 3));
    for (uint32_t k = t; k < (uint32_t)nwords; k += kThreads) stage[k] = bswap64(src[k]);
  }
  __syncthreads();
  s_order[s_bin[bin] + rank] = (uint16_t)t;
  __syncthreads();
  const uint64_t j = j0 + s_order[t];
  int z = MP3G_LINES;  // first line this lane's row still needs zeroed
  if (j < n_jobs) {
    const mp3g_hjob J = jobs[j];
    if (staged) {
      // a corrupt stream's part 2 can start past the span (part2_3_length
      // sums overrunning the main data): clamp, so the reader's nw never wraps
      const uint64_t off64 = J.sf_kind != MP3G_SF_NONE ? (job_base(J) - lo) >> 6 : 0ull;
      const uint32_t off = (uint32_t)(off64 < nwords ? off64 : nwords);
      z = decode_job<false>(J, j, &stage[off], (uint32_t)nwords - off, gran, coef, T, s_root, s_lin);
    } else {
      z = decode_job_direct(J, j, md, gran, coef, T, s_root, s_lin);
    }
  }
  if (!full_rows) {
    // rows to count1 only (MP3G_HUFF_ROWS_COUNT1): the default plan kernels
    // read lines below count1 in 6-line pieces, i.e. up to count1 + 5 <= z + 5
    // (z >= count1 is the end of the lane's last 16-line block): one 16-B slot
    // of zeros past it covers that.  c3: 2.79 -> 2.42 ms (tools/gpu_r03z.sh)
    if (z < MP3G_LINES) *reinterpret_cast<uint4*>(coef + j * MP3G_LINES + z) = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  // zero tails of the wave's 64 rows, one row at a time with the whole wave
  for (int rr = 0; rr < 64; rr++) {
    const int zr = __shfl(z, rr, 64);
    if (zr >= MP3G_LINES) continue;  // wave-uniform
    const uint64_t jr = ((uint64_t)__shfl((uint32_t)(j >> 32), rr, 64) << 32) | __shfl((uint32_t)j, rr, 64);
    uint4* row = reinterpret_cast<uint4*>(coef + jr * MP3G_LINES);
    for (int s8 = (zr >> 3) + lane; s8 < MP3G_LINES / 8; s8 += 64) row[s8] = make_uint4(0u, 0u, 0u, 0u);
  }
}

}  // namespace huff

hipError_t launch_huffman(const mp3g_hjob* d_jobs, uint64_t n_jobs, const uint8_t* d_md, mp3g_granule* d_gran,
                          int16_t* d_coef, bool full_rows, int stage, hipStream_t stream) {
  if (n_jobs == 0) return hipSuccess;
  const uint64_t blocks = (n_jobs + huff::kThreads - 1) / huff::kThreads;
  if (stage == 2)
    hipLaunchKernelGGL(huff::huffman_sorted_kernel<huff::kBlockStageWide>, dim3((uint32_t)blocks),
                       dim3(huff::kThreads), 0, stream, d_jobs, n_jobs, d_md, d_gran, d_coef, full_rows ? 1u : 0u);
  else if (stage == 1)
    hipLaunchKernelGGL(huff::huffman_sorted_kernel<huff::kBlockStageMid>, dim3((uint32_t)blocks),
                       dim3(huff::kThreads), 0, stream, d_jobs, n_jobs, d_md, d_gran, d_coef, full_rows ? 1u : 0u);
  else
    hipLaunchKernelGGL(huff::huffman_sorted_kernel<huff::kBlockStage>, dim3((uint32_t)blocks),
                       dim3(huff::kThreads), 0, stream, d_jobs, n_jobs, d_md, d_gran, d_coef, full_rows ? 1u : 0u);
  return hipGetLastError();
}

}  // namespace mp3g
