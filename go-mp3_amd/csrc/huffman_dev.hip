// huffman_dev.hip -- main-data decode on the GPU.
//
// One lane per (granule, channel) job of the host scan (host_parse.cpp,
// FrameScanner): the lane reads its channel's scale factors and Huffman codes
// straight out of the concatenated main-data buffer, writes the scale factors
// + count1 into the granule descriptor (whose side-info fields the scan
// filled) and the channel's 576 int16 coefficients (huffman_job.h).
// Decoding inside a channel is bit-serial; the parallelism is across jobs
// (two per granule, 64 per wave).  A wave's 64 consecutive jobs read one
// contiguous span of the main data: the wave stages it in LDS with coalesced
// 8-byte loads (byte-swapped once), so the bit-serial loop never waits on
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
// Main data staged per wave: 64 consecutive jobs (16 MPEG-1 stereo frames)
// span ~6.1 KB at 128 kbps.  7.5 KB per wave + the 9 KB of tables keep the
// block under 40 KB of LDS (4 blocks = 16 waves per CU); a wave whose span
// does not fit reads straight from global memory.
#ifndef MP3G_HUFF_STAGE_WORDS
#define MP3G_HUFF_STAGE_WORDS 960
#endif
constexpr int kStageWords = MP3G_HUFF_STAGE_WORDS;  // 0: no staging (experiments)

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

__global__ void __launch_bounds__(kThreads)
huffman_kernel(const mp3g_hjob* __restrict__ jobs, uint64_t n_jobs, const uint8_t* __restrict__ md,
               mp3g_granule* __restrict__ gran, int16_t* __restrict__ coef) {
  __shared__ uint32_t T2[kHuffMaxEntries / 2];  // the 16-bit entries, two per word
  __shared__ uint32_t s_root[34], s_lin[34];
  // + 4 words: the LDS reader loads up to 3 words past a job's last word
  __shared__ uint64_t stage[kWaves][kStageWords ? kStageWords + 4 : 1];
  const uint32_t n_w = (g_huff.n_entries + 1) / 2;
  const uint32_t* src_e = reinterpret_cast<const uint32_t*>(g_huff.e);
  for (uint32_t i = threadIdx.x; i < n_w; i += kThreads) T2[i] = src_e[i];
  const uint16_t* T = reinterpret_cast<const uint16_t*>(T2);
  if (threadIdx.x < 34) {
    s_root[threadIdx.x] = g_huff.root[threadIdx.x];
    s_lin[threadIdx.x] = g_huff.linbits[threadIdx.x];
  }
  const uint64_t j = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool valid = j < n_jobs;
  mp3g_hjob J{};
  if (valid) J = jobs[j];
  // the wave's main-data span [lo, hi) in bits, lo 64-bit aligned
  const bool reads = valid && J.sf_kind != MP3G_SF_NONE;
  const uint64_t base = job_base(J);
  const uint64_t lo = wave_min(reads ? base : ~0ull);
  const uint64_t hi = wave_max(reads ? J.bit_end : 0ull);
  const uint64_t nwords = hi > lo && lo != ~0ull ? ((hi - lo + 63) >> 6) : 0ull;
  const bool staged = kStageWords && nwords <= (uint64_t)kStageWords;  // wave-uniform
  const int wv = threadIdx.x >> 6;
  if (staged) {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(md + (lo >> 3));
    for (uint32_t k = threadIdx.x & 63; k < (uint32_t)nwords; k += 64) stage[wv][k] = bswap64(src[k]);
  }
  __syncthreads();
  int z = MP3G_LINES;  // first line this lane's row still needs zeroed
  if (valid) {
    if (staged) {
      // a corrupt stream's part 2 can start past the wave's span (part2_3_length
      // sums overrunning the main data): clamp, so the reader's nw never wraps
      // and its loads stay inside this wave's staging buffer
      const uint64_t off64 = reads ? (base - lo) >> 6 : 0ull;
      const uint32_t off = (uint32_t)(off64 < nwords ? off64 : nwords);
      z = decode_job<false>(J, j, &stage[wv][off], (uint32_t)nwords - off, gran, coef, T, s_root, s_lin);
    } else {
      z = decode_job_direct(J, j, md, gran, coef, T, s_root, s_lin);
    }
  }
  // zero tails of the wave's 64 rows (consecutive jobs), one row at a time
  // with the whole wave: contiguous 16-B slots instead of a burst of
  // scattered per-lane stores at the end of every job
  const int lane = threadIdx.x & 63;
  const uint64_t j0 = j - (uint64_t)lane;
  for (int rr = 0; rr < 64; rr++) {
    const int zr = __shfl(z, rr, 64);
    if (zr >= MP3G_LINES) continue;  // wave-uniform
    uint4* row = reinterpret_cast<uint4*>(coef + (j0 + rr) * MP3G_LINES);
    for (int s8 = (zr >> 3) + lane; s8 < MP3G_LINES / 8; s8 += 64) row[s8] = make_uint4(0u, 0u, 0u, 0u);
  }
}

}  // namespace huff

hipError_t launch_huffman(const mp3g_hjob* d_jobs, uint64_t n_jobs, const uint8_t* d_md, mp3g_granule* d_gran,
                          int16_t* d_coef, hipStream_t stream) {
  if (n_jobs == 0) return hipSuccess;
  const uint64_t blocks = (n_jobs + huff::kThreads - 1) / huff::kThreads;
  hipLaunchKernelGGL(huff::huffman_kernel, dim3((uint32_t)blocks), dim3(huff::kThreads), 0, stream, d_jobs, n_jobs,
                     d_md, d_gran, d_coef);
  return hipGetLastError();
}

}  // namespace mp3g
