// huffman_dev.hip -- main-data decode on the GPU.
//
// One lane per (granule, channel) job of the host scan (host_parse.cpp,
// FrameScanner): the lane reads its channel's scale factors and Huffman codes
// straight out of the concatenated main-data buffer, writes the scale factors
// + count1 into the granule descriptor (whose side-info fields the scan
// filled) and the channel's 576 int16 coefficients (huffman_job.h).
// Decoding inside a channel is bit-serial; the parallelism is across jobs
// (two per granule, 64 per wave; neighbouring lanes read neighbouring
// main-data bytes).  The Huffman tables (huff_lut.h, 18 KB) live in LDS.
// (compiled as part of kernels.hip)
#include "huffman_job.h"

namespace mp3g {
namespace huff {

constexpr int kThreads = 256;

__global__ void __launch_bounds__(kThreads)
huffman_kernel(const mp3g_hjob* __restrict__ jobs, uint64_t n_jobs, const uint8_t* __restrict__ md,
               mp3g_granule* __restrict__ gran, int16_t* __restrict__ coef) {
  __shared__ uint32_t T[kHuffMaxEntries];
  __shared__ uint32_t s_root[34], s_lin[34];
  const uint32_t n_e = g_huff.n_entries;
  for (uint32_t i = threadIdx.x; i < n_e; i += kThreads) T[i] = g_huff.e[i];
  if (threadIdx.x < 34) {
    s_root[threadIdx.x] = g_huff.root[threadIdx.x];
    s_lin[threadIdx.x] = g_huff.linbits[threadIdx.x];
  }
  __syncthreads();
  const uint64_t j = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (j >= n_jobs) return;
  decode_job(jobs[j], j, md, gran, coef, T, s_root, s_lin);
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
