// store_calib.hip -- calibration of rocprofv3's WRITE_SIZE for the main-data
// kernel's store patterns (MI355X_MICROARCH.md: WRITE_SIZE
// reads 16-B-per-lane streaming stores exactly, other widths uncalibrated).
// Each kernel writes a byte count known on the host (printed); run under
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace -- ./store_calib
// and divide the counter (KiB) by the printed bytes.
//   k_stream16   the reference: 16 B per lane, consecutive lanes consecutive
//   k_row32      huffman_job.h LineWriter: one lane per 1,152-B coefficient
//                row, each row written front to back in 32-B blocks (two
//                back-to-back 16-B stores), every row whole
//   k_row32_c1   the same up to a per-row count1 (a multiple of 16 lines,
//                MP3G_HUFF_ROWS_COUNT1): only the bytes below it
//   k_sf         SfRegs::store: bytes [11, 72) of each 72-B channel record of
//                a 160-B granule (1 + 4 + 8/16 + 3 x 16 B stores per job)
//   k_zero_tail  huffman_dev.hip's zero fill of the rows from count1 to 576
//                by the wave's lanes together (16 B per lane, row by row)
//   k_slow<B>    k_row32_c1's rows written in B-byte blocks with a dependent
//                VALU chain (~ one block's symbol decode) before each block,
//                at the main-data kernel's occupancy (16 waves per CU through
//                its LDS): a row's 128-B line stays partial in the L2 for as
//                long as the decode of its next blocks takes
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kRow = 1152;  // bytes per coefficient row (576 x int16)

__host__ __device__ inline uint32_t c1_lines(uint32_t r) {  // count1 rounded up to 16 lines, 0..576
  uint32_t h = r * 2654435761u;
  h ^= h >> 15;
  return 16u * (h % 37u);
}

__global__ void __launch_bounds__(256) k_stream16(uint4* out, size_t n16) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    out[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

template <bool kCount1>
__global__ void __launch_bounds__(256) k_row32(uint8_t* out, int rows) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const uint32_t lines = kCount1 ? c1_lines((uint32_t)r) : 576u;
  uint4* p = reinterpret_cast<uint4*>(out + (size_t)r * kRow);
  for (uint32_t b = 0; b < lines / 16; b++) {  // 32-B block = two 16-B stores
    p[2 * b] = make_uint4(r, b, 1, 2);
    p[2 * b + 1] = make_uint4(r, b, 3, 4);
  }
}

__global__ void __launch_bounds__(256) k_sf(uint8_t* gran, int jobs) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= jobs) return;
  const int ch = j & 1;
  uint8_t* cb = gran + (size_t)(j >> 1) * 160 + 8 + 72 * ch;
  const uint32_t v = (uint32_t)j;
  cb[11] = (uint8_t)v;
  *reinterpret_cast<uint32_t*>(cb + 12) = v;
  if (ch == 0) {
    *reinterpret_cast<uint2*>(cb + 16) = make_uint2(v, v);
    *reinterpret_cast<uint4*>(cb + 24) = make_uint4(v, v, v, v);
    *reinterpret_cast<uint4*>(cb + 40) = make_uint4(v, v, v, v);
    *reinterpret_cast<uint4*>(cb + 56) = make_uint4(v, v, v, v);
  } else {
    *reinterpret_cast<uint4*>(cb + 16) = make_uint4(v, v, v, v);
    *reinterpret_cast<uint4*>(cb + 32) = make_uint4(v, v, v, v);
    *reinterpret_cast<uint4*>(cb + 48) = make_uint4(v, v, v, v);
    *reinterpret_cast<uint2*>(cb + 64) = make_uint2(v, v);
  }
}

// rows [64 w, 64 w + 64) of wave w: each row's tail [count1, 576) zeroed by
// the wave's lanes, 16 B per lane per step
__global__ void __launch_bounds__(256) k_zero_tail(uint8_t* out, int rows) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 256 + (threadIdx.x & ~63));
  for (int q = 0; q < 64 && r0 + q < rows; q++) {
    const uint32_t z = c1_lines((uint32_t)(r0 + q));
    uint4* p = reinterpret_cast<uint4*>(out + (size_t)(r0 + q) * kRow);
    for (uint32_t k = z / 8 + lane; k < 72; k += 64) p[k] = make_uint4(0, 0, 0, 0);
  }
}

template <int kBytes>
__global__ void __launch_bounds__(256) k_slow(uint8_t* out, int rows, int spin) {
  extern __shared__ uint32_t lds[];  // occupancy only
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const uint32_t lines = c1_lines((uint32_t)r);
  uint4* p = reinterpret_cast<uint4*>(out + (size_t)r * kRow);
  float x = (float)r;
  for (uint32_t b = 0; b < 2 * lines / kBytes; b++) {
    for (int i = 0; i < spin; i++) x = __builtin_fmaf(x, 0.999f, 1.0f);
    const uint32_t v = __float_as_uint(x) & 1u;  // 0: the stores depend on the chain
#pragma unroll
    for (int q = 0; q < kBytes / 16; q++) p[(kBytes / 16) * b + q] = make_uint4(r, b, q, v);
  }
  if (x == -1.0f) lds[threadIdx.x] = 1u;
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 4194304;  // c3: 2 x 2,097,152 jobs
  uint8_t* d = nullptr;
  const size_t bytes = (size_t)rows * kRow;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  uint64_t c1_bytes = 0, tail_bytes = 0;
  for (int r = 0; r < rows; r++) {
    c1_bytes += 2ull * c1_lines((uint32_t)r);
    tail_bytes += kRow - 2ull * c1_lines((uint32_t)r);
  }
  const int blocks = (rows + 255) / 256;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int v = 0; v < 8; v++) {
    (void)hipEventRecord(a);
    uint64_t known = 0;
    const char* name = "";
    if (v == 0) {
      hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint4*>(d), bytes / 16);
      known = bytes, name = "k_stream16";
    } else if (v == 1) {
      hipLaunchKernelGGL(k_row32<false>, dim3(blocks), dim3(256), 0, 0, d, rows);
      known = bytes, name = "k_row32";
    } else if (v == 2) {
      hipLaunchKernelGGL(k_row32<true>, dim3(blocks), dim3(256), 0, 0, d, rows);
      known = c1_bytes, name = "k_row32_c1";
    } else if (v == 3) {
      hipLaunchKernelGGL(k_sf, dim3(blocks), dim3(256), 0, 0, d, rows);
      known = (uint64_t)rows * 61, name = "k_sf";  // bytes [11, 72) of each channel record
    } else if (v == 4) {
      hipLaunchKernelGGL(k_zero_tail, dim3(blocks), dim3(256), 0, 0, d, rows);
      known = tail_bytes, name = "k_zero_tail";
    } else if (v == 5) {
      hipLaunchKernelGGL(k_slow<32>, dim3(blocks), dim3(256), 36 * 1024, 0, d, rows, 64);
      known = c1_bytes, name = "k_slow32";
    } else if (v == 6) {
      hipLaunchKernelGGL(k_slow<64>, dim3(blocks), dim3(256), 36 * 1024, 0, d, rows, 128);
      known = c1_bytes, name = "k_slow64";
    } else {
      hipLaunchKernelGGL(k_slow<32>, dim3(blocks), dim3(256), 36 * 1024, 0, d, rows, 0);
      known = c1_bytes, name = "k_slow32_nospin";
    }
    (void)hipEventRecord(b);
    if (hipEventSynchronize(b) != hipSuccess) return 2;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%s known_bytes %llu ms %.4f\n", name, (unsigned long long)known, ms);
  }
  (void)hipFree(d);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
