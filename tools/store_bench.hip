// store_bench.hip -- how the coefficient-store pattern of the main-data
// kernel prices on gfx950: 64 rows of 1152 B per wave, written
//   v0: one lane per row, 72 x 16-B stores per lane (row-per-lane)
//   v1: 4 lanes per 64-B segment of a row (16 rows per store instruction)
//   v2: 8 lanes per 128-B segment (8 rows per store instruction)
//   v3: the wave's 72 KB contiguous, 1 KB per store instruction
// Usage: ./store_bench [rows]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kRow = 1152;

__global__ void __launch_bounds__(256) v0(uint4* out, int rows) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  uint4* p = out + (size_t)r * (kRow / 16);
  for (int k = 0; k < kRow / 16; k++) p[k] = make_uint4(r, k, 1, 2);
}
template <int kLanes>  // lanes per segment (segment = 16 * kLanes bytes)
__global__ void __launch_bounds__(256) vseg(uint4* out, int rows) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 256 + (threadIdx.x & ~63));
  const int per = 64 / kLanes;  // rows per instruction
  for (int c = 0; c < kRow / (16 * kLanes); c++)
    for (int q = 0; q < kLanes; q++) {
      const int r = r0 + q * per + lane / kLanes;
      if (r < rows) out[(size_t)r * (kRow / 16) + c * kLanes + lane % kLanes] = make_uint4(r, c, q, 2);
    }
}
__global__ void __launch_bounds__(256) v3(uint4* out, int rows) {
  const int lane = threadIdx.x & 63;
  const size_t r0 = (blockIdx.x * 256 + (threadIdx.x & ~63));
  if ((int)r0 >= rows) return;
  uint4* p = out + r0 * (kRow / 16);
  for (int k = 0; k < kRow / 16; k++) p[k * 64 + lane] = make_uint4(lane, k, 1, 2);
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 4194304;
  uint4* d = nullptr;
  if (hipMalloc(&d, (size_t)rows * kRow) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int blocks = (rows + 255) / 256;
  for (int v = 0; v < 4; v++) {
    float best = 1e9f;
    for (int it = 0; it < 6; it++) {
      (void)hipEventRecord(a);
      if (v == 0) hipLaunchKernelGGL(v0, dim3(blocks), dim3(256), 0, 0, d, rows);
      if (v == 1) hipLaunchKernelGGL(vseg<4>, dim3(blocks), dim3(256), 0, 0, d, rows);
      if (v == 2) hipLaunchKernelGGL(vseg<8>, dim3(blocks), dim3(256), 0, 0, d, rows);
      if (v == 3) hipLaunchKernelGGL(v3, dim3(blocks), dim3(256), 0, 0, d, rows);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      if (it && ms < best) best = ms;
    }
    printf("v%d %.4f ms  %.1f GB/s\n", v, best, (double)rows * kRow / (best * 1e-3) / 1e9);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
