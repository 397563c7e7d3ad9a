// Microbenchmark: wave64 throughput of v_fma_f32 vs v_pk_fma_f32 on gfx950
// (does packed FP32 double the FMA rate?).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float float2_t __attribute__((ext_vector_type(2)));
__global__ void k_fma(float* out, float a, float b, int iters) {
  float x[16];
  for (int i = 0; i < 16; i++) x[i] = threadIdx.x + i;
  for (int it = 0; it < iters; it++)
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = __builtin_fmaf(x[i], a, b);
  float s = 0; for (int i = 0; i < 16; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pkfma(float* out, float a, float b, int iters) {
  float2_t x[8];
  for (int i = 0; i < 8; i++) x[i] = (float2_t){(float)threadIdx.x + i, (float)i};
  float2_t av = {a, a}, bv = {b, b};
  for (int it = 0; it < iters; it++)
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_elementwise_fma(x[i], av, bv);
  float s = 0; for (int i = 0; i < 8; i++) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  float* d; hipMalloc(&d, 256 * 1024 * 4 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 4096, blocks = 256 * 8, threads = 256;
  for (int rep = 0; rep < 2; rep++) {
    float ms;
    hipEventRecord(e0); hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, d, 0.999f, 0.001f, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double fmas = (double)blocks * threads * iters * 16;
    printf("v_fma_f32     : %.1f TFLOP/s\n", 2 * fmas / ms / 1e9);
    hipEventRecord(e0); hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(threads), 0, 0, d, 0.999f, 0.001f, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("v_pk_fma_f32  : %.1f TFLOP/s (%.0f FMA counted per lane-op pair)\n", 2 * fmas / ms / 1e9, 2.0);
  }
  return 0;
}
