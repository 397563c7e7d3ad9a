// Microbenchmark: does v_mfma_f32_32x32x2_f32 steal VALU issue on gfx950?
// 4 waves per SIMD; each loop step issues M MFMAs (independent accumulators)
// and V independent v_fmac_f32.  Prints memtime cycles per step per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f16v __attribute__((ext_vector_type(16)));
template <int M, int V>
__global__ void __launch_bounds__(256) k(float* out, int iters, unsigned long long* cyc) {
  f16v acc0 = {}, acc1 = {};
  float a = threadIdx.x * 1e-3f, b = 1.0f;
  float v[8];
  for (int i = 0; i < 8; i++) v[i] = threadIdx.x + i;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int m = 0; m < M; m++) {
      if (m & 1) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc1, 0, 0, 0);
      else acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < V; j++) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v[j & 7]) : "v"(a), "v"(b));
    }
    if (M == 0) {
#pragma unroll
      for (int j = 0; j < V; j++) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v[j & 7]) : "v"(a), "v"(b));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  float s = 0;
  for (int i = 0; i < 16; i++) s += acc0[i] + acc1[i];
  for (int i = 0; i < 8; i++) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
typedef void (*kfn)(float*, int, unsigned long long*);
int main() {
  const int blocks = 256 * 4, threads = 256, iters = 500;
  float* d;
  unsigned long long* c;
  hipMalloc(&d, blocks * threads * 4);
  hipMalloc(&c, blocks * 4 * 8);
  static unsigned long long h[256 * 4 * 4];
  struct { const char* n; kfn f; int m, v; } ks[] = {
      {"8 mfma", k<8, 0>, 8, 0},         {"8 mfma + 8x8 fmac", k<8, 8>, 8, 8}, {"8 mfma + 8x16 fmac", k<8, 16>, 8, 16},
      {"8 mfma + 8x32 fmac", k<8, 32>, 8, 32}, {"64 fmac", k<0, 64>, 0, 64},    {"128 fmac", k<0, 128>, 0, 128},
      {"256 fmac", k<0, 256>, 0, 256}};
  for (auto& q : ks) {
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(q.f, dim3(blocks), dim3(threads), 0, 0, d, iters, c);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, c, blocks * 4 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks * 4; i++) s += h[i];
    const double per_step = s / (blocks * 4) / iters / 4.0;  // per loop step, per SIMD (4 waves)
    printf("%-22s %8.1f cycles/step/SIMD  (mfma %d, fmac %d)\n", q.n, per_step, q.m, q.m ? q.m * q.v : q.v);
  }
  return 0;
}
