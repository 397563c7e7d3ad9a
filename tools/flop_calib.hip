// Calibration of the gfx950 flop counters (SQ_INSTS_VALU_FLOPS_FP32 /
// _FP32_TRANS and the per-class SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F32): one
// kernel per instruction kind with a known count -- every lane executes
// ITERS x 64 instructions of that kind -- so a rocprofv3 --pmc pass over this
// program gives each counter's weight per instruction (is a v_pk_fma_f32 one
// FMA or two?  does FLOPS_FP32 count lanes?).  Used to turn the bench
// kernels' counters into executed flops (tools/profile.sh flops pass,
// tools/summarize_profile.py).
//   hipcc --offload-arch=gfx950 -O3 tools/flop_calib.hip -o tools/flop_calib
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 100, kBlocks = 256, kThreads = 256;

#define R8(X) X X X X X X X X
#define KERNEL(NAME, T, INIT, INSTR)                                                                   \
  __global__ void __launch_bounds__(256) NAME(float* out, int iters) {                                 \
    T a0 = INIT(0), a1 = INIT(1), a2 = INIT(2), a3 = INIT(3), a4 = INIT(4), a5 = INIT(5), a6 = INIT(6), \
      a7 = INIT(7), b0 = INIT(8), b1 = INIT(9);                                                        \
    for (int it = 0; it < iters; it++) {                                                               \
      R8(asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)          \
                      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                      : "v"(b0), "v"(b1));)                                                            \
    }                                                                                                  \
    T s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = sum(s);                                               \
  }
__device__ __forceinline__ float sum(float x) { return x; }
__device__ __forceinline__ float sum(f2 x) { return x.x + x.y; }
#define INIT1(k) (0.001f * (threadIdx.x + k))
#define INIT2(k) (f2){0.001f * (threadIdx.x + k), 0.002f * (threadIdx.x + k)}
#define I_FMA(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n"
#define I_ADD(i) "v_add_f32 %" #i ", %" #i ", %8\n"
#define I_MUL(i) "v_mul_f32 %" #i ", %" #i ", %8\n"
#define I_EXP(i) "v_exp_f32 %" #i ", %8\n"
#define I_PKFMA(i) "v_pk_fma_f32 %" #i ", %" #i ", %8, %9\n"
#define I_PKMUL(i) "v_pk_mul_f32 %" #i ", %" #i ", %8\n"
#define I_PKADD(i) "v_pk_add_f32 %" #i ", %" #i ", %8\n"
KERNEL(calib_fma_f32, float, INIT1, I_FMA)
KERNEL(calib_add_f32, float, INIT1, I_ADD)
KERNEL(calib_mul_f32, float, INIT1, I_MUL)
KERNEL(calib_exp_f32, float, INIT1, I_EXP)
KERNEL(calib_pk_fma_f32, f2, INIT2, I_PKFMA)
KERNEL(calib_pk_mul_f32, f2, INIT2, I_PKMUL)
KERNEL(calib_pk_add_f32, f2, INIT2, I_PKADD)

int main() {
  float* out;
  if (hipMalloc(&out, kBlocks * kThreads * sizeof(float)) != hipSuccess) return 1;
  void (*ks[])(float*, int) = {calib_fma_f32, calib_add_f32, calib_mul_f32, calib_exp_f32,
                               calib_pk_fma_f32, calib_pk_mul_f32, calib_pk_add_f32};
  for (auto k : ks) hipLaunchKernelGGL(k, dim3(kBlocks), dim3(kThreads), 0, 0, out, kIters);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  // per kernel: lanes x instructions per lane, and wave-instructions
  const double lanes = (double)kBlocks * kThreads, per_lane = kIters * 64.0;
  std::printf("{\"lane_instructions\": %.0f, \"wave_instructions\": %.0f}\n", lanes * per_lane,
              lanes / 64 * per_lane);
  hipFree(out);
  return 0;
}
