// Microbenchmark: issue cost of single VALU instruction kinds on gfx950 at
// the fast kernel's occupancy (16 waves per CU = 4 per SIMD), from s_memtime
// per wave.  Prints cycles per instruction per SIMD (4 waves' instructions
// share one SIMD).  hipcc --offload-arch=gfx950 -O3 tools/valu_cost.hip -o tools/valu_cost
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X X X X X X X X
// 8 independent registers per step, 8 steps per iteration
#define KERNEL(NAME, INSTR, CONS)                                                                         \
  __global__ void __launch_bounds__(256) NAME(float* out, int iters, unsigned long long* cyc) {        \
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, \
          a7 = a0 + 7, b0 = 1.0001f, b1 = 0.9999f;                                                       \
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();                 \
    for (int it = 0; it < iters; it++) {                                                                  \
      R8(asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)             \
                      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)    \
                      : CONS(b0), CONS(b1));)                                                             \
    }                                                                                                     \
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();                 \
    if ((threadIdx.x & 63) == 0) { cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0; cyc[4096 + blockIdx.x * 4 + (threadIdx.x >> 6)] = r1 - r0; } \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                   \
  }
#define VV(x) "v"(x)
#define I_ADD(i) "v_add_f32 %" #i ", %" #i ", %8\n"
#define I_FMA(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n"
#define I_FMAC(i) "v_fmac_f32 %" #i ", %8, %9\n"
#define I_MUL(i) "v_mul_f32 %" #i ", %" #i ", %8\n"
#define I_MOV(i) "v_mov_b32 %" #i ", %8\n"
#define I_CND(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n"
#define I_DPP(i) "v_mov_b32_dpp %" #i ", %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define I_EXP(i) "v_exp_f32 %" #i ", %8\n"
#define I_LOG(i) "v_log_f32 %" #i ", %8\n"
#define I_SWP(i) "v_permlane32_swap_b32 %" #i ", %8\n"
#define I_BFE(i) "v_bfe_u32 %" #i ", %8, 3, 5\n"
#define I_BCNT(i) "v_bcnt_u32_b32 %" #i ", %8, %" #i "\n"
#define I_LSHLADD(i) "v_lshl_add_u32 %" #i ", %8, 1, %" #i "\n"
#define I_CVT(i) "v_cvt_f32_i32 %" #i ", %8\n"
#define I_MED3(i) "v_med3_f32 %" #i ", %" #i ", %8, %9\n"
#define I_PERM(i) "v_perm_b32 %" #i ", %8, %" #i ", %9\n"
#define I_FMAMIX(i) "v_fma_mix_f32 %" #i ", %" #i ", %8, %9 op_sel_hi:[0,0,1]\n"
#define I_CNDE(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, s[40:41]\n"
#define I_CNDV(i) "v_cndmask_b32 %" #i ", %8, %" #i ", vcc\n"
#define I_FMAS(i) "v_fma_f32 %" #i ", %" #i ", s40, %9\n"
#define I_FMACDPP(i) "v_fmac_f32_dpp %" #i ", %8, %9 row_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define I_XOR(i) "v_xor_b32 %" #i ", %8, %" #i "\n"
#define I_ADDU(i) "v_add_u32 %" #i ", %8, %" #i "\n"
#define I_SUBF(i) "v_sub_f32 %" #i ", %8, %" #i "\n"
#define I_RFL(i) "v_readfirstlane_b32 s40, %" #i "\n"
#define I_CNDV2(i) "v_cmp_gt_f32 vcc, %8, %9\n v_cndmask_b32 %" #i ", %8, %" #i ", vcc\n"
#define I_CMP(i) "v_cmp_gt_f32 s[40:41], %" #i ", %8\n"
#define I_CMPV(i) "v_cmp_gt_f32 vcc, %" #i ", %8\n"
#define I_CNDE2(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, vcc\n"
#define I_CVTI(i) "v_cvt_i32_f32 %" #i ", %8\n"
#define I_MADU(i) "v_mad_u32_u24 %" #i ", %8, %9, %" #i "\n"
#define I_MULU(i) "v_mul_u32_u24 %" #i ", %8, %" #i "\n"
#define I_SWP16(i) "v_permlane16_swap_b32 %" #i ", %8\n"
#define I_LDEXP(i) "v_ldexp_f32 %" #i ", %" #i ", %8\n"
#define I_BFI(i) "v_bfi_b32 %" #i ", %8, %" #i ", %9\n"
KERNEL(k_add, I_ADD, VV)
KERNEL(k_fma, I_FMA, VV)
KERNEL(k_fmac, I_FMAC, VV)
KERNEL(k_mul, I_MUL, VV)
KERNEL(k_mov, I_MOV, VV)
KERNEL(k_cnd, I_CND, VV)
KERNEL(k_dpp, I_DPP, VV)
KERNEL(k_exp, I_EXP, VV)
KERNEL(k_log, I_LOG, VV)
KERNEL(k_swp, I_SWP, VV)
KERNEL(k_bfe, I_BFE, VV)
KERNEL(k_bcnt, I_BCNT, VV)
KERNEL(k_lshladd, I_LSHLADD, VV)
KERNEL(k_cvt, I_CVT, VV)
KERNEL(k_med3, I_MED3, VV)
KERNEL(k_perm, I_PERM, VV)
KERNEL(k_fmamix, I_FMAMIX, VV)
KERNEL(k_bfi, I_BFI, VV)
KERNEL(k_cndv2, I_CNDV2, VV)
KERNEL(k_cmp, I_CMP, VV)
KERNEL(k_cmpv, I_CMPV, VV)
KERNEL(k_cnde2, I_CNDE2, VV)
KERNEL(k_cvti, I_CVTI, VV)
KERNEL(k_madu, I_MADU, VV)
KERNEL(k_mulu, I_MULU, VV)
KERNEL(k_swp16, I_SWP16, VV)
KERNEL(k_ldexp, I_LDEXP, VV)
KERNEL(k_cnde, I_CNDE, VV)
KERNEL(k_cndv, I_CNDV, VV)
KERNEL(k_fmas, I_FMAS, VV)
KERNEL(k_fmacdpp, I_FMACDPP, VV)
KERNEL(k_xor, I_XOR, VV)
KERNEL(k_addu, I_ADDU, VV)
KERNEL(k_subf, I_SUBF, VV)

// packed: 64-bit operands
typedef float f2 __attribute__((ext_vector_type(2)));
#define PKERNEL(NAME, INSTR)                                                                               \
  __global__ void __launch_bounds__(256) NAME(float* out, int iters, unsigned long long* cyc) {          \
    f2 a0 = {(float)threadIdx.x, 1}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,      \
       a6 = a0 + 6, a7 = a0 + 7, b0 = {1.0001f, 0.999f}, b1 = {0.5f, 0.25f};                                \
    unsigned long long t0 = __builtin_amdgcn_s_memtime();                                                   \
    for (int it = 0; it < iters; it++) {                                                                    \
      R8(asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)               \
                      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                      : "v"(b0), "v"(b1));)                                                                 \
    }                                                                                                       \
    unsigned long long t1 = __builtin_amdgcn_s_memtime();                                                   \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;                       \
    f2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;                                                 \
  }
#define P_FMA(i) "v_pk_fma_f32 %" #i ", %" #i ", %8, %9\n"
#define P_ADD(i) "v_pk_add_f32 %" #i ", %" #i ", %8\n"
#define P_MUL(i) "v_pk_mul_f32 %" #i ", %" #i ", %8\n"
#define P_MOV(i) "v_pk_mov_b32 %" #i ", %8, %9 op_sel:[0,1]\n"
#define P_FMAS(i) "v_pk_fma_f32 %" #i ", %" #i ", s[40:41], %9 op_sel_hi:[1,0,1]\n"
#define P_FMAOP(i) "v_pk_fma_f32 %" #i ", %" #i ", %8, %9 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]\n"
#define P_MOV64(i) "v_mov_b64 %" #i ", %8\n"
PKERNEL(p_fma, P_FMA)
PKERNEL(p_add, P_ADD)
PKERNEL(p_mul, P_MUL)
PKERNEL(p_mov, P_MOV)
PKERNEL(p_mov64, P_MOV64)
PKERNEL(p_fmas, P_FMAS)
PKERNEL(p_fmaop, P_FMAOP)

typedef void (*kfn)(float*, int, unsigned long long*);
int main() {
  const int blocks = 256 * 4, threads = 256, iters = 2000;  // 4 blocks x 4 waves per CU = 4 waves per SIMD
  float* d;
  unsigned long long* c;
  hipMalloc(&d, blocks * threads * 4);
  hipMalloc(&c, 2 * blocks * 4 * 8);
  static unsigned long long h[2 * 256 * 4 * 4];
  struct {
    const char* n;
    kfn f;
  } ks[] = {{"v_add_f32", k_add},     {"v_fma_f32", k_fma},       {"v_fmac_f32", k_fmac},   {"v_mul_f32", k_mul},
            {"v_mov_b32", k_mov},     {"v_cndmask_b32", k_cnd},   {"v_mov_b32_dpp", k_dpp}, {"v_exp_f32", k_exp},
            {"v_log_f32", k_log},     {"v_permlane32_swap", k_swp}, {"v_bfe_u32", k_bfe},   {"v_bcnt_u32", k_bcnt},
            {"v_lshl_add_u32", k_lshladd}, {"v_cvt_f32_i32", k_cvt}, {"v_med3_f32", k_med3}, {"v_perm_b32", k_perm},
            {"v_fma_mix_f32", k_fmamix}, {"v_bfi_b32", k_bfi},    {"v_pk_fma_f32", p_fma},  {"v_pk_add_f32", p_add},
            {"v_pk_mul_f32", p_mul},  {"v_pk_mov_b32", p_mov},   {"v_mov_b64", p_mov64},
            {"v_cndmask_e64 sgpr", k_cnde}, {"v_cndmask vcc", k_cndv}, {"v_fma_f32 sgpr", k_fmas},
            {"v_fmac_f32_dpp", k_fmacdpp}, {"v_xor_b32", k_xor}, {"v_add_u32", k_addu}, {"v_sub_f32", k_subf},
            {"v_pk_fma sgpr", p_fmas}, {"v_pk_fma opsel/neg", p_fmaop}, {"v_add_f32 (again)", k_add},
            {"v_cmp+v_cndmask vcc (2 instr)", k_cndv2}, {"v_cmp_gt_f32 sgpr", k_cmp}, {"v_cmp_gt_f32 vcc", k_cmpv},
            {"v_cndmask_e64 vcc", k_cnde2}, {"v_cvt_i32_f32", k_cvti}, {"v_mad_u32_u24", k_madu}, {"v_mul_u32_u24", k_mulu},
            {"v_permlane16_swap", k_swp16}, {"v_ldexp_f32", k_ldexp}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, iters, c);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, c, 2 * blocks * 4 * 8, hipMemcpyDeviceToHost);
    double s = 0, rt = 0;
    for (int i = 0; i < blocks * 4; i++) { s += h[i]; rt += h[4096 + i]; }
    printf("[memtime ticks per us: %.0f] ", s / (rt / 100.0));
    const double wave_cycles = s / (blocks * 4);
    const double instrs = (double)iters * 64;
    // 4 waves share a SIMD: cycles per instruction of the SIMD
    printf("%-20s %6.2f cycles/instr/SIMD (wave: %.2f)\n", k.n, wave_cycles / instrs / 4.0, wave_cycles / instrs);
  }
  return 0;
}
