// valu_rate.hip -- issue rate of the integer VALU forms the main-data kernel's
// bit reader uses (v_lshrrev_b64 / v_lshlrev_b64 vs 32-bit shifts and
// v_alignbit_b32), relative to v_add_u32.  Each lane runs 8 independent
// chains of the instruction; 16 waves per CU on every CU; HIP-event time.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate && ./tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

#define BODY8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

template <int kKind>
__global__ void __launch_bounds__(256) rate_kernel(unsigned long long* out, unsigned sh) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
                     a7 = a0 + 7;
  const unsigned long long m = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
  unsigned long long m2;
  for (int it = 0; it < kIters; it++) {
    if constexpr (kKind == 0) {  // v_add_u32 (on the low halves)
#define OP(x) asm volatile("v_add_u32 %0, %1, %0" : "+v"(*reinterpret_cast<unsigned*>(&x)) : "v"(sh));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 1) {  // v_lshrrev_b64
#define OP(x) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(x) : "v"(sh));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 2) {  // v_lshlrev_b64
#define OP(x) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(x) : "v"(sh));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 3) {  // v_lshrrev_b32
#define OP(x) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(*reinterpret_cast<unsigned*>(&x)) : "v"(sh));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 4) {  // v_alignbit_b32
#define OP(x)                                                                          \
  asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(*reinterpret_cast<unsigned*>(&x)) \
               : "v"(*(reinterpret_cast<unsigned*>(&x) + 1)), "v"(sh));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 5) {  // v_mov_b64
#define OP(x) asm volatile("v_mov_b64 %0, %0" : "+v"(x));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 6) {  // v_cndmask_b32 (vcc from a compare outside the loop)
#define OP(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(*reinterpret_cast<unsigned*>(&x)) : "v"(sh));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 7) {  // v_cndmask_b32 (VOP3, lane mask in an SGPR pair)
#define OP(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(*reinterpret_cast<unsigned*>(&x)) : "v"(sh), "s"(m));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 8) {  // v_add_u32 with an SGPR operand
#define OP(x) asm volatile("v_add_u32 %0, %1, %0" : "+v"(*reinterpret_cast<unsigned*>(&x)) : "s"(sh));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 9) {  // v_bfi_b32
#define OP(x)                                                                        \
  asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(*reinterpret_cast<unsigned*>(&x)) \
               : "v"(sh), "v"(*(reinterpret_cast<unsigned*>(&x) + 1)));
      BODY8(OP)
#undef OP
    } else if constexpr (kKind == 10) {  // v_cndmask_b32 (VOP3, lane mask from a VALU compare in the loop)
#define OP(x)                                                                                  \
  asm volatile("v_cmp_lt_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1"              \
               : "+v"(*reinterpret_cast<unsigned*>(&x)), "=s"(m2) : "v"(sh));
      BODY8(OP)
#undef OP
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int kKind>
float time_kind(unsigned long long* d, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(rate_kernel<kKind>, dim3(blocks), dim3(256), 0, 0, d, 3u);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(rate_kernel<kKind>, dim3(blocks), dim3(256), 0, 0, d, 3u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 4;  // 16 waves per CU
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned long long) * blocks * 256) != hipSuccess) return 1;
  const char* names[] = {"v_add_u32", "v_lshrrev_b64", "v_lshlrev_b64", "v_lshrrev_b32", "v_alignbit_b32", "v_mov_b64",
                         "v_cndmask_b32", "v_cndmask_b32_e64 (SGPR mask)", "v_add_u32 (SGPR operand)", "v_bfi_b32",
                         "v_cmp_lt_u32_e64 + v_cndmask_b32_e64"};
  float t[11];
  t[0] = time_kind<0>(d, blocks);
  t[1] = time_kind<1>(d, blocks);
  t[2] = time_kind<2>(d, blocks);
  t[3] = time_kind<3>(d, blocks);
  t[4] = time_kind<4>(d, blocks);
  t[5] = time_kind<5>(d, blocks);
  t[6] = time_kind<6>(d, blocks);
  t[7] = time_kind<7>(d, blocks);
  t[8] = time_kind<8>(d, blocks);
  t[9] = time_kind<9>(d, blocks);
  t[10] = time_kind<10>(d, blocks);
  // wave-instructions per SIMD per ms: waves per SIMD (4) x 8 x kIters
  printf("{");
  for (int k = 0; k < 11; k++)
    printf("%s\"%s\": {\"ms\": %.4f, \"relative_cost\": %.2f}", k ? ", " : "", names[k], t[k], t[k] / t[0]);
  printf("}\n");
  (void)hipFree(d);
  return 0;
}
