// pk_opsel.hip -- does gfx950 honour op_sel / op_sel_hi / neg_lo / neg_hi on
// an SGPR-pair source of v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32?  (The
// fast kernel's twiddles would then need one constant pair (c, s) instead of
// two.)  Prints each form's result against the expected pair.
//   hipcc --offload-arch=gfx950 -O2 -o tools/pk_opsel tools/pk_opsel.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void probe(const float* in, float* out) {
  const f2 a = {in[0], in[1]}, acc = {in[2], in[3]};
  const float c = in[4], s = in[5];
  unsigned long long cs;
  {
    unsigned lo, hi;
    std::memcpy(&lo, &c, 4);
    std::memcpy(&hi, &s, 4);
    cs = (unsigned long long)hi << 32 | lo;
  }
  cs = __builtin_amdgcn_readfirstlane((unsigned)cs) | (unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(cs >> 32)) << 32;
  f2 r[8];
  // 0: a * (c, s)
  asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(r[0]) : "v"(a), "s"(cs));
  // 1: a * (s, c): swap the SGPR halves
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r[1]) : "v"(a), "s"(cs));
  // 2: a * (c, -s)
  asm volatile("v_pk_mul_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r[2]) : "v"(a), "s"(cs));
  // 3: a * (s, -c)
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r[3]) : "v"(a), "s"(cs));
  // 4: (a.x, a.x) * (c, s)
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r[4]) : "v"(a), "s"(cs));
  // 5: fma((a.y, a.y), (s, c), acc)
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r[5]) : "v"(a), "s"(cs), "v"(acc));
  // 6: fma((a.y, a.y), (s, -c), acc)
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[0,1,0]" : "=v"(r[6]) : "v"(a), "s"(cs), "v"(acc));
  // 7: acc + (-i) a = (acc.x + a.y, acc.y - a.x)
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r[7]) : "v"(acc), "v"(a));
  if (threadIdx.x == 0)
    for (int i = 0; i < 8; i++) {
      out[2 * i] = r[i].x;
      out[2 * i + 1] = r[i].y;
    }
}

int main() {
  const float h_in[6] = {3.0f, 5.0f, 7.0f, 11.0f, 2.0f, 0.5f};  // a, acc, c, s
  const float a0 = 3, a1 = 5, x0 = 7, x1 = 11, c = 2, s = 0.5f;
  const float want[16] = {a0 * c, a1 * s, a0 * s, a1 * c, a0 * c, -a1 * s, a0 * s, -a1 * c,
                          a0 * c, a0 * s, a1 * s + x0, a1 * c + x1, a1 * s + x0, -a1 * c + x1, x0 + a1, x1 - a0};
  float *d_in, *d_out, h_out[16];
  if (hipMalloc(&d_in, sizeof h_in) != hipSuccess || hipMalloc(&d_out, sizeof h_out) != hipSuccess) return 1;
  if (hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_in, d_out);
  if (hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad = 0;
  for (int i = 0; i < 8; i++) {
    const bool ok = h_out[2 * i] == want[2 * i] && h_out[2 * i + 1] == want[2 * i + 1];
    bad += !ok;
    std::printf("form %d: got (%g, %g) want (%g, %g) %s\n", i, h_out[2 * i], h_out[2 * i + 1], want[2 * i],
                want[2 * i + 1], ok ? "ok" : "DIFFERS");
  }
  return bad ? 2 : 0;
}
