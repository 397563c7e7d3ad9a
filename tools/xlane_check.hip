// On-device check of go-mp3_amd/csrc/xlane.h against ds_bpermute shuffles.
// Build: hipcc --offload-arch=gfx950 -O3 tools/xlane_check.hip -o tools/xlane_check
#include <cstdio>
#include "../go-mp3_amd/csrc/xlane.h"
__global__ void k(int* bad) {
  const int l = threadIdx.x;
  const float v = 1000.0f + l;
  int b = 0;
  if (l > 0 && mp3g::xl::from_prev(v) != __shfl_up(v, 1)) b |= 1;
  if (l < 63 && mp3g::xl::from_next(v) != __shfl_down(v, 1)) b |= 2;
  if (mp3g::xl::xor32(v) != __shfl_xor(v, 32)) b |= 4;
  if (mp3g::xl::xor31(v) != __shfl_xor(v, 31)) b |= 8;
  if (mp3g::xl::xor32i(l) != (l ^ 32)) b |= 16;
  bad[l] = b;
}
int main() {
  int* d; int h[64];
  if (hipMalloc(&d, 256) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, 256, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int any = 0;
  for (int i = 0; i < 64; i++) if (h[i]) { printf("lane %d bad mask %d\n", i, h[i]); any = 1; }
  printf(any ? "XLANE FAIL\n" : "XLANE OK\n");
  return any;
}
