// fetch_calib.hip -- calibration of rocprofv3's FETCH_SIZE for the fused fast
// kernel's load patterns (MI355X_MICROARCH.md: on gfx950
// FETCH_SIZE reads exactly half the bytes of a wide coalesced 16-B-per-lane
// streaming read; other widths are uncalibrated).  Each kernel reads a byte
// count known on the host (printed) and sinks what it read into one dword per
// wave; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_calib
// and divide the counter (KiB x 1024) by the printed bytes
// (tools/summarize_calib.py).
//   k_stream16   the reference: 16 B per lane, consecutive lanes consecutive
//   k_lines12    granule_fast.hip load_lines_lim: one wave per 64-granule
//                chunk, granule after granule; lane (ch, sb) reads its 18
//                lines as three 12-B buffer loads at ch * 1152 + 36 sb, every
//                row whole
//   k_lines12_c1 the same, the loads of a lane only below its row's count1
//                (bytes requested: 12 per issued load, as the fused kernel)
//   k_lines12_c1_slow<spin> k_lines12_c1 with a dependent VALU chain after
//                each granule (~ the fused kernel's ~4,000 cycles of work per
//                granule at 16 waves per CU): the time between a wave's
//                granules as in the real kernel
//   k_desc       the 160-B descriptors, lanes 0..9 one 16-B load each
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr int kGranBytes = 2304;  // [2][576] int16
constexpr int kChunk = 64;        // granules per wave (c3's auto chunk)
constexpr int kLds = 64 * 1024;   // dynamic LDS per 8-wave workgroup: 2 per CU

__host__ __device__ inline int c1_of(uint32_t g, int ch) {  // count1 in lines, 0..576, c3-like spread
  uint32_t h = (2 * g + (uint32_t)ch) * 2654435761u;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  return 2 * (int)(h % 289u);
}

__global__ void __launch_bounds__(256) k_stream16(const uint4* in, size_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;  // (never: keeps the loads)
}

template <bool kCount1, int kSpin>
__global__ void __launch_bounds__(512, 4) k_lines12(const int16_t* coef, uint32_t n_gran, uint32_t* sink) {
  extern __shared__ uint32_t lds[];  // occupancy only: 2 workgroups (16 waves) per CU, as the fused kernel
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 8 + (threadIdx.x >> 6);
  const uint32_t g0 = wave * kChunk;
  if (g0 >= n_gran) return;
  const uint32_t g1 = g0 + kChunk < n_gran ? g0 + kChunk : n_gran;
  const int ch = lane >> 5, l0 = 18 * (lane & 31), off = ch * 1152 + 2 * l0;
  uint32_t acc = 0;
  float x = (float)lane;
  for (uint32_t g = g0; g < g1; g++) {
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int16_t*>(coef + (size_t)g * 1152), (short)0, kGranBytes, 0x00020000);
    const int lim = kCount1 ? c1_of(g, ch) : 576;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b96(rc, l0 + 6 * i < lim ? off + 12 * i : 0x7ffffff0, 0, 0);
      acc ^= v[0] ^ v[1] ^ v[2];
    }
    if (kSpin) {
      x += (float)(acc & 1u);
      for (int i = 0; i < kSpin; i++) x = __builtin_fmaf(x, 0.999f, 1.0f);
    }
  }
  if (acc == 0x9e3779b9u || x == -1.0f) {
    lds[threadIdx.x] = acc;
    sink[wave] = lds[threadIdx.x ^ 1];
  }
}

__global__ void __launch_bounds__(256) k_desc(const uint4* gran, uint32_t n_gran, uint32_t* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t acc = 0;
  for (uint32_t g = wave * kChunk; g < (wave + 1) * kChunk && g < n_gran; g++)
    if (lane < 10) {
      const uint4 v = gran[(size_t)g * 10 + lane];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  if (acc == 0x9e3779b9u) sink[wave] = acc;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 2097152u;  // c3's granules
  int16_t* coef = nullptr;
  uint4* gran = nullptr;
  uint32_t* sink = nullptr;
  const size_t cbytes = (size_t)n * kGranBytes;
  if (hipMalloc(&coef, cbytes) != hipSuccess || hipMalloc(&gran, (size_t)n * 160) != hipSuccess ||
      hipMalloc(&sink, 1 << 20) != hipSuccess)
    return 1;
  (void)hipMemset(coef, 1, cbytes);
  (void)hipMemset(gran, 1, (size_t)n * 160);
  uint64_t c1_bytes = 0;
  for (uint32_t g = 0; g < n; g++)
    for (int ch = 0; ch < 2; ch++) {
      const int lim = c1_of(g, ch);
      for (int sb = 0; sb < 32; sb++)
        for (int i = 0; i < 3; i++) c1_bytes += 18 * sb + 6 * i < lim ? 12 : 0;
    }
  const uint32_t waves = (n + kChunk - 1) / kChunk;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int v = 0; v < 6; v++) {
    (void)hipEventRecord(a);
    uint64_t known = 0;
    const char* name = "";
    if (v == 0) {
      hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const uint4*>(coef), cbytes / 16,
                         sink);
      known = cbytes, name = "k_stream16";
    } else if (v == 1) {
      hipLaunchKernelGGL((k_lines12<false, 0>), dim3((waves + 7) / 8), dim3(512), kLds, 0, coef, n, sink);
      known = cbytes, name = "k_lines12";
    } else if (v == 2) {
      hipLaunchKernelGGL((k_lines12<true, 0>), dim3((waves + 7) / 8), dim3(512), kLds, 0, coef, n, sink);
      known = c1_bytes, name = "k_lines12_c1";
    } else if (v == 3) {
      hipLaunchKernelGGL((k_lines12<true, 256>), dim3((waves + 7) / 8), dim3(512), kLds, 0, coef, n, sink);
      known = c1_bytes, name = "k_lines12_c1_slow256";
    } else if (v == 4) {
      hipLaunchKernelGGL((k_lines12<true, 1024>), dim3((waves + 7) / 8), dim3(512), kLds, 0, coef, n, sink);
      known = c1_bytes, name = "k_lines12_c1_slow1024";
    } else {
      hipLaunchKernelGGL(k_desc, dim3((waves + 3) / 4), dim3(256), 0, 0, gran, n, sink);
      known = (uint64_t)n * 160, name = "k_desc";
    }
    (void)hipEventRecord(b);
    if (hipEventSynchronize(b) != hipSuccess) return 2;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%s known_bytes %llu ms %.4f\n", name, (unsigned long long)known, ms);
  }
  (void)hipFree(coef);
  (void)hipFree(gran);
  (void)hipFree(sink);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
