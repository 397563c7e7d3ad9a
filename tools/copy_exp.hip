// copy_exp.hip -- the pipelined drop-in's PCM copy-out (mp3g_decode_streams_into):
// one group's PCM (302 MB at c3), device -> pinned host, four ways, timed with
// host clocks (run it WITHOUT a profiler too: under rocprofv3 HIP picked a
// different engine for the same hipMemcpyAsync):
//   memcpy      hipMemcpyAsync on a non-blocking stream (the runtime picks
//               SDMA or a blit kernel)
//   memcpy+up   the same while a host -> device copy runs on another stream
//   kernel/N    a copy kernel of our own (16 B per lane, non-temporal stores
//               into the pinned buffer) on a stream limited to N CUs
// into host memory from hipHostMalloc with the default flags, hipHostMalloc
// non-coherent, and hipHostRegister of page-aligned malloc memory.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) copy_out(const u4* __restrict__ src, u4* __restrict__ dst, size_t n16) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(src[i], &dst[i]);
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                        \
    }                                                                  \
  } while (0)

static hipStream_t masked(int want, int ncu) {
  hipStream_t s = nullptr;
  if (want <= 0 || want >= ncu) {
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    return s;
  }
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int i = 0; i < want; i++) {
    const int cu = (int)((long)i * ncu / want);
    mask[cu / 32] |= 1u << (cu % 32);
  }
  (void)hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  return s;
}

int main() {
  const size_t bytes = 302u << 20, in_bytes = 60u << 20;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  void *d, *din, *hin;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&din, in_bytes));
  CK(hipMemset(d, 1, bytes));
  CK(hipHostMalloc(&hin, in_bytes, hipHostMallocDefault));
  void* hosts[3] = {};
  const char* hname[3] = {"hostmalloc-default", "hostmalloc-noncoherent", "hostregister"};
  CK(hipHostMalloc(&hosts[0], bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&hosts[1], bytes, hipHostMallocNonCoherent));
  hosts[2] = std::aligned_alloc(4096, bytes);
  CK(hipHostRegister(hosts[2], bytes, hipHostRegisterDefault));
  hipStream_t s2, s3;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  const int cus[4] = {0, 16, 32, 64};
  hipStream_t ks[4];
  for (int i = 0; i < 4; i++) ks[i] = masked(cus[i], ncu);
  for (int hk = 0; hk < 3; hk++) {
    void* h = hosts[hk];
    void* hd = nullptr;  // the device view of the pinned buffer
    CK(hipHostGetDevicePointer(&hd, h, 0));
    for (int rep = 0; rep < 3; rep++) {
      for (int c = 0; c < 6; c++) {
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        char name[64];
        if (c == 0) {
          std::snprintf(name, sizeof name, "memcpy");
          CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s2));
        } else if (c == 1) {
          std::snprintf(name, sizeof name, "memcpy+up");
          CK(hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, s3));
          CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s2));
        } else {
          const int i = c - 2;
          std::snprintf(name, sizeof name, "kernel/%d", cus[i] ? cus[i] : ncu);
          const int blocks = 8 * (cus[i] ? cus[i] : ncu);
          hipLaunchKernelGGL(copy_out, dim3(blocks), dim3(256), 0, ks[i], static_cast<const u4*>(d),
                             static_cast<u4*>(hd), bytes / 16);
          CK(hipGetLastError());
        }
        CK(hipDeviceSynchronize());
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (rep > 0) std::printf("%-24s %-12s %8.3f ms %6.1f GB/s\n", hname[hk], name, ms, bytes / ms / 1e6);
      }
    }
    if (std::memcmp(static_cast<char*>(h) + bytes - 64, static_cast<char*>(h), 64) != 0) std::printf("content?\n");
  }
  return 0;
}
