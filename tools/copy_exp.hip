// copy_exp.hip -- which engine HIP picks for the pipelined drop-in's PCM
// copy-out (mp3g_decode_streams_into): a device -> pinned-host copy of one
// group's PCM (302 MB at c3) issued
//   A  alone on its stream
//   B  on its own stream after hipStreamWaitEvent on a kernel of another stream
//   C  as B, with a host -> device copy on a third stream at the same time
//   D  on the stream of the kernel it follows (no cross-stream wait)
// Run under rocprofv3 --kernel-trace --memory-copy-trace: an SDMA copy is a
// memory-copy record, a blit is an __amd_rocclr_copyBuffer kernel (which
// takes CUs from the decode kernels).  Prints each case's wall time.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void touch(uint32_t* p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] += 1u;
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  const size_t bytes = 302u << 20, in_bytes = 60u << 20;
  void *d, *h, *din, *hin;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&din, in_bytes));
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&hin, in_bytes, hipHostMallocDefault));
  hipStream_t s1, s2, s3;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int rep = 0; rep < 2; rep++) {
    for (char c : {'A', 'B', 'C', 'D'}) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      if (c == 'A') {
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s2));
      } else if (c == 'D') {
        hipLaunchKernelGGL(touch, dim3(1024), dim3(256), 0, s1, static_cast<uint32_t*>(d), (size_t)1 << 20);
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s1));
      } else {
        hipLaunchKernelGGL(touch, dim3(1024), dim3(256), 0, s1, static_cast<uint32_t*>(d), (size_t)1 << 20);
        CK(hipEventRecord(ev, s1));
        CK(hipStreamWaitEvent(s2, ev, 0));
        CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s2));
        if (c == 'C') CK(hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, s3));
      }
      CK(hipDeviceSynchronize());
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      std::printf("rep %d case %c: %.3f ms (%.1f GB/s for the D2H bytes)\n", rep, c, ms, bytes / ms / 1e6);
    }
  }
  return 0;
}
