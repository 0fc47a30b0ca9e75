// Probe: the per-launch cost of a one-round kernel (256 blocks x 512 threads, 150 KiB LDS each,
// one block per CU like dx3) as a function of the bytes it stores -- does the dispatch's
// duration beyond its blocks' own span grow with the data left dirty in L2 (an end-of-kernel
// write-back), and do back-to-back launches hide it?  Times 20 back-to-back launches per size
// with HIP events, plain stream launches and the same 20 captured in a hipGraph.
// Build: hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o tools/ab_lib/launch_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512, 1) store_kernel(f4* out, int64_t n4, int spin) {
  __shared__ f4 lds[150 * 1024 / 16];
  lds[threadIdx.x] = f4{1.f, 2.f, 3.f, 4.f};
  __syncthreads();
  f4 v = lds[(threadIdx.x + 1) & 511];
  for (int i = 0; i < spin; ++i) v = v * 1.0001f + 0.5f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) out[i] = v;
}

#define CK(x)                                                       \
  do {                                                              \
    if ((x) != hipSuccess) {                                        \
      printf("HIP error %s at line %d\n", #x, __LINE__);            \
      return 1;                                                     \
    }                                                               \
  } while (0)

int main() {
  const int64_t maxb = 128ll << 20;
  f4* buf;
  CK(hipMalloc(&buf, maxb));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int64_t sizes[] = {0, 4ll << 20, 16ll << 20, 48ll << 20, 96ll << 20};
  const int spins[] = {0, 4000};
  for (int spin : spins) {
    for (int64_t bytes : sizes) {
      const int64_t n4 = bytes / 16;
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(store_kernel, dim3(256), dim3(512), 0, s, buf, n4, spin);
      CK(hipStreamSynchronize(s));
      float ms1 = 0.f, msg = 0.f;
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(store_kernel, dim3(256), dim3(512), 0, s, buf, n4, spin);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms1, e0, e1));
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(store_kernel, dim3(256), dim3(512), 0, s, buf, n4, spin);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&msg, e0, e1));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      printf("spin %5d  stores %4lld MiB: stream %8.2f us/launch  graph %8.2f us/launch  (%.2f TB/s at stream)\n",
             spin, (long long)(bytes >> 20), 1000.f * ms1 / 20, 1000.f * msg / 20,
             bytes ? bytes / (1e6 * ms1 / 20) / 1e3 : 0.0);
    }
  }
  return 0;
}
