// Probe: does an LDS-DMA (buffer_load ... lds) of a workgroup whose LDS allocation does not start
// at the CU's LDS address 0 land in its own allocation?  Kernel A (small LDS, many blocks)
// fills its LDS with a per-block pattern, waits ~2 ms and checks it; kernel B (128 KiB LDS),
// launched on a second stream while A's blocks hold the low LDS of every CU, DMAs 1-KiB pieces
// of a known buffer into its whole LDS and checks what it reads back.
// Build: hipcc --offload-arch=gfx950 -O2 tools/lds_cores_probe.hip -o tools/ab_lib/lds_cores_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(64) small_lds(uint32_t* bad, long long spin) {
  __shared__ uint32_t lds[1024];  // 4 KiB
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = 0xA5000000u ^ (blockIdx.x * 1024u + i);
  __syncthreads();
  const long long t0 = clock64();
  while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(10);
  int nb = 0;
  for (int i = lane; i < 1024; i += 64) nb += lds[i] != (0xA5000000u ^ (blockIdx.x * 1024u + i));
  if (nb) atomicAdd(bad, (uint32_t)nb);
}

constexpr int kBigBytes = 128 * 1024;

__global__ void __launch_bounds__(64) big_dma(const uint32_t* src, uint32_t* bad, int reps) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kBigBytes / 4];
  const int lane = threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, kBigBytes, 0x00020000);
  int nb = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int i = lane; i < kBigBytes / 4; i += 64) lds[i] = 0;
    __syncthreads();
    for (int p = 0; p < kBigBytes / 1024; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          r, (__attribute__((address_space(3))) void*)(lds + p * 256), 16,
          (uint32_t)(p * 1024 + lane * 16), 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = lane; i < kBigBytes / 4; i += 64) nb += lds[i] != src[i];
    __syncthreads();
  }
  if (nb) atomicAdd(bad + 1, (uint32_t)nb);
}

int main() {
  uint32_t *src, *bad;
  if (hipMalloc(&src, kBigBytes) != hipSuccess || hipMalloc(&bad, 8) != hipSuccess) return 1;
  static uint32_t h[kBigBytes / 4];
  for (int i = 0; i < kBigBytes / 4; ++i) h[i] = 0x3C000000u + i;
  if (hipMemcpy(src, h, kBigBytes, hipMemcpyHostToDevice) != hipSuccess) return 1;
  if (hipMemset(bad, 0, 8) != hipSuccess) return 1;
  hipStream_t s1, s2;
  if (hipStreamCreateWithFlags(&s1, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) return 1;
  // ~2 ms at ~2 GHz clock64; 256 CUs x 8 blocks of 4 KiB: the low 32 KiB of every CU
  hipLaunchKernelGGL(small_lds, dim3(256 * 8), dim3(64), 0, s1, bad, 4000000LL);
  hipLaunchKernelGGL(big_dma, dim3(256), dim3(64), 0, s2, src, bad, 50);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  uint32_t o[2];
  if (hipMemcpy(o, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("small-LDS blocks: corrupted words %u; big DMA blocks: wrong words read back %u\n", o[0], o[1]);
  return 0;
}
