// Probe: what a buffer_load ... lds whose offset fails the descriptor's range check leaves in
// LDS (zeros, or the bytes that were there).  One wave: LDS filled with 0xDEADBEEF, then one
// 1-KiB piece in range and one past the buffer's end (the dx3 kernel's kDxOff halo slots).
// Build: hipcc --offload-arch=gfx950 -O2 tools/lds_oob_probe.hip -o tools/ab_lib/lds_oob_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(64) probe(const float* src, int nbytes, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[512];
  const int lane = threadIdx.x;
  for (int i = lane; i < 512; i += 64) lds[i] = 0xDEADBEEFu;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nbytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           (uint32_t)lane * 16u, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + 256), 16,
                                           0x80000000u + (uint32_t)lane * 16u, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 512; i += 64) out[i] = lds[i];
}

int main() {
  float* src;
  uint32_t* out;
  if (hipMalloc(&src, 4096) != hipSuccess || hipMalloc(&out, 2048) != hipSuccess) return 1;
  float h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 1.0f + i;
  hipMemcpy(src, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, 4096, out);
  uint32_t o[512];
  if (hipMemcpy(o, out, 2048, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int in_ok = 0, oob_zero = 0, oob_stale = 0;
  for (int i = 0; i < 256; ++i) in_ok += o[i] == __builtin_bit_cast(uint32_t, h[i]);
  for (int i = 256; i < 512; ++i) {
    oob_zero += o[i] == 0u;
    oob_stale += o[i] == 0xDEADBEEFu;
  }
  printf("in-range words correct %d/256; out-of-range piece: zero %d, untouched %d, other %d\n",
         in_ok, oob_zero, oob_stale, 256 - oob_zero - oob_stale);
  return 0;
}
