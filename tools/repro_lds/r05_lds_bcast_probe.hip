// Probe: do wave-uniform (broadcast) ds_read_b128 of one workgroup return wrong data while
// another workgroup on the same CU runs LDS-DMA (buffer_load ... lds) and / or MFMA?
// Kernel A (4 KiB LDS table, 8 blocks a CU) re-reads its table with uniform-address b128 reads
// and counts words that differ from the pattern; kernel B (120 KiB LDS, one block a CU) runs
// a DMA loop (mode & 1) and an MFMA loop (mode & 2), launched while A's blocks are resident.
// Build: hipcc --offload-arch=gfx950 -O2 tools/lds_bcast_probe.hip -o tools/ab_lib/lds_bcast_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t pat(uint32_t i) { return 0x3F800000u + i * 2654435761u % 4096u; }

__global__ void __launch_bounds__(256) reader(uint32_t* bad, int iters) {
  __shared__ __attribute__((aligned(16))) uint32_t t[1024];
  for (int i = threadIdx.x; i < 1024; i += 256) t[i] = pat(i);
  __syncthreads();
  uint32_t nb = 0, lanes = 0;
  for (int it = 0; it < iters; ++it) {
    const int base = __builtin_amdgcn_readfirstlane((it * 4) & 1023);
    asm volatile("" ::: "memory");
    const uint4 v = *(const uint4*)(t + base);
    const uint32_t m = (v.x != pat(base)) + (v.y != pat(base + 1)) + (v.z != pat(base + 2)) +
                       (v.w != pat(base + 3));
    nb += m;
    lanes |= m ? 1u : 0u;
  }
  if (nb) {
    atomicAdd(bad, nb);
    atomicAdd(bad + 1, 1u);  // lanes that saw a wrong word
  }
}

constexpr int kBig = 120 * 1024;

__global__ void __launch_bounds__(256) other(const uint32_t* src, int mode, int reps, float* sink) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kBig / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, kBig, 0x00020000);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  h8 a, b;
  for (int k = 0; k < 8; ++k) {
    a[k] = (_Float16)(0.001f * (lane + k));
    b[k] = (_Float16)(0.002f * (lane - k));
  }
  for (int rep = 0; rep < reps; ++rep) {
    if (mode & 1) {
      for (int p = wave; p < kBig / 1024; p += 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(lds + p * 256), 16,
            (uint32_t)(p * 1024 + lane * 16), 0, 0, 0);
    }
    if (mode & 2) {
      for (int k = 0; k < 64; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (acc[0] == 12345.0f) sink[0] = acc[1] + (float)lds[lane];
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 3;
  uint32_t *src, *bad;
  float* sink;
  if (hipMalloc(&src, kBig) != hipSuccess || hipMalloc(&bad, 8) != hipSuccess ||
      hipMalloc(&sink, 16) != hipSuccess)
    return 1;
  if (hipMemset(src, 0x5A, kBig) != hipSuccess || hipMemset(bad, 0, 8) != hipSuccess) return 1;
  hipStream_t s1, s2;
  if (hipStreamCreateWithFlags(&s1, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess)
    return 1;
  for (int round = 0; round < 4; ++round) {
    hipLaunchKernelGGL(reader, dim3(256 * 8), dim3(256), 0, s1, bad, 200000);
    if (mode) hipLaunchKernelGGL(other, dim3(256), dim3(256), 0, s2, src, mode, 2000, sink);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  uint32_t o[2];
  if (hipMemcpy(o, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("mode %d (1 DMA, 2 MFMA): wrong words %u, lanes that saw one %u\n", mode, o[0], o[1]);
  return 0;
}
