// Achievable f32 MFMA rate on this chip: every CU, 8 waves, 16 independent
// v_mfma_f32_16x16x4_f32 accumulators per wave, no memory traffic in the loop.
// Also a variant with VALU adds interleaved (the Winograd input-transform mix).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float w4 __attribute__((ext_vector_type(4)));

template <int VALU>
__global__ void __launch_bounds__(512) mfma_loop(float* out, int iters, float seed) {
  w4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = w4{0, 0, 0, 0};
  // random-looking operands (power, hence clock, depends on the operand bits)
  uint32_t h = (blockIdx.x * 512 + threadIdx.x) * 2654435761u + (uint32_t)seed;
  h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
  float a = (float)(h & 0xFFFFF) * 1e-6f - 0.5f;
  h *= 0x27d4eb2du; h ^= h >> 15;
  float b = (float)(h & 0xFFFFF) * 1e-6f - 0.5f;
  float x0 = a, x1 = b, x2 = a + 1, x3 = b + 1;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
      if (VALU && (i & 1)) { x0 = x0 + x1; x1 = x1 - x2; x2 = x2 + x3; }
    }
    a = a + x0 * 1e-30f;
    b = -b;
  }
  float s = x0 + x1 + x2 + x3;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  int cus = 256, iters = argc > 1 ? atoi(argv[1]) : 4000;
  float* out;
  hipMalloc(&out, sizeof(float) * 512 * cus * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(mfma_loop<0>, dim3(cus), dim3(512), 0, 0, out, iters, 1.0f);
      else hipLaunchKernelGGL(mfma_loop<1>, dim3(cus), dim3(512), 0, 0, out, iters, 1.0f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double flops = 2.0 * 16 * 16 * 4 * 16.0 * iters * 8 * cus;
      printf("valu=%d blocks=%d: %.3f ms  %.1f TF/s\n", v, cus, ms, flops / ms / 1e9);
    }
  }
  hipFree(out);
  return 0;
}
