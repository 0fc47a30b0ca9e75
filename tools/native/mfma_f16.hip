// Rates of the MFMA forms a split-f16 ("3 x f16") fp32 conv could use, on every CU with
// 8 waves and 12 independent accumulators per wave, no memory traffic in the loop:
//   v_mfma_f32_16x16x4_f32   (the exact-f32 form the Winograd conv uses today)
//   v_mfma_f32_16x16x16_f16  (K = 16: a lane's A/B fragment = one channel quad)
//   v_mfma_f32_16x16x32_f16  (K = 32)
// plus a check that f16 MFMA keeps subnormal operands (the low halves of small values).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef float w4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

template <int KIND>
__global__ void __launch_bounds__(512) mfma_loop(float* out, int iters, float seed) {
  w4 acc[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = w4{0, 0, 0, 0};
  uint32_t h = (blockIdx.x * 512 + threadIdx.x) * 2654435761u + (uint32_t)seed;
  h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
  float a = (float)(h & 0xFFFFF) * 1e-6f - 0.5f;
  h *= 0x27d4eb2du; h ^= h >> 15;
  float b = (float)(h & 0xFFFFF) * 1e-6f - 0.5f;
  h4 a4 = {(_Float16)a, (_Float16)b, (_Float16)(a * b), (_Float16)(a - b)};
  h4 b4 = {(_Float16)b, (_Float16)a, (_Float16)(a + b), (_Float16)(a * 0.5f)};
  h8 a8 = {a4[0], a4[1], a4[2], a4[3], a4[1], a4[0], a4[3], a4[2]};
  h8 b8 = {b4[0], b4[1], b4[2], b4[3], b4[2], b4[3], b4[0], b4[1]};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      if (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
      if (KIND == 1) acc[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc[i], 0, 0, 0);
      if (KIND == 2) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc[i], 0, 0, 0);
    }
    a = -a; b4 = -b4; b8 = -b8;
  }
  float s = a;
#pragma unroll
  for (int i = 0; i < 12; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

// D = A * B for one 16x16x16 f16 tile; A[r][k] in lane (r + 16 * (k / 4)), element k % 4.
__global__ void mfma_tile(const _Float16* A, const _Float16* B, float* D) {
  const int l = threadIdx.x;
  h4 a, b;
  for (int j = 0; j < 4; ++j) {
    a[j] = A[(l & 15) * 16 + 4 * (l >> 4) + j];
    b[j] = B[(4 * (l >> 4) + j) * 16 + (l & 15)];
  }
  w4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main(int argc, char** argv) {
  int cus = 256, iters = argc > 1 ? atoi(argv[1]) : 4000;
  float* out;
  hipMalloc(&out, sizeof(float) * 512 * cus * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"16x16x4_f32 ", "16x16x16_f16", "16x16x32_f16"};
  const double kk[3] = {4, 16, 32};
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(mfma_loop<0>, dim3(cus), dim3(512), 0, 0, out, iters, 1.0f);
      if (v == 1) hipLaunchKernelGGL(mfma_loop<1>, dim3(cus), dim3(512), 0, 0, out, iters, 1.0f);
      if (v == 2) hipLaunchKernelGGL(mfma_loop<2>, dim3(cus), dim3(512), 0, 0, out, iters, 1.0f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double n_mfma = 12.0 * iters * 8 * cus;
      const double flops = 2.0 * 16 * 16 * kk[v] * n_mfma;
      // cycles per MFMA per SIMD at a nominal 2.4 GHz: 2 waves per SIMD
      const double cyc = ms * 1e-3 * 2.4e9 / (12.0 * iters * 2);
      printf("%s: %.3f ms  %.1f TF/s  %.1f cyc/MFMA/SIMD @2.4GHz\n", names[v], ms, flops / ms / 1e9, cyc);
    }
  }
  // subnormal operands: A = 2^-20 (f16 subnormal), B = 3 -> D = 16 * 3 * 2^-20 per row
  _Float16 hA[256], hB[256];
  for (int i = 0; i < 256; ++i) {
    hA[i] = (_Float16)ldexpf(1.0f + (i % 3), -20 - (i % 4));
    hB[i] = (_Float16)(1.0f + (i % 5) * 0.25f);
  }
  _Float16 *dA, *dB;
  float* dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 1024);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma_tile, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  float hD[256];
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  double maxrel = 0;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      double ref = 0;
      for (int k = 0; k < 16; ++k) ref += (double)(float)hA[r * 16 + k] * (double)(float)hB[k * 16 + c];
      double e = fabs(hD[r * 16 + c] - ref) / fabs(ref);
      if (e > maxrel) maxrel = e;
    }
  printf("subnormal f16 operands: max rel error %.3e (%s)\n", maxrel, maxrel < 1e-6 ? "kept" : "FLUSHED/inexact");
  hipFree(out);
  return 0;
}
