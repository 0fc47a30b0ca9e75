#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float w4 __attribute__((ext_vector_type(4)));
__global__ void k(const float* A, const float* B, float* D) {
  int l = threadIdx.x; h8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)A[l*8+j]; b[j] = (_Float16)B[l*8+j]; }
  w4 c = {0,0,0,0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l*4+r] = c[r];
}
int main() {
  float hA[512], hB[512], hD[256];
  srand(1);
  for (int i = 0; i < 512; ++i) { hA[i] = (float)(rand() % 7 - 3); hB[i] = (float)(rand() % 7 - 3); }
  float *dA, *dB, *dD; hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dD, 1024);
  hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  // hypotheses for k(l, j)
  for (int h = 0; h < 3; ++h) {
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r4 = 0; r4 < 4; ++r4) {
      int row = 4 * (l >> 4) + r4, col = l & 15;
      double ref = 0;
      for (int kk = 0; kk < 32; ++kk) {
        // find A element with row, k = kk and B element with col, k = kk
        double a = 0, b = 0;
        for (int la = 0; la < 64; ++la) for (int j = 0; j < 8; ++j) {
          int g = la >> 4, kA;
          if (h == 0) kA = 8 * g + j;
          else if (h == 1) kA = 4 * g + (j & 3) + 16 * (j >> 2);
          else kA = 2 * g + (j & 1) + 8 * (j >> 1);
          if (kA != kk) continue;
          if ((la & 15) == row) a = hA[la*8+j];
          if ((la & 15) == col) b = hB[la*8+j];
        }
        ref += a * b;
      }
      if (ref != hD[l*4+r4]) ++bad;
    }
    printf("hypothesis %d: %d mismatches\n", h, bad);
  }
  return 0;
}
