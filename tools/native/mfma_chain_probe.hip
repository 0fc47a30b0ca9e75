#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float w4 __attribute__((ext_vector_type(4)));
// per lane: H[4], L[4] (A: tile l&15, channels 4g+j), UH[4], UL[4] (B: channel 4g+j, n = l&15)
template <int ORDER>
__global__ void k(const float* H, const float* L, const float* UH, const float* UL, float* D) {
  int l = threadIdx.x;
  h4 h, lo, uh, ul;
  for (int j = 0; j < 4; ++j) { h[j] = (_Float16)H[l*4+j]; lo[j] = (_Float16)L[l*4+j]; uh[j] = (_Float16)UH[l*4+j]; ul[j] = (_Float16)UL[l*4+j]; }
  h8 a = __builtin_shufflevector(h, h, 0,1,2,3,0,1,2,3);
  h8 b = __builtin_shufflevector(uh, ul, 0,1,2,3,4,5,6,7);
  w4 c = {0,0,0,0};
  if (ORDER == 0) {
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(lo, uh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  } else if (ORDER == 1) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(lo, uh, c, 0, 0, 0);
  } else {
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(lo, uh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(h, uh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(h, ul, c, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[l*4+r] = c[r];
}
int main() {
  float hH[256], hL[256], hUH[256], hUL[256], hD[256];
  srand(2);
  for (int i = 0; i < 256; ++i) { hH[i] = rand()%9-4; hL[i] = (rand()%9-4)/1024.0f; hUH[i] = rand()%9-4; hUL[i] = (rand()%9-4)/2048.0f; }
  float *d[5]; for (int i = 0; i < 5; ++i) hipMalloc(&d[i], 1024);
  hipMemcpy(d[0], hH, 1024, hipMemcpyHostToDevice); hipMemcpy(d[1], hL, 1024, hipMemcpyHostToDevice);
  hipMemcpy(d[2], hUH, 1024, hipMemcpyHostToDevice); hipMemcpy(d[3], hUL, 1024, hipMemcpyHostToDevice);
  for (int o = 0; o < 3; ++o) {
    if (o == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, d[0], d[1], d[2], d[3], d[4]);
    if (o == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, d[0], d[1], d[2], d[3], d[4]);
    if (o == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, d[0], d[1], d[2], d[3], d[4]);
    hipMemcpy(hD, d[4], 1024, hipMemcpyDeviceToHost);
    double maxe = 0;
    for (int l = 0; l < 64; ++l) for (int r4 = 0; r4 < 4; ++r4) {
      int row = 4*(l>>4)+r4, col = l&15; double ref = 0;
      for (int ch = 0; ch < 16; ++ch) {  // channel ch = 4g + j lives in lanes with l>>4 == ch/4
        int g = ch >> 2, j = ch & 3;
        int la = 16*g + row, lb = 16*g + col;
        ref += (double)hL[la*4+j]*hUH[lb*4+j] + (double)hH[la*4+j]*hUH[lb*4+j] + (double)hH[la*4+j]*hUL[lb*4+j];
      }
      double e = fabs(ref - hD[l*4+r4]); if (e > maxe) maxe = e;
    }
    printf("order %d: max abs error %.3e\n", o, maxe);
  }
  return 0;
}
