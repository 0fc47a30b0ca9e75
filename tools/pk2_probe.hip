#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* in, float* out) {
  const int l = threadIdx.x;
  f2 w = {in[l], in[64 + l]}, c = {in[128 + l], in[192 + l]};
  const float x = in[256 + l];
  f2 p = __builtin_elementwise_fma(w, f2{x, x}, c);
  float a = w[0], b = w[1], c0 = c[0], c1 = c[1], xx = x;
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c0), "+v"(c1), "+v"(xx));
  float s0 = __builtin_fmaf(a, xx, c0);
  asm volatile("" : "+v"(s0));
  float s1 = __builtin_fmaf(b, xx, c1);
  out[l] = p[0]; out[64 + l] = p[1]; out[128 + l] = s0; out[192 + l] = s1;
}
int main() {
  float h[320], o[256], *di, *dout;
  for (int i = 0; i < 320; ++i) h[i] = 1.0f + 0.37f * ((i * 7919) % 101) / 101.0f - (i % 3 == 0 ? 0.9f : 0.f);
  if (hipMalloc(&di, 320 * 4) || hipMalloc(&dout, 256 * 4)) return 1;
  if (hipMemcpy(di, h, 1280, hipMemcpyHostToDevice)) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout);
  if (hipMemcpy(o, dout, 1024, hipMemcpyDeviceToHost)) return 2;
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    double e0 = (double)h[l] * h[256 + l] + h[128 + l], e1 = (double)h[64 + l] * h[256 + l] + h[192 + l];
    if (o[l] != o[128 + l] || o[64 + l] != o[192 + l]) {
      if (bad < 4) printf("lane %d pk %.9g %.9g scalar %.9g %.9g exact %.9g %.9g\n", l, o[l], o[64 + l], o[128 + l], o[192 + l], e0, e1);
      ++bad;
    }
  }
  printf("lanes where packed != scalar: %d of 64\n", bad);
  return 0;
}
