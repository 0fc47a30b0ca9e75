// Timing-only ablation harness for the bf16 DenseLayer conv (conv3_bf16.hip): built once per
// IDF_BF16_ABLATE value (tools/native/Makefile), times config 3's level-0/1/2 widest layers
// (B = 1024) on random data.  Outputs are meaningless for ablate != 0.
#include "../../finalproject-losslessimagecompression_amd/csrc/conv3_bf16.hip"

#include <stdio.h>
#include <stdlib.h>
#include <vector>

template <typename T>
static T* dev_random(size_t n, bool bf) {
  std::vector<T> h(n);
  for (size_t i = 0; i < n; ++i) {
    const float v = ((float)rand() / RAND_MAX - 0.5f) * 0.1f;
    uint32_t u;
    __builtin_memcpy(&u, &v, 4);
    if (bf) {
      const uint16_t hb = (uint16_t)(u >> 16);  // truncation is fine for timing data
      __builtin_memcpy(&h[i], &hb, 2);
    } else {
      __builtin_memcpy(&h[i], &v, 4);
    }
  }
  T* d;
  if (hipMalloc(&d, n * sizeof(T)) != hipSuccess) abort();
  if (hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) abort();
  return d;
}

int main() {
  struct Case { int B, hw, c; } cases[] = {{1024, 32, 496}, {1024, 16, 504}, {1024, 8, 520}};
  const int N = 44, n_alloc = 48;
  for (auto& cs : cases) {
    const int64_t P = (int64_t)cs.B * cs.hw * cs.hw;
    const int ld = (cs.c + N + 15) / 16 * 16, ld16 = (cs.c + N + 63) / 64 * 64;
    const int nslab = (cs.c + 31) / 32;
    float* X = dev_random<float>((size_t)P * ld, false);
    uint16_t* X16 = dev_random<uint16_t>((size_t)P * ld16, true);
    uint16_t* Wb = dev_random<uint16_t>((size_t)nslab * 9 * 4 * n_alloc * 8, true);
    float* b = dev_random<float>(n_alloc * 10, false);
    const int64_t wsn = idf_conv3x3_bf16_workspace(cs.B, cs.hw, cs.hw, cs.c, N);
    float* ws = wsn ? dev_random<float>(wsn, false) : nullptr;
    const int n16 = (cs.c + N + 7) / 8 * 8 - cs.c;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int rep = 0; rep < 6; ++rep) {
      (void)hipEventRecord(e0, 0);
      int rc = idf_conv3x3_bf16(nullptr, cs.B, cs.hw, cs.hw, cs.c, X16, ld16, Wb, n_alloc, b,
                                b + n_alloc, n_alloc, b + 8 * n_alloc, N, X + cs.c, ld,
                                X16 + cs.c, ld16, n16, 0, 0.f, ws, wsn);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      if (rc) { printf("rc=%d\n", rc); return 1; }
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    const double mfma = 2.0 * P * 9 * (nslab * 32.0) * n_alloc;
    printf("ablate=%d hw=%d c=%d: %.1f us  executed-MFMA %.1f TF/s\n", IDF_BF16_ABLATE, cs.hw, cs.c,
           best * 1e3, mfma / best / 1e9);
    (void)hipFree(X); (void)hipFree(X16); (void)hipFree(Wb); (void)hipFree(b);
    if (ws) (void)hipFree(ws);
  }
  return 0;
}
