// Timing-only ablation harness for the wk conv kernel (conv3_wk.hip): built once per
// IDF_WK_ABLATE value (tools/native/Makefile wk_ablate_N), times imagenet64 layer shapes on
// random data.  Outputs are meaningless for ablate != 0.
#include "../../finalproject-losslessimagecompression_amd/csrc/conv3_wk.hip"

#include <stdio.h>
#include <stdlib.h>
#include <vector>

static float* dev_random(size_t n) {
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)rand() / RAND_MAX - 0.5f;
  float* d;
  if (hipMalloc(&d, n * 4) != hipSuccess) abort();
  if (hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) abort();
  return d;
}

static uint16_t* dev_random_f16(size_t n) {
  std::vector<_Float16> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (_Float16)(((float)rand() / RAND_MAX - 0.5f) * 0.05f);
  uint16_t* d;
  if (hipMalloc(&d, n * 2) != hipSuccess) abort();
  if (hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice) != hipSuccess) abort();
  return d;
}

int main(int argc, char** argv) {
  uint32_t* flag;
  if (hipMalloc(&flag, 4) != hipSuccess) abort();
  struct Case { int B, hw, c; } cases[] = {{256, 32, 496}, {256, 32, 12}, {256, 32, 140},
                                           {256, 16, 504}, {256, 8, 520}};
  const int N = 43, n_alloc = 48;
  for (auto& cs : cases) {
    const int P = cs.B * cs.hw * cs.hw, ld = (cs.c + N + 15) / 16 * 16 + 4, nslab = (cs.c + 31) / 32;
    const bool slabm = getenv("WK_SLABMAJOR") != nullptr;
    float* X = dev_random((size_t)P * ld + (slabm ? (size_t)nslab * P * 32 : 0));
    float* XS = X + (size_t)P * ld;  // slab-major copy region (random data; timing only)
    uint16_t* U = dev_random_f16((size_t)16 * nslab * (n_alloc / 16) * 1024);
    float* b = dev_random(n_alloc * 10);
    const int64_t wsn0 = idf_conv3x3_wk_workspace(cs.B, cs.hw, cs.hw, cs.c, N);
    const int64_t nstamp = (int64_t)cs.B * cs.hw * cs.hw / 256 * 64 + 64;
    const int64_t wsn = IDF_WK_STAMPS && wsn0 < nstamp ? nstamp : wsn0;
    float* ws = wsn ? dev_random(wsn) : nullptr;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f, sum = 0;
    for (int rep = 0; rep < 8; ++rep) {
      (void)hipEventRecord(e0, 0);
      int rc = slabm ? idf_conv3x3_wk_slabmajor(nullptr, cs.B, cs.hw, cs.hw, cs.c, XS, (int64_t)P * 32, U,
                                                n_alloc / 16, 1.0f, b, b + n_alloc, n_alloc, b + 8 * n_alloc,
                                                N, X + cs.c, ld, 0, 0.f, flag, 0, ws, wsn)
                     : idf_conv3x3_wk(nullptr, cs.B, cs.hw, cs.hw, cs.c, X, ld, U, n_alloc / 16, 1.0f, b,
                                      b + n_alloc, n_alloc, b + 8 * n_alloc, N, X + cs.c, ld, 0, 0.f, flag, 0,
                                      ws, wsn);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      if (rc) { printf("rc=%d\n", rc); return 1; }
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 2) { sum += ms; if (ms < best) best = ms; }
    }
    if (IDF_WK_STAMPS && wsn0 == 0) {
      std::vector<float> h((size_t)nstamp);
      (void)hipMemcpy(h.data(), ws, nstamp * 4, hipMemcpyDeviceToHost);
      const int nb = cs.B * cs.hw * cs.hw / 256;
      double t[5] = {0, 0, 0, 0, 0};
      for (int b = 0; b < nb; ++b)
        for (int w = 0; w < 8; ++w)
          for (int k = 0; k < 5; ++k) t[k] += h[(b * 8 + w) * 8 + k];
      printf("  stamps (cycles/wave): prologue %.0f (final drain %.0f)  loop %.0f  S-write+barrier %.0f  finish %.0f\n",
             t[0] / nb / 8, t[4] / nb / 8, t[1] / nb / 8, t[2] / nb / 8, t[3] / nb / 8);
    }
    const double fl = 2.0 * P * 9.0 * cs.c * N;
    printf("wk%s ablate=%d hw=%d c=%d: best %.1f us  mean %.1f us  %.1f TF/s algorithmic\n",
           slabm ? "-slab" : "", IDF_WK_ABLATE, cs.hw, cs.c, best * 1e3, sum / 6 * 1e3, fl / best / 1e9);
    (void)hipFree(X); (void)hipFree(U); (void)hipFree(b); if (ws) (void)hipFree(ws);
  }
  return 0;
}
