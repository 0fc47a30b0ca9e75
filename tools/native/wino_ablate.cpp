// Timing-only ablation harness for the Winograd conv kernel: built once per
// IDF_WINO_ABLATE value (tools/native/Makefile), times the imagenet64 level-0 and level-2
// widest layers on random data.  Outputs are meaningless for ablate != 0.
// WINO_SRC: an alternative copy of the kernel source (same-box A/B against a baseline)
#ifdef WINO_SRC
#include WINO_SRC
#else
#include "../../finalproject-losslessimagecompression_amd/csrc/conv3_wino.hip"
#endif

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

// U for the split-f16 (x3) kernel: every float slot holds two small f16 values (random
// float bits reinterpreted as f16 pairs would put NaN / inf in the products and make every
// thread of the epilogue hit the range guard's atomic)
static float* dev_random_f16pairs(size_t n) {
  std::vector<_Float16> h(2 * n);
  for (size_t i = 0; i < 2 * n; ++i) h[i] = (_Float16)(((float)rand() / RAND_MAX - 0.5f) * 0.05f);
  float* d;
  if (hipMalloc(&d, n * 4) != hipSuccess) abort();
  if (hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) abort();
  return d;
}

int main(int argc, char** argv) {
  const bool x3 = argc > 1 && argv[1][0] == 'x';
  uint32_t* flag;
  if (hipMalloc(&flag, 4) != hipSuccess) abort();
  struct Case { int B, hw, c; } cases[] = {{256, 32, 496}, {256, 16, 504}, {256, 8, 520}, {256, 32, 16}};
  const int N = 44, n_alloc = 48;
  for (auto& cs : cases) {
    const int P = cs.B * cs.hw * cs.hw, ld = (cs.c + N + 15) / 16 * 16, nslab = (cs.c + 15) / 16;
    float* X = dev_random((size_t)P * ld);
    float* U = x3 ? dev_random_f16pairs((size_t)16 * nslab * (n_alloc / 16) * 256)
                  : dev_random((size_t)16 * nslab * (n_alloc / 16) * 256);
    float* b = dev_random(n_alloc * 10);
    const int64_t wsn = idf_conv3x3_wino_workspace(cs.B, cs.hw, cs.hw, cs.c, N);
    const int64_t nblk_dbg = (int64_t)cs.B * cs.hw * cs.hw / 64 * 8 * 12 + 4096;
    float* ws = (wsn || IDF_WINO_STAMPS) ? dev_random(wsn > nblk_dbg ? wsn : nblk_dbg) : nullptr;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int rep = 0; rep < 6; ++rep) {
      (void)hipEventRecord(e0, 0);
      int rc = x3 ? idf_conv3x3_wx3(nullptr, cs.B, cs.hw, cs.hw, cs.c, X, ld, (const uint16_t*)U,
                                    n_alloc / 16, 1.0f, b, b + n_alloc, n_alloc, b + 8 * n_alloc, N,
                                    X + cs.c, ld, 1, 0.f, flag, 0, ws, wsn)
                  : idf_conv3x3_wino(nullptr, cs.B, cs.hw, cs.hw, cs.c, X, ld, U, n_alloc / 16, b,
                                     b + n_alloc, n_alloc, b + 8 * n_alloc, N, X + cs.c, ld, 1, 0.f,
                                     ws, wsn);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      if (rc) { printf("rc=%d\n", rc); return 1; }
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    if (IDF_WINO_STAMPS && x3 && wsn == 0) {
      std::vector<float> h((size_t)nblk_dbg);
      (void)hipMemcpy(h.data(), ws, nblk_dbg * 4, hipMemcpyDeviceToHost);
      const int nb = cs.B * cs.hw * cs.hw / 256;
      double sw = 0, si = 0, st = 0, se = 0;
      for (int b = 0; b < nb; ++b)
        for (int w = 0; w < 8; ++w) {
          sw += h[(b * 8 + w) * 4]; si += h[(b * 8 + w) * 4 + 1]; st += h[(b * 8 + w) * 4 + 2];
          se += h[(b * 8 + w) * 4 + 3];
        }
      printf("  stamps (memtime units/wave): loop %.0f  barrier-wait %.0f  prologue %.0f  epilogue %.0f\n",
             st / nb / 8, sw / nb / 8, si / nb / 8, se / nb / 8);
      double ep[8] = {0};
      for (int b = 0; b < nb; ++b)
        for (int w = 0; w < 8; ++w)
          for (int k = 0; k < 7; ++k) ep[k] += h[(size_t)nb * 32 + (b * 8 + w) * 8 + k];
      printf("  epilogue phases: pre %.0f | j0 write+bar %.0f  rest %.0f | j1 %.0f %.0f | j2 %.0f %.0f\n",
             ep[0] / nb / 8, ep[1] / nb / 8, ep[2] / nb / 8, ep[3] / nb / 8, ep[4] / nb / 8,
             ep[5] / nb / 8, ep[6] / nb / 8);
    }
    const double mfma = 2.0 * cs.B * (cs.hw / 2) * (cs.hw / 2) * 16 * (nslab * 16.0) * n_alloc;
    printf("%s ablate=%d hw=%d c=%d: %.1f us  executed-MFMA %.1f TF/s\n", x3 ? "x3 " : "f32", IDF_WINO_ABLATE, cs.hw, cs.c,
           best * 1e3, mfma / best / 1e9);
    (void)hipFree(X); (void)hipFree(U); (void)hipFree(b); if (ws) (void)hipFree(ws);
  }
  return 0;
}
