// Timing harness for the rANS kernels (built per IDF_DECODE_STAMPS by tools/native/Makefile):
// 256 streams x N symbols of quantized logistic samples, encoded on the device, then the
// decode timed and checked for a bit-exact round trip.
#ifdef RANS_SRC  // same-box A/B against a saved copy of the kernel source (ab/, untracked)
#include RANS_SRC
#else
#include "../../finalproject-losslessimagecompression_amd/csrc/rans_kernels.hip"
#endif

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CKH(x) do { if ((x) != hipSuccess) { printf("hip error line %d\n", __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int S = 256;
  const int N = argc > 1 ? atoi(argv[1]) : 3072;
  const int64_t n = (int64_t)S * N;
  std::vector<float> x(n), mean(n), scale(n);
  srand(1);
  for (int64_t i = 0; i < n; ++i) {
    mean[i] = ((float)rand() / RAND_MAX - 0.5f) * 4.0f;
    scale[i] = 0.01f + (float)rand() / RAND_MAX * 0.5f;
    float u = ((float)rand() + 1.0f) / ((float)RAND_MAX + 2.0f);
    float v = mean[i] + scale[i] * logf(u / (1.0f - u));
    // inside the coder's window [lower + 1, lower + 2046] (an out-of-window symbol does not
    // round-trip in the reference either, and corrupts the rest of its stream)
    const float lo = roundf(mean[i] * 256.0f - 1024.0f);
    x[i] = fminf(fmaxf(roundf(v * 256.0f), lo + 1.0f), lo + 2046.0f) / 256.0f;
  }
  std::vector<int64_t> off(S + 1);
  for (int k = 0; k <= S; ++k) off[k] = (int64_t)k * N;
  float *dx, *dm, *ds, *dout;
  int64_t *doff, *dnw, *dwoff;
  uint64_t *dinit, *dfin, *dfin2;
  uint32_t* dw;
  int32_t *dst, *dst2;
  void* ws;
  const int64_t wsb = idf_rans_encode_workspace_bytes(n);
  CKH(hipMalloc(&dx, n * 4)); CKH(hipMalloc(&dm, n * 4)); CKH(hipMalloc(&ds, n * 4));
  CKH(hipMalloc(&dout, n * 4)); CKH(hipMalloc(&doff, (S + 1) * 8)); CKH(hipMalloc(&dnw, S * 8));
  CKH(hipMalloc(&dwoff, S * 8)); CKH(hipMalloc(&dinit, S * 8)); CKH(hipMalloc(&dfin, S * 8));
  CKH(hipMalloc(&dfin2, S * 8)); CKH(hipMalloc(&dw, n * 4)); CKH(hipMalloc(&dst, S * 4));
  CKH(hipMalloc(&dst2, S * 4)); CKH(hipMalloc(&ws, wsb));
  void* dws;
  CKH(hipMalloc(&dws, idf_rans_decode_workspace_bytes(n)));
  CKH(hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(dm, mean.data(), n * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(ds, scale.data(), n * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(doff, off.data(), (S + 1) * 8, hipMemcpyHostToDevice));
  std::vector<uint64_t> init(S, 0x100000000ull);
  CKH(hipMemcpy(dinit, init.data(), S * 8, hipMemcpyHostToDevice));
  if (idf_rans_encode_streams(nullptr, S, n, doff, dx, dm, ds, dinit, dfin, dw, dnw, dst, ws, wsb)) return 1;
  CKH(hipMemcpy(dwoff, off.data(), S * 8, hipMemcpyHostToDevice));  // words live at sym_off
  hipEvent_t e0, e1;
  CKH(hipEventCreate(&e0)); CKH(hipEventCreate(&e1));
  float best = 1e9f, enc_best = 1e9f;
  for (int rep = 0; rep < 5; ++rep) {
    CKH(hipEventRecord(e0, 0));
    if (idf_rans_encode_streams(nullptr, S, n, doff, dx, dm, ds, dinit, dfin, dw, dnw, dst, ws, wsb)) return 1;
    CKH(hipEventRecord(e1, 0));
    CKH(hipEventSynchronize(e1));
    float ms;
    CKH(hipEventElapsedTime(&ms, e0, e1));
    if (ms < enc_best) enc_best = ms;
    CKH(hipEventRecord(e0, 0));
    if (idf_rans_decode_streams(nullptr, S, n, doff, dwoff, dnw, dw, dm, ds, dfin, dfin2, dout, dst2, dws,
                                idf_rans_decode_workspace_bytes(n))) return 1;
    CKH(hipEventRecord(e1, 0));
    CKH(hipEventSynchronize(e1));
    CKH(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  std::vector<float> out(n);
  CKH(hipMemcpy(out.data(), dout, n * 4, hipMemcpyDeviceToHost));
  int64_t bad = 0;
  for (int64_t i = 0; i < n; ++i) bad += out[i] != x[i];
#if IDF_DECODE_STAMPS
  static unsigned long long st[256][6];
  CKH(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamp), sizeof(st)));
  double acc[6] = {0};
  for (int i = 100; i < 200; ++i) {
    for (int j = 1; j < 6; ++j) acc[j] += (double)(st[i][j] - st[i][j - 1]);
    acc[0] += (double)(st[i + 1][0] - st[i][5]);
  }
  printf("stamps (memtime ticks, mean of symbols 100..199): renorm %.0f  ballot %.0f  cdf %.0f  "
         "pick %.0f  update %.0f  to-next %.0f\n", acc[1] / 100, acc[2] / 100, acc[3] / 100,
         acc[4] / 100, acc[5] / 100, acc[0] / 100);
#endif
  printf("mode=%d streams=%d syms/stream=%d: encode %.3f ms (%.1f ns/sym)  decode %.3f ms (%.1f ns/sym)  mismatches=%lld\n",
         IDF_DECODE_STAMPS, S, N, enc_best, enc_best * 1e6 / N, best, best * 1e6 / N, (long long)bad);
  return 0;
}
