// tests/native/expf_check.cpp -- exhaustive host check that the restated glibc
// expf of csrc/idf_cdf.h equals the host libm expf (the function the reference
// coder calls, rans.pyx:6-9) on every one of the 2^32 float bit patterns.
// Also prints an order-independent checksum of libm expf over all inputs that
// the GPU test compares the device build against.
//   g++ -O2 -ffp-contract=off -fopenmp -I<csrc> expf_check.cpp -o expf_check
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <cstring>
#include "idf_cdf.h"

int main(int argc, char **argv) {
  uint64_t lo = 0, hi = 1ull << 32;
  if (argc >= 3) { lo = strtoull(argv[1], 0, 0); hi = strtoull(argv[2], 0, 0); }
  unsigned long long mism = 0, sum = 0;
#pragma omp parallel for reduction(+ : mism, sum) schedule(static, 1 << 20)
  for (long long i = (long long)lo; i < (long long)hi; ++i) {
    float x = idf::u2f((uint32_t)i);
    float a = expf(x);
    float b = idf::expf_glibc(x);
    uint32_t ua = idf::f2u(a), ub = idf::f2u(b);
    bool both_nan = (a != a) && (b != b);
    if (ua != ub && !both_nan) ++mism;
    // checksum: NaNs canonicalised so payload differences do not matter
    uint32_t h = (a != a) ? 0x7fc00000u : ua;
    sum += (unsigned long long)h * ((uint64_t)i * 2654435761ull | 1ull);
  }
  printf("range [%llu, %llu) mismatches=%llu checksum=%llu\n", (unsigned long long)lo,
         (unsigned long long)hi, mism, sum);
  return mism ? 1 : 0;
}
