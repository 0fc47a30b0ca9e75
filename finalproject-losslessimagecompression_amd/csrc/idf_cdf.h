// idf_cdf.h -- bit-exact discretised-logistic CDF of the reference rANS coder,
// usable from host and device code (gfx950).
//
// Restates, bit for bit:
//   * glibc 2.35 expf, x86-64 FMA ifunc variant (the function the reference's
//     `exp(float)` resolves to: rans.pyx:6-9,25-26). Every
//     mul+add of glibc's e_expf.c is an explicit fma here; the file is compiled
//     with -ffp-contract=off so nothing else is contracted.
//   * CDF(x, mean, scale, lower) of rans.pyx:31-35 with the exact float/double
//     mix of the generated rans.cpp:1395-1484.
//   * the window origin `lower` of rans.pyx:51 (encode) and rans.pyx:91-93 (decode).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define IDF_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define IDF_HD static inline
#endif

#pragma clang fp contract(off)

namespace idf {

// glibc e_exp2f_data.c: T[i] = asuint64(2^(i/32)) - (i << 47)
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint64_t kExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};

IDF_HD uint32_t f2u(float f) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(uint32_t, f);
#else
  uint32_t u; memcpy(&u, &f, 4); return u;
#endif
}
IDF_HD uint64_t d2u(double d) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(uint64_t, d);
#else
  uint64_t u; memcpy(&u, &d, 8); return u;
#endif
}
IDF_HD double u2d(uint64_t u) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(double, u);
#else
  double d; memcpy(&d, &u, 8); return d;
#endif
}
IDF_HD float u2f(uint32_t u) {
#if defined(__HIPCC__)
  return __builtin_bit_cast(float, u);
#else
  float f; memcpy(&f, &u, 4); return f;
#endif
}

IDF_HD double fma_d(double a, double b, double c) {
#if defined(__HIPCC__)
  return __builtin_fma(a, b, c);
#else
  return fma(a, b, c);
#endif
}

// glibc 2.35 sysdeps/ieee754/flt-32/e_expf.c (EXP2F_TABLE_BITS = 5, poly order 3),
// as compiled with FMA contraction (x86-64 ifunc __expf_fma).
IDF_HD float expf_glibc(float x, const uint64_t* tab = kExp2fTab) {
  const double InvLn2N = 0x1.71547652b82fep+0 * 32;
  const double SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / (32.0 * 32.0 * 32.0);
  const double C1 = 0x1.ebfce50fac4f3p-3 / (32.0 * 32.0);
  const double C2 = 0x1.62e42ff0c52d6p-1 / 32.0;
  uint32_t ux = f2u(x);
  uint32_t abstop = (ux >> 20) & 0x7ff;
  if (abstop >= ((f2u(88.0f) >> 20) & 0x7ff)) {
    if (ux == f2u(-__builtin_inff())) return 0.0f;
    if (abstop >= ((f2u(__builtin_inff()) >> 20) & 0x7ff)) return x + x;
    if (x > 0x1.62e42ep6f) return __builtin_inff();   // __math_oflowf
    if (x < -0x1.9fe368p6f) return 0.0f;              // __math_uflowf
  }
  double xd = (double)x;
  double kd = fma_d(InvLn2N, xd, SHIFT);
  uint64_t ki = d2u(kd);
  kd -= SHIFT;
  double r = fma_d(InvLn2N, xd, -kd);
  uint64_t t = tab[ki % 32];
  t += ki << 47;
  double s = u2d(t);
  double z = fma_d(C0, r, C1);
  double r2 = r * r;
  double y = fma_d(C2, r, 1.0);
  y = fma_d(z, r2, y);
  y = y * s;
  return (float)y;
}

IDF_HD double round_d(double v) {
#if defined(__HIPCC__)
  return __builtin_round(v);
#else
  return round(v);
#endif
}
IDF_HD float round_f(float v) {
#if defined(__HIPCC__)
  return __builtin_roundf(v);
#else
  return roundf(v);
#endif
}

// rans.pyx:31-35 (rans.cpp:1418-1449). Returns part1 + part2.
// Caller guarantees scale != 0 (the reference raises ZeroDivisionError).
// tab: the 2^(j/32) table; device hot loops pass a copy in LDS (kExp2fTab itself is a
// constant-memory load per lookup, a long latency inside a serial decode chain).
IDF_HD int rans_cdf(float x, float mean, float scale, float lower,
                    const uint64_t* tab = kExp2fTab) {
  float d = x - lower;                                        // f32 subtraction
  int part2 = (int)round_d((double)d * 256.0) + 1;            // libm round (double)
  double t = ((double)x + 0.001953125) - (double)mean;       // (x + 0.5/256) - mean in f64
  float u = (float)(t / (double)scale);                       // logistic(float) argument
  double l = 1.0 / (1.0 + (double)expf_glibc(-u, tab));      // logistic, rans.pyx:26
  float p = (float)(l * 16775168.0);                          // * (M - 2048) then PyFloat->float
  int part1 = (int)round_f(p);                                // (int)round(float) -> roundf
  return part1 + part2;
}

// rans.pyx:51 -- lower = int(round(mean*256 - 1024)) / 256.  (the float window origin)
IDF_HD int rans_lower_int(float mean) {
  return (int)round_d((double)mean * 256.0 - 1024.0);
}
IDF_HD float rans_lower_f(int lower) { return (float)((double)lower / 256.0); }

}  // namespace idf
