// rans_kernels.hip -- CDNA4 (gfx950) rANS coder, bit-identical to the
// reference Cython coder (/root/reference/rans/rans.pyx:37-110) per stream.
//
// A "stream" is one reference encode()/decode() call: symbols
// [sym_off[k], sym_off[k+1]) coded from init_state[k].  Many independent
// streams run at once (one reference-format stream per lane/wave).
//
// Kernels
//   rans_cdf_freq   : pass 1 of encode (rans.pyx:50-56), one thread per symbol,
//                     fully parallel, HBM-bound (12 B in, 8 B out per symbol).
//   rans_encode_prep: the streamed encoder's pass 1: (start, freq), the window
//                     flag and 1/freq per symbol, fully parallel.
//   rans_encode     : pass 2 (rans.pyx:61-66), ONE WAVE per stream: the state chain
//                     on the scalar unit (readlane of coalesced 64-symbol record chunks,
//                     magic-reciprocal quotient), words stored 64 at a time.
//   rans_decode     : rans.pyx:69-110, ONE WAVE per stream (plus one table-producer wave
//                     that computes, a window ahead in LDS, the EXACT CDF at the last bin
//                     of each of the 2048-bin window's 64 blocks, per symbol).  The reference's
//                     11-12 step binary search over the 2048-bin window is
//                     replaced by one integer ballot of mod against the 64 exact block
//                     boundaries and ONE round of 33 exact CDF probes over the chosen
//                     block (cdf_bin: branch-free, bit-identical to rans_cdf).  The CDF
//                     is strictly increasing in s for scale > 0 (part2 steps by 1,
//                     part1 is monotone: glibc expf verified monotone on every float),
//                     so this is the reference's s; scales outside the fast range take
//                     a two-round exact 64-ary search and scale <= 0 or NaN the
//                     reference's serial binary search.
//   gather_words    : compacts per-stream word runs into one contiguous buffer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "idf_cdf.h"
#include "idf_codec_internal.h"

#pragma clang fp contract(off)

// Timing-only instrumentation for tools/native/rans_bench (never set in the library build):
// s_memtime stamps at six points of the decode chain for symbols 0..255 of stream 0.
#ifndef IDF_DECODE_STAMPS
#define IDF_DECODE_STAMPS 0
#endif
#ifndef IDF_DECODE_SETTLE
#define IDF_DECODE_SETTLE 1
#endif
#ifndef IDF_DECODE_FAKE_CDF
#define IDF_DECODE_FAKE_CDF 0
#endif
#if IDF_DECODE_STAMPS
__device__ unsigned long long g_stamp[256][6];
#define STAMP(j, sym) do { if (k == 0 && (sym) < 256) g_stamp[(sym)][j] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define STAMP(j, sym) do { } while (0)
#endif

namespace idf {

static constexpr uint64_t kRansL = 0x100000000ull;

__device__ __forceinline__ void window_check(float x, int lower, int32_t* flag) {
  // symbol index s = x*256 must satisfy lower <= s <= lower+2047 to round-trip
  float s = x * 256.0f;
  if (!(s >= (float)lower && s <= (float)(lower + 2047))) *flag |= IDF_STREAM_OUT_OF_WINDOW;
}

// ---------------------------------------------------------------- pass 1
__global__ void __launch_bounds__(256) rans_cdf_freq_kernel(int64_t n, const float* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ scale,
                                                            int32_t* __restrict__ start,
                                                            int32_t* __restrict__ freq) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float xi = x[i], mi = mean[i], si = scale[i];
  if (si == 0.0f) {  // ZeroDivisionError("float division"), rans.cpp:1435-1438
    start[i] = 0;
    freq[i] = IDF_FREQ_SCALE_ZERO;
    return;
  }
  int lo = rans_lower_int(mi);
  float lower = rans_lower_f(lo);  // rans.pyx:51
  float xm = (float)((double)xi - 1.0 / 256.0);
  int s = rans_cdf(xm, mi, si, lower);  // rans.pyx:52
  int e = rans_cdf(xi, mi, si, lower);  // rans.pyx:53
  start[i] = s;
  freq[i] = e - s;
}

// ---------------------------------------------------------------- pass 2
// Pass 1 for the streamed encoder: everything per symbol that does not depend on the
// state chain -- (start, freq), the window flag and the divisor's reciprocal -- so the
// serial pass 2 is a load, a compare, one multiply-correct division and an add.
struct EncSym {
  int32_t start, freq, wflag, pad;
};

__global__ void __launch_bounds__(256) rans_encode_prep_kernel(
    int64_t n, const float* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ scale, EncSym* __restrict__ sym, uint64_t* __restrict__ rcp) {
  __shared__ uint64_t tab[32];
  if (threadIdx.x < 32) tab[threadIdx.x] = kExp2fTab[threadIdx.x];
  __syncthreads();
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float xi = x[i], mi = mean[i], si = scale[i];
  EncSym e = {0, IDF_FREQ_SCALE_ZERO, 0, 0};
  uint64_t r = 0;
  const int lo = rans_lower_int(mi);
  if (si != 0.0f) {  // ZeroDivisionError("float division"), rans.cpp:1435-1438
    float lower = rans_lower_f(lo);  // rans.pyx:51
    float xm = (float)((double)xi - 1.0 / 256.0);
    e.start = rans_cdf(xm, mi, si, lower, tab);      // rans.pyx:52
    e.freq = rans_cdf(xi, mi, si, lower, tab) - e.start;  // rans.pyx:53
    // the divisor as the reference widens it (vector<ull>.push_back(int))
    const uint64_t f = (uint64_t)(int64_t)e.freq;
    if (f != 0) r = ~0ull / f;
  }
  int32_t f = 0;
  window_check(xi, lo, &f);
  e.wflag = f;
  sym[i] = e;
  rcp[i] = r;
}

// High 64 bits of a 64x64-bit product from 32-bit pieces (uniform operands: SALU
// s_mul_i32 / s_mul_hi_u32 and carry adds).
__device__ __forceinline__ uint64_t mulhi_u64(uint64_t a, uint64_t b) {
  const uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32);
  const uint32_t bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
  const uint64_t ll = (uint64_t)al * bl, lh = (uint64_t)al * bh;
  const uint64_t hl = (uint64_t)ah * bl, hh = (uint64_t)ah * bh;
  const uint64_t mid = (ll >> 32) + (uint32_t)lh + (uint32_t)hl;
  return hh + (lh >> 32) + (hl >> 32) + (mid >> 32);
}

// a >= b on 32-bit halves (keeps uniform compares on the scalar unit)
__device__ __forceinline__ bool ge_u64(uint64_t a, uint64_t b) {
  const uint32_t ah = (uint32_t)(a >> 32), bh = (uint32_t)(b >> 32);
  return ah != bh ? ah > bh : (uint32_t)a >= (uint32_t)b;
}

// Exact q = state / f, r = state % f for any f >= 1, state < 2^64, given
// m = floor((2^64 - 1) / f): m*f = 2^64 - 1 - rho (0 <= rho < f), so
// state*m / 2^64 lies in (state/f - 1, state/f] and mulhi(state, m) is q or q - 1.
__device__ __forceinline__ void divmod_u64_magic(uint64_t state, uint64_t f, uint64_t m,
                                                 uint64_t& q, uint64_t& r) {
  uint64_t qe = mulhi_u64(state, m);
  uint64_t rr = state - qe * f;
  if (ge_u64(rr, f)) {
    qe += 1;
    rr -= f;
  }
  q = qe;
  r = rr;
}

// Pass 2 (rans.pyx:61-66), one wave per stream.  The wave loads the records of 64 symbols
// at a time with coalesced 16-B + 8-B loads (the next 64 in flight), and the state chain
// runs on wave-uniform values -- v_readlane of symbol u's record into SGPRs, then scalar
// arithmetic -- so a symbol costs a few dozen scalar instructions instead of a lane's
// dependent 64-bit VALU chain.  Emitted words collect in one VGPR (lane = the
// fill index, one select) and leave as coalesced 256-B stores.
__global__ void __launch_bounds__(64) rans_encode_kernel(
    int64_t nstreams, const int64_t* __restrict__ sym_off, const EncSym* __restrict__ sym,
    const uint64_t* __restrict__ magic, const uint64_t* __restrict__ init_state,
    uint64_t* __restrict__ final_state, uint32_t* __restrict__ words, int64_t* __restrict__ nwords,
    int32_t* __restrict__ status) {
  const int64_t k = blockIdx.x;
  if (k >= nstreams) return;
  const int lane = threadIdx.x;
  const int64_t b = sym_off[k], e = sym_off[k + 1];
  uint64_t state = init_state[k];
  uint32_t* out = words + b;
  int64_t nw = 0;  // words stored
  int fill = 0;    // words waiting in wbuf (lanes 0..fill-1)
  uint32_t wbuf = 0;
  int32_t wflag = 0, stop = 0;
  EncSym cur = {0, 0, 0, 0};
  uint64_t mcur = 0;
  if (b + lane < e) {
    cur = sym[b + lane];
    mcur = magic[b + lane];
  }
  for (int64_t i0 = b; i0 < e; i0 += 64) {
    EncSym nxt = {0, 0, 0, 0};
    uint64_t mnxt = 0;
    if (i0 + 64 + lane < e) {
      nxt = sym[i0 + 64 + lane];
      mnxt = magic[i0 + 64 + lane];
    }
    const int cnt = (int)(e - i0 < 64 ? e - i0 : 64);
    const uint32_t mlo_v = (uint32_t)mcur, mhi_v = (uint32_t)(mcur >> 32);
    int u = 0;
    for (; u < cnt; ++u) {
      const int32_t st = __builtin_amdgcn_readlane(cur.start, u);
      const int32_t fr = __builtin_amdgcn_readlane(cur.freq, u);
      const uint64_t m = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(mhi_v, u) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane(mlo_v, u);
      if (fr <= 0) {  // rare: the scale-zero marker, a zero or a negative (non-monotone) freq
        if (fr == IDF_FREQ_SCALE_ZERO && st == 0) {
          stop = IDF_STREAM_SCALE_ZERO;
          break;
        }
        const uint64_t f = (uint64_t)(int64_t)fr;  // vector<ull>.push_back(int)
        if (state >= (f << 40)) {                  // rans.pyx:62-64
          wbuf = lane == fill ? (uint32_t)state : wbuf;
          if (++fill == 64) {
            out[nw + lane] = wbuf;
            nw += 64;
            fill = 0;
          }
          state >>= 32;
        }
        if (f == 0) {  // ZeroDivisionError, rans.cpp:1825-1834
          stop = IDF_STREAM_FREQ_ZERO;
          break;
        }
        uint64_t q, r;
        divmod_u64_magic(state, f, m, q, r);
        state = (q << 24) + r + (uint64_t)(int64_t)st;  // rans.pyx:65
        continue;
      }
      // rans.pyx:62-64: state >= f << 40; the low word of f << 40 is 0, so compare high
      // words.  Branch-free: the word goes to lane `fill` only when emitted.
      const uint32_t sh = (uint32_t)(state >> 32);
      const bool emit = sh >= ((uint32_t)fr << 8);
      wbuf = lane == (emit ? fill : 64) ? (uint32_t)state : wbuf;
      fill += emit ? 1 : 0;
      state = emit ? (uint64_t)sh : state;
      if (fill == 64) {
        out[nw + lane] = wbuf;
        nw += 64;
        fill = 0;
      }
      // rans.pyx:65 with q = state / f from the magic reciprocal (q or q - 1); the
      uint64_t q = mulhi_u64(state, m);
      // remainder and its correction fit 32 bits; rr - f borrows (bit 31) iff rr < f
      const uint32_t rr = (uint32_t)state - (uint32_t)q * (uint32_t)fr;
      const uint32_t d = rr - (uint32_t)fr;
      uint32_t borrow = d >> 31;
      asm("" : "+s"(borrow));  // opaque: a scalar shift, not a compare + VALU bool select
      q += 1u - borrow;
      const uint32_t r = d < rr ? d : rr;
      state = (q << 24) + r + (uint64_t)(int64_t)st;
    }
    if (lane < u) wflag |= cur.wflag;  // flags of the symbols coded
    if (stop) break;
    cur = nxt;
    mcur = mnxt;
  }
  if (lane < fill) out[nw + lane] = wbuf;
  nw += fill;
  // OR of the lanes' window flags
  for (int d = 32; d >= 1; d >>= 1) wflag |= __shfl_xor(wflag, d, 64);
  if (lane == 0) {
    final_state[k] = state;
    nwords[k] = nw;
    status[k] = wflag | stop;
  }
}

// ---------------------------------------------------------------- decode
__device__ __forceinline__ float sym_x(int s) { return (float)((double)s / 256.0); }

// Reference binary search (rans.pyx:96-104) for the non-monotone corner
// (scale <= 0 or NaN).  Returns s and flags.
__device__ int ref_binary_search(uint64_t mod, int lower, float mean, float scale, float lf,
                                 int32_t* flag, const uint64_t* tab) {
  int upper = lower + 0x7FF;
  while (lower <= upper) {
    int s = (lower + upper) >> 1;
    int c = rans_cdf(sym_x(s), mean, scale, lf, tab);
    if (c < 0) *flag |= IDF_STREAM_NEG_CDF;
    if ((uint64_t)(int64_t)c > mod) upper = s - 1;
    else lower = s + 1;
  }
  return lower;
}

// ---- bit-exact CDF with the divisions in their unscaled form.
// hipcc lowers a f64 division x / y to v_div_scale (x2), v_rcp + two Newton steps on the
// scaled y, q = x * r, a residual FMA, v_div_fmas and v_div_fixup.  For the operands the
// coder produces (float inputs widened to double, |quotient| far inside the double
// range, finite nonzero y) div_scale leaves both operands unchanged (VCC = 0), div_fmas
// is a plain FMA and div_fixup returns its input, so the same arithmetic without them is
// bit-identical; the y-only half (the refined reciprocal) is hoisted per symbol.
__device__ __forceinline__ double rcp_refined(double y) {
  double r = __builtin_amdgcn_rcp(y);
  r = __builtin_fma(r, __builtin_fma(-y, r, 1.0), r);
  return __builtin_fma(r, __builtin_fma(-y, r, 1.0), r);
}
__device__ __forceinline__ double div_unscaled(double x, double y, double r) {
  const double q = x * r;
  return __builtin_fma(__builtin_fma(-y, q, x), r, q);
}
// scale range in which the hoisted division is used (else rans_cdf's own '/')
__device__ __forceinline__ bool fast_scale_ok(float scale) {
  return scale >= 0x1p-60f && scale <= 0x1p60f;
}
// rans_cdf (idf_cdf.h) with rs = rcp_refined((double)scale), fast_scale_ok(scale).
__device__ __forceinline__ int rans_cdf_rs(float x, float mean, float scale, float lower,
                                           const uint64_t* tab, double rs) {
  float d = x - lower;
  int part2 = (int)round_d((double)d * 256.0) + 1;
  double t = ((double)x + 0.001953125) - (double)mean;
  float u = (float)div_unscaled(t, (double)scale, rs);
  double y = 1.0 + (double)expf_glibc(-u, tab);
  double l = __builtin_isinf(y) ? 0.0 : div_unscaled(1.0, y, rcp_refined(y));
  float p = (float)(l * 16775168.0);
  int part1 = (int)round_f(p);
  return part1 + part2;
}

// part1 = round((M - 2048) / (1 + expf(-u))) of rans.pyx:34 as a function of the float
// logistic argument u alone, in few instructions (the decoder's serial chain is issue-bound:
// one wave, one instruction per ~4 cycles):
//   * glibc expf's table path on x = -u clamped to [-0x1.9fe368p6, 0x1.62e42ep6] (one
//     v_med3): outside that range glibc returns 0 (below) or inf (above), and the clamp ends
//     give the same part1 through the table path -- expf(lo) is below 2^-53, so 1 + expf
//     rounds to 1 and part1 = M - 2048; expf(hi) is ~2^128, so part1 rounds to 0;
//   * 1/y by v_rcp_f64, ONE Newton step and the quotient correction (the IEEE division
//     hipcc emits takes two Newton steps, div_scale and div_fixup);
//   * roundf(p) for p >= 0 as v_cvt_rpi_i32_f32 (floor(p + 0.5) without rounding the sum).
// Equal to part1_ref (the reference's arithmetic) on every non-NaN float u
// (idf_rans_part1_selfcheck: all 2^32 bit patterns); u is never NaN here (scale > 0).
__device__ __forceinline__ int part1_ref(float u, const uint64_t* tab) {
  const double l = 1.0 / (1.0 + (double)expf_glibc(-u, tab));
  return (int)round_f((float)(l * 16775168.0));
}
__device__ __forceinline__ int part1_fast(float u, const uint64_t* tab) {
  const double InvLn2N = 0x1.71547652b82fep+0 * 32;
  const double SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / (32.0 * 32.0 * 32.0);
  const double C1 = 0x1.ebfce50fac4f3p-3 / (32.0 * 32.0);
  const double C2 = 0x1.62e42ff0c52d6p-1 / 32.0;
  const float x = __builtin_amdgcn_fmed3f(-u, -0x1.9fe368p6f, 0x1.62e42ep6f);
  const double xd = (double)x;
  double kd = __builtin_fma(InvLn2N, xd, SHIFT);
  const uint64_t ki = d2u(kd);
  kd -= SHIFT;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  const double sc = u2d(tab[ki % 32] + (ki << 47));
  const double z = __builtin_fma(C0, r, C1);
  const double r2 = r * r;
  double ey = __builtin_fma(C2, r, 1.0);
  ey = __builtin_fma(z, r2, ey);
  const double y = 1.0 + (double)(float)(ey * sc);
  double rc = __builtin_amdgcn_rcp(y);
  rc = __builtin_fma(rc, __builtin_fma(-y, rc, 1.0), rc);
  const double l = __builtin_fma(__builtin_fma(-y, rc, 1.0), rc, rc);  // 1/y, correctly rounded
  const float p = (float)(l * 16775168.0);
  int pn;
  asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(pn) : "v"(p));
  return pn;
}
// The exact CDF at bin q (x = q/256) for scale > 0 with fast_scale_ok(scale): rans_cdf_rs with
// the integer-exact forms of its x terms -- part2 = round((x - lower_f) * 256) + 1 = q - lower + 1
// (both operands are multiples of 2^-8: the f32 subtraction is exact), (double)x + 2^-9 =
// (2q + 1) * 2^-9 (exact, so fma((2q + 1), 2^-9, -mean) is the reference's rounded difference)
// -- and part1_fast.
__device__ __forceinline__ int cdf_bin(int q, int lower, double mean_d, double scale_d, double rs,
                                       const uint64_t* tab) {
  // (2q + 1) * 2^-9 is exact, so one fma rounds exactly as the reference's subtraction
  const double t = __builtin_fma((double)(2 * q + 1), 0.001953125, -mean_d);
  const float u = (float)div_unscaled(t, scale_d, rs);
  return part1_fast(u, tab) + (q - lower + 1);
}
// the exact CDF at bin q for any scale != 0 (rans_cdf, or cdf_bin where it applies)
__device__ __forceinline__ int cdf_any(int q, int lower, float mean, float scale, const uint64_t* tab) {
  if (scale > 0.0f && fast_scale_ok(scale))
    return cdf_bin(q, lower, (double)mean, (double)scale, rcp_refined((double)scale), tab);
  return rans_cdf(sym_x(q), mean, scale, rans_lower_f(lower), tab);
}

// Exact two-round 64-ary search over the reference window (rans.pyx:96-104 result):
// round 1: lane L probes the last bin of block L; round 2: 33 lanes probe the chosen
// block and its left neighbour.  The slow path: scale > 0 outside fast_scale_ok.
__device__ __forceinline__ void exact_search(uint64_t mod, int lower, float mi, float si, float lf,
                                             int lane, int* s_out, int* c_lo, int* c_hi,
                                             const uint64_t* tab) {
  int p1 = lower + 32 * lane + 31;
  int c1 = rans_cdf(sym_x(p1), mi, si, lf, tab);
  uint64_t m1 = __ballot((uint64_t)(int64_t)c1 > mod);
  if (m1 == 0) {
    // no bin in the window has CDF > mod: reference leaves s = lower + 2048
    int s = lower + 2048;
    int q = s - 1 + (lane & 1);
    int cq = rans_cdf(sym_x(q), mi, si, lf, tab);
    *s_out = s;
    *c_lo = __builtin_amdgcn_readlane(cq, 0);
    *c_hi = __builtin_amdgcn_readlane(cq, 1);
    return;
  }
  int blk = __ffsll((unsigned long long)m1) - 1;
  int base = lower + 32 * blk - 1;  // probe base-1 .. base+31 (33 points)
  int q = base + (lane <= 32 ? lane : 32);
  int cq = rans_cdf(sym_x(q), mi, si, lf, tab);
  uint64_t m2 = __ballot(lane >= 1 && lane <= 32 && (uint64_t)(int64_t)cq > mod);
  int kk = __ffsll((unsigned long long)m2) - 1;  // >= 1
  *s_out = base + kk;
  *c_lo = __builtin_amdgcn_readlane(cq, kk - 1);
  *c_hi = __builtin_amdgcn_readlane(cq, kk);
}

// Per-symbol parameters of the decoder's fast loop (32 B): twice the window origin plus one,
// -mean and scale widened to double and the refined reciprocal of the scale.
struct DecRec {
  int32_t l2, pad;  // 2 * lower + 1
  double mneg, sd, rs;
};

// The table producer of one decoded stream ("helper" wave): for every window of 64 symbols
// (in decode order), the EXACT CDF at the last bin of each of the window's 64 blocks of 32
// bins, bt[t * 64 + l] = CDF(lower_t + 32 l + 31) (scale <= 0: unused, 0), and the symbols'
// DecRecs, written into the LDS slot the decoding wave reads next.  Nothing of it depends on
// the state chain, so it runs a window ahead of the chain on another wave of the block and
// the decode needs no device workspace: the boundaries never leave the CU.
__device__ __forceinline__ void dec_fill_window(const float* __restrict__ mean,
                                                const float* __restrict__ scale, int64_t i_hi,
                                                int cnt, int lane, int32_t* bt, DecRec* rc,
                                                const uint64_t* tab) {
  float mv = 0.0f, sv = 1.0f;
  if (lane < cnt) {  // lane t: symbol i_hi - t (the reverse order the chain decodes in)
    mv = mean[i_hi - lane];
    sv = scale[i_hi - lane];
  }
  const int lower_v = rans_lower_int(mv);
  const bool fast_v = sv > 0.0f && fast_scale_ok(sv);
  const double rs_v = fast_v ? rcp_refined((double)sv) : 0.0;
  rc[lane] = DecRec{2 * lower_v + 1, 0, -(double)mv, (double)sv, rs_v};
  const uint64_t rsb = __builtin_bit_cast(uint64_t, rs_v);
  for (int t = 0; t < cnt; ++t) {
    const int lower = __builtin_amdgcn_readlane(lower_v, t);
    const float mi = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mv), t));
    const float si = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, sv), t));
    const int q = lower + 32 * lane + 31;
    int c = 0;
    if (si > 0.0f && fast_scale_ok(si)) {
      const double rs = __builtin_bit_cast(
          double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(rsb >> 32), t) << 32) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rsb, t));
      c = cdf_bin(q, lower, (double)mi, (double)si, rs, tab);
    } else if (si > 0.0f) {
      c = rans_cdf(sym_x(q), mi, si, rans_lower_f(lower), tab);
    }
    bt[t * 64 + lane] = c;
  }
}

// The decoding wave's progress marker once it has stopped: its table producer exits
constexpr int kDecDone = 1 << 30;

// PAIRS streams per block.  Waves 0..PAIRS-1 decode one stream each (the serial chain);
// wave PAIRS + p fills stream p's window tables (dec_fill_window) one window ahead, through
// a two-slot LDS ring and two LDS counters per pair (ready: windows filled, consumed: windows
// decoded; workgroup-scope release/acquire).  The decoding waves never synchronise with each
// other, so packing PAIRS streams per block only concentrates the decode on fewer CUs
// (nstreams / PAIRS), which leaves the rest of the chip to a concurrent lane's convolutions
// (ImageCodec lanes).
//
// Per symbol (rans.pyx:84-109), for scale > 0 in the fast range:
//   1. one integer ballot of mod against the 64 exact block boundaries gives the block b of
//      the reference's answer: the first block whose last bin has CDF > mod, or b = 64 when
//      none has (then s = lower + 2048, rans.pyx's loop exit);
//   2. ONE exact round: lane j evaluates the CDF at q = lower + 32 b - 1 + j (lanes 1..32
//      the block, lane 0 its left neighbour); the CDF is strictly increasing for scale > 0
//      (part2 steps by one, part1 is monotone: glibc expf verified monotone on every float),
//      so the first lane in 1..32 with CDF > mod (or q past the window) is s, and lanes k-1,
//      k hold CDF(s - 1), CDF(s) -- no bracket checks and no second search.
// Other scales take the reference's own searches (exact_search, ref_binary_search).
template <int PAIRS>
__global__ void __launch_bounds__(128 * PAIRS) rans_decode_kernel(
    int64_t nstreams, const int64_t* __restrict__ sym_off, const int64_t* __restrict__ word_off,
    const int64_t* __restrict__ nwords, const uint32_t* __restrict__ words,
    const float* __restrict__ mean, const float* __restrict__ scale,
    const uint64_t* __restrict__ init_state, uint64_t* __restrict__ final_state,
    float* __restrict__ out, int32_t* __restrict__ status) {
  __shared__ uint64_t tab[32];
  // block boundaries and parameter records, 2 windows per stream
  // (one spare row each: the fast loop reads one symbol ahead unconditionally)
  __shared__ __attribute__((aligned(16))) int32_t bt_all[PAIRS][2][65 * 64];
  __shared__ __attribute__((aligned(16))) DecRec rc_all[PAIRS][2][65];
  __shared__ int ready[PAIRS], consumed[PAIRS];
  if (threadIdx.x < 32) tab[threadIdx.x] = kExp2fTab[threadIdx.x];
  if (threadIdx.x < PAIRS) {
    ready[threadIdx.x] = 0;
    consumed[threadIdx.x] = 0;
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pr = wave < PAIRS ? wave : wave - PAIRS;
  const int64_t k = (int64_t)blockIdx.x * PAIRS + pr;
  if (k >= nstreams) return;
  auto& bt = bt_all[pr];
  auto& rc = rc_all[pr];
  if (wave >= PAIRS) {  // the table producer
    const int lane = threadIdx.x & 63;
    const int64_t b = sym_off[k], n = sym_off[k + 1] - b;
    int win = 0;
    for (int64_t j0 = 0; j0 < n; j0 += 64, ++win) {
      // slot win & 1 is free once window win - 2 is decoded
      for (;;) {
        const int c = __hip_atomic_load(&consumed[pr], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (c >= kDecDone) return;
        if (c >= win - 1) break;
        __builtin_amdgcn_s_sleep(2);
      }
      const int cnt = n - j0 < 64 ? (int)(n - j0) : 64;
      dec_fill_window(mean, scale, b + n - 1 - j0, cnt, lane, bt[win & 1], rc[win & 1], tab);
      __hip_atomic_store(&ready[pr], win + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return;
  }
  __builtin_amdgcn_s_setprio(2);  // the chain's instructions first on a SIMD shared with a producer
  const int lane = threadIdx.x & 63;
  const int64_t b = sym_off[k], n = sym_off[k + 1] - b;
  const uint32_t* w = words + word_off[k];
  int64_t pos = nwords[k];
  uint64_t state = init_state[k];
  int32_t flag = 0;
  // Nothing the chain needs waits on memory: symbols are decoded in windows of 64 whose
  // (mean, scale) and derived (lower, 1/scale) sit one per lane, computed in parallel
  // while the previous window decodes; the window's block boundaries are copied into LDS
  // by DMA one window ahead; words come from a 64-word register window read with a
  // uniform lane index; each lane keeps its symbol's output for one coalesced store per
  // window.
  auto ld_params = [&](int64_t j0, float& mv, float& sv) {
    const int64_t i = b + n - 1 - j0 - lane;  // reverse order
    mv = 0.0f;
    sv = 1.0f;
    if (j0 + lane < n) {
      mv = mean[i];
      sv = scale[i];
    }
  };
  // Words: a 128-word register buffer (lane l of wA holds w[wb - 1 - l], of wB w[wb - 65 - l])
  // loaded at the START of the previous window from that window's pos: a window consumes at
  // most 64 words (one per symbol, rans.pyx:86-89), so the buffer covers the next window too
  // and no word read ever waits on memory.
  auto ld_words = [&](int64_t base, uint32_t& a, uint32_t& c) {
    const int64_t i0 = base - 1 - lane, i1 = base - 65 - lane;
    a = i0 >= 0 ? w[i0] : 0u;
    c = i1 >= 0 ? w[i1] : 0u;
  };
  int64_t wb = pos, wnb = pos;
  uint32_t wA, wB, wnA, wnB;
  ld_words(wb, wA, wB);
  wnA = wA;
  wnB = wB;
  // rans.pyx:86-89 (buffer read in reverse), branch-free on the scalar unit; running out of
  // words flags the stream (the reference indexes past its buffer) and decoding goes on
  // with garbage that the status marks
  auto renorm = [&]() {
    const bool need = __builtin_amdgcn_readfirstlane((int)(state >> 32)) == 0;
    const int idx = (int)(wb - pos);
    const uint32_t wa = (uint32_t)__builtin_amdgcn_readlane((int)wA, idx & 63);
    const uint32_t wc = (uint32_t)__builtin_amdgcn_readlane((int)wB, idx & 63);
    const uint32_t word = idx < 64 ? wa : wc;
    flag |= (need && pos <= 0) ? IDF_STREAM_UNDERFLOW : 0;
    state = need ? ((state << 32) | (uint64_t)word) : state;
    pos -= need ? 1 : 0;
  };
  // the word a renormalisation at the current pos would read (w[pos - 1])
  auto next_word = [&]() -> uint32_t {
    const int idx = (int)(wb - pos);
    const uint32_t wa = (uint32_t)__builtin_amdgcn_readlane((int)wA, idx & 63);
    const uint32_t wc = (uint32_t)__builtin_amdgcn_readlane((int)wB, idx & 63);
    return idx < 64 ? wa : wc;
  };
  float mcur, scur, mnxt = 0.0f, snxt = 1.0f;
  ld_params(0, mcur, scur);
  asm volatile("" ::"v"(wA), "v"(wB), "v"(mcur), "v"(scur));
  bool stop = false;
  int slot = 0, win = 0;
  for (int64_t j0 = 0; j0 < n && !stop; j0 += 64, slot ^= 1, ++win) {
    const int cnt = n - j0 < 64 ? (int)(n - j0) : 64;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // parameters and words landed
    // this window's boundaries and records are in LDS slot `slot` once ready > win
    while (__hip_atomic_load(&ready[pr], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= win)
      __builtin_amdgcn_s_sleep(1);
    wA = wnA;  // j0 = 0: the same buffer
    wB = wnB;
    wb = wnb;
    if (j0 + 64 < n) {
      ld_params(j0 + 64, mnxt, snxt);
      ld_words(pos, wnA, wnB);
      wnb = pos;
    }
    // per-lane derived parameters of this window's symbols
    const int lower_l = rans_lower_int(mcur);  // rans.pyx:91
    const bool fast_l = scur > 0.0f && fast_scale_ok(scur);
    const double rs_l = fast_l ? rcp_refined((double)scur) : 0.0;
    float outv = 0.0f;
    int done = 0;
    int ablk = bt[slot][lane];
    // Windows whose symbols all take the fast path run a straight-line loop: the state stays
    // in SGPRs, the next symbol's parameters and block boundaries are fetched one symbol
    // ahead, and the loop has no branch but its back-edge.
    if (__ballot(lane < cnt && !fast_l) == 0) {
      // The window's words in ONE register: lane l holds w[P - 1 - l], P = pos now (a window
      // reads at most 64 words), gathered from the 128-word buffer.
      const int P = (int)pos;
      const int dsh = (int)(wb - pos);  // 0..64
      const int src = ((lane + dsh) & 63) * 4;
      const uint32_t ga = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wA);
      const uint32_t gc = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wB);
      const uint32_t wcur = lane + dsh < 64 ? ga : gc;
      int ipos = P;
      uint32_t wnext = (uint32_t)__builtin_amdgcn_readlane((int)wcur, 0);
      int outi = 0;  // lane t: s - lower of symbol t
      uint32_t st_lo = (uint32_t)state, st_hi = (uint32_t)(state >> 32);
      // LDS addresses kept in VGPRs (one add per symbol each, immediate offsets per field); the
      // next symbol's record and block boundaries are read one symbol ahead
      typedef int i4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) const i4* lds_i4;
      typedef __attribute__((address_space(3))) const int* lds_i1;
      int ra = (int)(uintptr_t)(const __attribute__((address_space(3))) void*)&rc[slot][0];
      int ba = (int)(uintptr_t)(const __attribute__((address_space(3))) void*)&bt[slot][lane];
      asm volatile("" : "+v"(ra), "+v"(ba));
      const int l2lane = 2 * lane;
      // one symbol: record (r0, r1) and block boundaries ab were read one symbol ahead
      auto symbol = [&](const i4& r0, const i4& r1, const int abc, const int t) {
        const int L2 = r0[0];
        const double mneg = __builtin_bit_cast(double, (uint64_t)(uint32_t)r0[2] | ((uint64_t)(uint32_t)r0[3] << 32));
        const double sd = __builtin_bit_cast(double, (uint64_t)(uint32_t)r1[0] | ((uint64_t)(uint32_t)r1[1] << 32));
        const double rs = __builtin_bit_cast(double, (uint64_t)(uint32_t)r1[2] | ((uint64_t)(uint32_t)r1[3] << 32));
        STAMP(0, j0 + t);
        // rans.pyx:86-89 with the next word already in an SGPR: SCC = (state < 2^32) selects
        // the shifted state and borrows one from pos
        asm volatile(
            "s_cmp_eq_u32 %1, 0\n\t"
            "s_cselect_b32 %1, %0, %1\n\t"
            "s_cselect_b32 %0, %3, %0\n\t"
            "s_subb_u32 %2, %2, 0"
            : "+s"(st_lo), "+s"(st_hi), "+s"(ipos) : "s"(wnext) : "scc");
        const int mod = (int)(st_lo & 0xffffffu);
        STAMP(1, j0 + t);
        const uint64_t mb = __ballot(abc > mod);
        uint32_t blk;  // first block whose last bin has CDF > mod, 64 if none (s_ff1 of 0 is -1)
        asm volatile("s_ff1_i32_b64 %0, %1\n\ts_min_u32 %0, %0, 64" : "=&s"(blk) : "s"(mb) : "scc");
        const int bs = 32 * (int)blk - 1;  // probe base - lower
        STAMP(2, j0 + t);
#if IDF_DECODE_FAKE_CDF  // timing-only: the loop skeleton without the CDF's dependent chain
        const int cq = (lane << 19) + (int)(sd > rs) + (int)(mneg > 0.0) + L2;
#else
        // q = lower + bs + lane: 2q + 1 = L2 + 2 bs + 2 lane
        const double td = __builtin_fma((double)(L2 + 2 * bs + l2lane), 0.001953125, mneg);
        const float u = (float)div_unscaled(td, sd, rs);
        const int cq = part1_fast(u, tab) + bs + 1 + lane;  // + part2 = q - lower + 1
#endif
        STAMP(3, j0 + t);
        // lane 0 (q = base) is never the answer: CDF(base) <= mod for blk > 0, and for blk = 0
        // the reference's search starts at lower = base + 1; blk = 64: s = lower + 2048
        const uint64_t m2 = __ballot(cq > mod) & ~1ull;
        const int kk = mb ? (int)__builtin_ctzll(m2) : 1;  // 1..32
        const int c_lo = __builtin_amdgcn_readlane(cq, kk - 1);
        const int c_hi = __builtin_amdgcn_readlane(cq, kk);
        STAMP(4, j0 + t);
        // freq >= 1 and c_lo >= 0 here (part2 steps by one, part1 >= 0); mod - c_lo may be
        // negative (blk = 0), the sum is the reference's modulo 2^64
        const uint64_t st = (((uint64_t)st_hi << 32 | st_lo) >> 24) * (uint64_t)(uint32_t)(c_hi - c_lo) +
                            (uint64_t)(int64_t)(mod - c_lo);
        st_lo = (uint32_t)st;
        st_hi = (uint32_t)(st >> 32);
        STAMP(5, j0 + t);
        {  // message.push_back(s / 256.): lane t keeps s - lower
          const int sv = bs + kk;
          asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(outi) : "s"(sv), "s"(t) : "m0");
        }
        wnext = (uint32_t)__builtin_amdgcn_readlane((int)wcur, (P - ipos) & 63);
        // the record's padding dword stays live to here, so the one-ahead boundary read never
        // lands in it (a write-after-write on a pending LDS read costs a full LDS round trip)
        asm volatile("" ::"v"(r0));
      };
      // Look-ahead LDS reads are issued only after an explicit wait for every earlier LDS read
      // (landed long ago: they were issued a symbol earlier); the wait-count pass then knows the
      // loaded registers are ready and adds no lgkmcnt(0) inside the chain that would also
      // wait for the reads just issued (it merges loop-carried loads conservatively).
      auto lds_settle = [] { __builtin_amdgcn_s_waitcnt(0xC07F); };  // lgkmcnt(0) only
      // two register sets, so the one-ahead reads need no copies; reads past the window's
      // last symbol land in the spare row and are never used
      i4 a0 = *(lds_i4)(uintptr_t)ra, a1 = *(lds_i4)(uintptr_t)(ra + 16);
      int aab = *(lds_i1)(uintptr_t)ba;
      int t = 0;
      for (; t + 1 < cnt; t += 2) {
        if (IDF_DECODE_SETTLE) lds_settle();
        const i4 b0 = *(lds_i4)(uintptr_t)(ra + 32), b1 = *(lds_i4)(uintptr_t)(ra + 48);
        const int bab = *(lds_i1)(uintptr_t)(ba + 256);
        symbol(a0, a1, aab, t);
        ra += 64;
        ba += 512;
        if (IDF_DECODE_SETTLE) lds_settle();
        a0 = *(lds_i4)(uintptr_t)ra;
        a1 = *(lds_i4)(uintptr_t)(ra + 16);
        aab = *(lds_i1)(uintptr_t)ba;
        symbol(b0, b1, bab, t + 1);
      }
      if (t < cnt) symbol(a0, a1, aab, t);
      state = (uint64_t)st_hi << 32 | st_lo;
      pos = ipos;
      flag |= ipos < 0 ? IDF_STREAM_UNDERFLOW : 0;  // ran out of words (pos never grows)
      outv = (float)(outi + lower_l) * 0.00390625f;
      done = cnt;
    } else {
      for (int t = 0; t < cnt; ++t) {
        ablk = bt[slot][t * 64 + lane];
        renorm();
        const int mod = (int)(state & 0xffffffull);
        const int lower = __builtin_amdgcn_readlane(lower_l, t);
        const float mi = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mcur), t));
        const float si = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, scur), t));
        int sym, c_lo, c_hi;
        if (si > 0.0f && fast_scale_ok(si)) {
          const uint64_t rsb = __builtin_bit_cast(uint64_t, rs_l);
          const double rs = __builtin_bit_cast(
              double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(rsb >> 32), t) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rsb, t));
          const uint64_t mb = __ballot(ablk > mod);
          const int blk = mb ? __ffsll((unsigned long long)mb) - 1 : 64;
          const int base = lower + 32 * blk - 1;
          const int q = base + lane;
          const int cq = cdf_bin(q, lower, (double)mi, (double)si, rs, tab);
          const uint64_t m2 = __ballot(cq > mod || q > lower + 2047) & ~1ull;
          const int kk = __ffsll((unsigned long long)m2) - 1;
          sym = base + kk;
          c_lo = __builtin_amdgcn_readlane(cq, kk - 1);
          c_hi = __builtin_amdgcn_readlane(cq, kk);
        } else {
          const float lf = rans_lower_f(lower);
          if (si > 0.0f) {
            exact_search((uint64_t)mod, lower, mi, si, lf, lane, &sym, &c_lo, &c_hi, tab);
          } else if (si == 0.0f) {
            flag |= IDF_STREAM_SCALE_ZERO;
            stop = true;
            break;
          } else {
            sym = ref_binary_search((uint64_t)mod, lower, mi, si, lf, &flag, tab);
            c_lo = rans_cdf(sym_x(sym - 1), mi, si, lf, tab);
            c_hi = rans_cdf(sym_x(sym), mi, si, lf, tab);
          }
        }
        if (c_lo < 0 || c_hi - c_lo < 0) flag |= IDF_STREAM_NEG_CDF;
        const uint64_t cdf_s = (uint64_t)(int64_t)c_lo;
        const uint64_t freq_s = (uint64_t)(int64_t)(c_hi - c_lo);
        state = (state >> 24) * freq_s + (state & 0xffffffull) - cdf_s;  // rans.pyx:108
        if (lane == t) outv = sym_x(sym);  // message.push_back(s / 256.)
        done = t + 1;
      }
    }
    if (lane < done) out[b + n - 1 - j0 - lane] = outv;
    mcur = mnxt;
    scur = snxt;
    // window win decoded: its slot may be refilled (the release orders this window's LDS reads)
    __hip_atomic_store(&consumed[pr], win + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __hip_atomic_store(&consumed[pr], kDecDone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (lane == 0) {
    final_state[k] = state;
    status[k] = flag | (pos > 0 ? IDF_STREAM_WORDS_LEFT : 0);
  }
}

// ---------------------------------------------------------------- compaction
__global__ void __launch_bounds__(256) gather_words_kernel(int64_t nstreams,
                                                           const int64_t* __restrict__ src_off,
                                                           const int64_t* __restrict__ nwords,
                                                           const int64_t* __restrict__ dst_off,
                                                           const uint32_t* __restrict__ src,
                                                           uint32_t* __restrict__ dst) {
  int64_t k = blockIdx.x;
  if (k >= nstreams) return;
  const uint32_t* s = src + src_off[k];
  uint32_t* d = dst + dst_off[k];
  for (int64_t i = threadIdx.x; i < nwords[k]; i += blockDim.x) d[i] = s[i];
}

__global__ void expf_kernel(int64_t n, const float* __restrict__ in, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = expf_glibc(in[i]);
}

// Exhaustive device check: order-independent checksum over a range of float
// bit patterns, same formula as tests/native/expf_check.cpp.
__global__ void __launch_bounds__(256) expf_checksum_kernel(uint64_t lo, uint64_t hi,
                                                            unsigned long long* acc) {
  uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long sum = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (; i < hi; i += stride) {
    float a = expf_glibc(u2f((uint32_t)i));
    uint32_t h = (a != a) ? 0x7fc00000u : f2u(a);
    sum += (unsigned long long)h * ((uint64_t)i * 2654435761ull | 1ull);
  }
  // wave reduce
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_down(sum, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(acc, sum);
}

// part1_fast == part1_ref over a range of float bit patterns of u (NaN skipped)
__global__ void __launch_bounds__(256) part1_selfcheck_kernel(uint64_t lo, uint64_t hi,
                                                              unsigned long long* bad) {
  __shared__ uint64_t tab[32];
  if (threadIdx.x < 32) tab[threadIdx.x] = kExp2fTab[threadIdx.x];
  __syncthreads();
  unsigned long long cnt = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += stride) {
    const float u = u2f((uint32_t)i);
    if (u != u) continue;
    cnt += part1_fast(u, tab) != part1_ref(u, tab);
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(bad, cnt);
}

// Self-check of rans_cdf_rs and cdf_bin against rans_cdf on pseudo-random (x, mean, scale): scale
// log-uniform over the fast range, mean in +-2^12, x on the 1/256 grid within the
// window around mean.  Counts mismatching CDF values.
__global__ void __launch_bounds__(256) cdf_selfcheck_kernel(uint64_t n, uint64_t seed,
                                                            unsigned long long* bad) {
  __shared__ uint64_t tab[32];
  if (threadIdx.x < 32) tab[threadIdx.x] = kExp2fTab[threadIdx.x];
  __syncthreads();
  unsigned long long cnt = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t h = (i + seed) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 31; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 29;
    const float e = (float)((h & 0xFFFF) / 65536.0) * 120.0f - 60.0f;  // scale = 2^e
    const float scale = exp2f(e);
    const float mean = (float)(((h >> 16) & 0xFFFFFF) / 16777216.0 * 8192.0 - 4096.0);
    const int lower = rans_lower_int(mean);
    const float lf = rans_lower_f(lower);
    const int sidx = lower - 1 + (int)((h >> 40) % 2050u);
    const float x = (float)((double)sidx / 256.0);
    if (!fast_scale_ok(scale)) continue;
    const int a = rans_cdf(x, mean, scale, lf, tab);
    const int b = rans_cdf_rs(x, mean, scale, lf, tab, rcp_refined((double)scale));
    const int c = cdf_bin(sidx, lower, (double)mean, (double)scale, rcp_refined((double)scale), tab);
    cnt += (a != b) + (a != c);
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(bad, cnt);
}

}  // namespace idf

// ============================================================== C-ABI
using namespace idf;

extern "C" {

int idf_rans_cdf_freq(void* stream, int64_t n, const float* x, const float* mean,
                      const float* scale, int32_t* start, int32_t* freq) {
  if (n < 0) return IDF_ERR_ARG;
  if (n == 0) return IDF_OK;
  int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(rans_cdf_freq_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, n, x, mean, scale, start, freq);
  return idf_last_error();
}

int64_t idf_rans_encode_workspace_bytes(int64_t nsym) {
  return (int64_t)(sizeof(EncSym) + sizeof(uint64_t)) * (nsym > 0 ? nsym : 1);
}

int idf_rans_encode_streams(void* stream, int64_t nstreams, int64_t nsym, const int64_t* sym_off,
                            const float* x, const float* mean, const float* scale,
                            const uint64_t* init_state, uint64_t* final_state, uint32_t* words,
                            int64_t* nwords, int32_t* status, void* workspace,
                            int64_t workspace_bytes) {
  if (nstreams < 0 || nsym < 0) return IDF_ERR_ARG;
  if (nstreams == 0) return IDF_OK;
  if (workspace_bytes < idf_rans_encode_workspace_bytes(nsym)) return IDF_ERR_WORKSPACE;
  EncSym* es = (EncSym*)workspace;
  uint64_t* rcp = (uint64_t*)(es + (nsym > 0 ? nsym : 1));
  int rc = IDF_OK;
  if (nsym > 0)
    hipLaunchKernelGGL(rans_encode_prep_kernel, dim3((unsigned)((nsym + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, nsym, x, mean, scale, es, rcp);
  if (rc) return rc;
  hipLaunchKernelGGL(rans_encode_kernel, dim3((unsigned)nstreams), dim3(64), 0, (hipStream_t)stream,
                     nstreams, sym_off, es, rcp, init_state, final_state, words, nwords, status);
  return idf_last_error();
}

// Streams per block: 4 by default (a quarter of the CUs: decode lanes run beside another
// lane's convs; alone it measures the same as 1), IDF_DECODE_WPB=1 for one per block.
// Streams per decode block (IDF_DECODE_WPB = 1, 2 or 4; timing only, the bits never change).
// Two: the block's four waves (two decoding, two producing) take one SIMD each, so no chain
// shares its SIMD's issue with a producer -- 215 vs 265 ns per symbol for four streams per
// block -- while a lane's launch still holds half the CUs one stream per block would
// (profiles/r04/rans_wpb/: pipelined bench neutral to +1.3%, back-to-back decode 28.7 -> 27.9
// ms same box).
static int decode_pairs_per_block() {
  const char* e = getenv("IDF_DECODE_WPB");
  const int v = e ? atoi(e) : 2;
  return (v == 1 || v == 4) ? v : 2;
}

// The block-boundary tables live in LDS only (rans_decode_kernel's producer waves): the
// decode needs no device workspace.  A nonzero size keeps callers' allocations well-formed.
int64_t idf_rans_decode_workspace_bytes(int64_t nsym) {
  (void)nsym;
  return 256;
}

int idf_rans_decode_streams(void* stream, int64_t nstreams, int64_t nsym, const int64_t* sym_off,
                            const int64_t* word_off, const int64_t* nwords, const uint32_t* words,
                            const float* mean, const float* scale, const uint64_t* init_state,
                            uint64_t* final_state, float* out, int32_t* status, void* workspace,
                            int64_t workspace_bytes) {
  if (nstreams < 0 || nsym < 0) return IDF_ERR_ARG;
  if (nstreams == 0) return IDF_OK;
  (void)workspace;
  if (workspace_bytes < idf_rans_decode_workspace_bytes(nsym)) return IDF_ERR_WORKSPACE;
  if (decode_pairs_per_block() == 4)
    hipLaunchKernelGGL(rans_decode_kernel<4>, dim3((unsigned)((nstreams + 3) / 4)), dim3(512), 0,
                       (hipStream_t)stream, nstreams, sym_off, word_off, nwords, words, mean,
                       scale, init_state, final_state, out, status);
  else if (decode_pairs_per_block() == 2)
    hipLaunchKernelGGL(rans_decode_kernel<2>, dim3((unsigned)((nstreams + 1) / 2)), dim3(256), 0,
                       (hipStream_t)stream, nstreams, sym_off, word_off, nwords, words, mean,
                       scale, init_state, final_state, out, status);
  else
    hipLaunchKernelGGL(rans_decode_kernel<1>, dim3((unsigned)nstreams), dim3(128), 0,
                       (hipStream_t)stream, nstreams, sym_off, word_off, nwords, words, mean,
                       scale, init_state, final_state, out, status);
  return idf_last_error();
}

int idf_gather_words(void* stream, int64_t nstreams, const int64_t* src_off, const int64_t* nwords,
                     const int64_t* dst_off, const uint32_t* src, uint32_t* dst) {
  if (nstreams < 0) return IDF_ERR_ARG;
  if (nstreams == 0) return IDF_OK;
  hipLaunchKernelGGL(gather_words_kernel, dim3((unsigned)nstreams), dim3(256), 0,
                     (hipStream_t)stream, nstreams, src_off, nwords, dst_off, src, dst);
  return idf_last_error();
}

int idf_expf_glibc(void* stream, int64_t n, const float* in, float* out) {
  if (n <= 0) return n < 0 ? IDF_ERR_ARG : IDF_OK;
  hipLaunchKernelGGL(expf_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n, in, out);
  return idf_last_error();
}

int idf_rans_cdf_selfcheck(void* stream, uint64_t n, uint64_t seed, unsigned long long* bad) {
  hipLaunchKernelGGL(cdf_selfcheck_kernel, dim3(4096), dim3(256), 0, (hipStream_t)stream, n, seed,
                     bad);
  return idf_last_error();
}

int idf_rans_part1_selfcheck(void* stream, uint64_t lo, uint64_t hi, unsigned long long* bad) {
  hipLaunchKernelGGL(part1_selfcheck_kernel, dim3(8192), dim3(256), 0, (hipStream_t)stream, lo, hi,
                     bad);
  return idf_last_error();
}

int idf_expf_checksum(void* stream, uint64_t lo, uint64_t hi, unsigned long long* acc) {
  hipLaunchKernelGGL(expf_checksum_kernel, dim3(8192), dim3(256), 0, (hipStream_t)stream, lo, hi,
                     acc);
  return idf_last_error();
}

// ---- host-buffer convenience: exactly one reference call (rans.pyx:37 / :69)
// The _on forms run on the caller's stream with the caller's device workspace
// (idf_rans_host_workspace_bytes): async copies in, the batched kernels, async copies out, then
// a sync of that stream only (the outputs are host buffers).  The plain forms keep the
// reference's signature and run the same on a per-thread non-blocking stream with a per-thread
// workspace that only grows (no allocation per call, no device-wide sync); both are
// deliberately kept until the process exits.
namespace {
struct HostCarve {
  char* p;
  char* end;
  char* take(size_t b) {
    char* r = p;
    p += (b + 255) & ~(size_t)255;
    return p <= end ? r : nullptr;
  }
};
struct HostCtx {
  hipStream_t stream = nullptr;
  void* ws = nullptr;
  int64_t ws_bytes = 0;
};
int host_ctx(int64_t need, HostCtx** out) {
  thread_local HostCtx ctx;
  if (!ctx.stream && hipStreamCreateWithFlags(&ctx.stream, hipStreamNonBlocking) != hipSuccess) {
    ctx.stream = nullptr;
    return IDF_ERR_HIP;
  }
  if (need > ctx.ws_bytes) {
    if (ctx.ws) (void)hipFree(ctx.ws);
    ctx.ws = nullptr;
    ctx.ws_bytes = 0;
    const int64_t grow = std::max<int64_t>(need, 1 << 20);
    if (hipMalloc(&ctx.ws, (size_t)grow) != hipSuccess) return IDF_ERR_HIP;
    ctx.ws_bytes = grow;
  }
  *out = &ctx;
  return IDF_OK;
}
inline int64_t carve(int64_t b) { return (b + 255) & ~(int64_t)255; }
}  // namespace

#define CK(expr)                                   \
  do {                                             \
    if ((expr) != hipSuccess && rc == IDF_OK) rc = IDF_ERR_HIP; \
  } while (0)

int64_t idf_rans_host_workspace_bytes(int64_t n, int64_t nwords) {
  if (n < 0 || nwords < 0) return -1;
  const int64_t nn = n > 0 ? n : 1, nwn = nwords > 0 ? nwords : 1;
  // encode: x, mean, scale, words (<= n), offsets, states, counts, status, kernel workspace
  const int64_t enc = 4 * carve(nn * 4) + 6 * carve(16) + carve(idf_rans_encode_workspace_bytes(n));
  // decode: mean, scale, out, words, offsets, states, counts, status, kernel workspace
  const int64_t dec = 3 * carve(nn * 4) + carve(nwn * 4) + 7 * carve(16) +
                      carve(idf_rans_decode_workspace_bytes(n));
  return std::max(enc, dec);
}

int idf_rans_encode_on(void* stream, void* d_workspace, int64_t workspace_bytes,
                       uint64_t* state_io, int64_t n, const float* x, const float* mean,
                       const float* scale, uint32_t* words, int64_t* nwords_out,
                       int32_t* status_out) {
  if (n < 0 || !state_io || !d_workspace || (n > 0 && (!x || !mean || !scale || !words)))
    return IDF_ERR_ARG;
  if (workspace_bytes < idf_rans_host_workspace_bytes(n, 0)) return IDF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nn = n > 0 ? n : 1;
  HostCarve c{(char*)d_workspace, (char*)d_workspace + workspace_bytes};
  float* dx = (float*)c.take(nn * 4);
  float* dm = (float*)c.take(nn * 4);
  float* ds = (float*)c.take(nn * 4);
  uint32_t* dw = (uint32_t*)c.take(nn * 4);
  int64_t* doff = (int64_t*)c.take(16);
  uint64_t* dst = (uint64_t*)c.take(8);
  uint64_t* dfs = (uint64_t*)c.take(8);
  int64_t* dnw = (int64_t*)c.take(8);
  int32_t* dstat = (int32_t*)c.take(4);
  (void)c.take(8);
  void* kws = c.take((size_t)idf_rans_encode_workspace_bytes(n));
  if (!kws) return IDF_ERR_ARG;
  int rc = IDF_OK;
  const int64_t off[2] = {0, n};
  if (n > 0) {
    CK(hipMemcpyAsync(dx, x, n * 4, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(dm, mean, n * 4, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(ds, scale, n * 4, hipMemcpyHostToDevice, s));
  }
  CK(hipMemcpyAsync(doff, off, 16, hipMemcpyHostToDevice, s));
  CK(hipMemcpyAsync(dst, state_io, 8, hipMemcpyHostToDevice, s));
  if (rc == IDF_OK)
    rc = idf_rans_encode_streams(s, 1, n, doff, dx, dm, ds, dst, dfs, dw, dnw, dstat, kws,
                                 idf_rans_encode_workspace_bytes(n));
  int64_t nw = 0;
  int32_t stat = 0;
  uint64_t fs = 0;
  if (rc == IDF_OK) {
    CK(hipMemcpyAsync(&fs, dfs, 8, hipMemcpyDeviceToHost, s));
    CK(hipMemcpyAsync(&nw, dnw, 8, hipMemcpyDeviceToHost, s));
    CK(hipMemcpyAsync(&stat, dstat, 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (rc == IDF_OK && nw > 0) {  // the count sizes the last copy
      CK(hipMemcpyAsync(words, dw, nw * 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
    }
  } else {
    (void)hipStreamSynchronize(s);  // inputs may still be in flight from the caller's buffers
  }
  if (rc == IDF_OK) *state_io = fs;
  if (nwords_out) *nwords_out = nw;
  if (status_out) *status_out = stat;
  return rc;
}

int idf_rans_decode_on(void* stream, void* d_workspace, int64_t workspace_bytes,
                       uint64_t* state_io, const uint32_t* words, int64_t nwords, int64_t n,
                       const float* mean, const float* scale, float* out, int32_t* status_out) {
  if (n < 0 || nwords < 0 || !state_io || !d_workspace || (nwords > 0 && !words) ||
      (n > 0 && (!mean || !scale || !out)))
    return IDF_ERR_ARG;
  if (workspace_bytes < idf_rans_host_workspace_bytes(n, nwords)) return IDF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nn = n > 0 ? n : 1, nwn = nwords > 0 ? nwords : 1;
  HostCarve c{(char*)d_workspace, (char*)d_workspace + workspace_bytes};
  float* dm = (float*)c.take(nn * 4);
  float* ds = (float*)c.take(nn * 4);
  float* dout = (float*)c.take(nn * 4);
  uint32_t* dw = (uint32_t*)c.take(nwn * 4);
  int64_t* doff = (int64_t*)c.take(16);
  int64_t* dhdr = (int64_t*)c.take(16);  // word offset 0, word count
  uint64_t* dst = (uint64_t*)c.take(8);
  uint64_t* dfs = (uint64_t*)c.take(8);
  int32_t* dstat = (int32_t*)c.take(4);
  (void)c.take(8);
  (void)c.take(8);
  void* kws = c.take((size_t)idf_rans_decode_workspace_bytes(n));
  if (!kws) return IDF_ERR_ARG;
  int rc = IDF_OK;
  const int64_t off[2] = {0, n}, hdr[2] = {0, nwords};
  if (n > 0) {
    CK(hipMemcpyAsync(dm, mean, n * 4, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(ds, scale, n * 4, hipMemcpyHostToDevice, s));
  }
  if (nwords > 0) CK(hipMemcpyAsync(dw, words, nwords * 4, hipMemcpyHostToDevice, s));
  CK(hipMemcpyAsync(doff, off, 16, hipMemcpyHostToDevice, s));
  CK(hipMemcpyAsync(dhdr, hdr, 16, hipMemcpyHostToDevice, s));
  CK(hipMemcpyAsync(dst, state_io, 8, hipMemcpyHostToDevice, s));
  if (rc == IDF_OK)
    rc = idf_rans_decode_streams(s, 1, n, doff, dhdr, dhdr + 1, dw, dm, ds, dst, dfs, dout,
                                 dstat, kws, idf_rans_decode_workspace_bytes(n));
  int32_t stat = 0;
  uint64_t fs = 0;
  if (rc == IDF_OK) {
    CK(hipMemcpyAsync(&fs, dfs, 8, hipMemcpyDeviceToHost, s));
    CK(hipMemcpyAsync(&stat, dstat, 4, hipMemcpyDeviceToHost, s));
    if (n > 0) CK(hipMemcpyAsync(out, dout, n * 4, hipMemcpyDeviceToHost, s));
  }
  CK(hipStreamSynchronize(s));
  if (rc == IDF_OK) *state_io = fs;
  if (status_out) *status_out = stat;
  return rc;
}

int idf_rans_encode(uint64_t* state_io, int64_t n, const float* x, const float* mean,
                    const float* scale, uint32_t* words, int64_t* nwords_out, int32_t* status_out) {
  if (n < 0 || !state_io) return IDF_ERR_ARG;
  HostCtx* ctx = nullptr;
  const int64_t need = idf_rans_host_workspace_bytes(n, 0);
  int rc = host_ctx(need, &ctx);
  if (rc != IDF_OK) return rc;
  return idf_rans_encode_on(ctx->stream, ctx->ws, ctx->ws_bytes, state_io, n, x, mean, scale,
                            words, nwords_out, status_out);
}

int idf_rans_decode(uint64_t* state_io, const uint32_t* words, int64_t nwords, int64_t n,
                    const float* mean, const float* scale, float* out, int32_t* status_out) {
  if (n < 0 || nwords < 0 || !state_io) return IDF_ERR_ARG;
  HostCtx* ctx = nullptr;
  const int64_t need = idf_rans_host_workspace_bytes(n, nwords);
  int rc = host_ctx(need, &ctx);
  if (rc != IDF_OK) return rc;
  return idf_rans_decode_on(ctx->stream, ctx->ws, ctx->ws_bytes, state_io, words, nwords, n,
                            mean, scale, out, status_out);
}

}  // extern "C"
