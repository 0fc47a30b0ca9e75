// vq_kernels.hip -- the VQ-VAE of the residual configs (configs 3-5; vqvae.py:22-168,
// roundlib.py:41-89, extenddim.py:40-67) on gfx950.
//
// Activations are pixel-major ("NHWC") like the flow engine.  Every convolution of the
// VQ-VAE -- Conv2d 4x4/s2/p1 and 3x3/p1 and 1x1 (VQEncoder), the ResBlock convs
// (nnblock.py:59-84), and ConvTranspose2d 4x4/s2/p1 (VQDecoder) -- is one implicit GEMM
// over a TAP TABLE: an output pixel on a "compute grid" (m, n) reads input pixels
// (m*isy + dy[t], n*isx + dx[t]) for each tap t, and is written to output pixel
// (m*osy + oy0, n*osx + ox0).  A stride-2 transposed conv is four such launches, one per
// output parity class (each a 2x2-tap conv), so no zero-stuffed input is ever read.
// K is ordered channel-slab-major, tap-minor (a slab's taps re-read the same lines from
// L1/L2), the reduction order depends only on the weights' shape, and the epilogue fuses
// bias, an optional residual add (ResBlock: act(x + conv)) and the activation.
//
// The vector quantiser (roundlib.py:56-62) is one fused kernel: a block streams 64 latent
// rows and a slice of the codebook through MFMA tiles and keeps a running (distance, index)
// minimum per row -- the [rows x 16384] distance matrix never exists.
// Distances are formed as the reference does, d = (|x|^2 + |e|^2) - 2 x.e in fp32, and
// ties go to the lowest index (torch.argmin).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>
#include <type_traits>

#include "idf_codec_internal.h"

#pragma clang fp contract(off)

namespace idf {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int kMaxTaps = 16;

struct ConvTapsArgs {
  const float* X;
  int64_t ldx;
  int32_t B, Hi, Wi, C;
  int32_t Hc, Wc;  // compute grid per image
  int32_t isy, isx;
  int32_t ntaps;
  int32_t dy[kMaxTaps], dx[kMaxTaps];
  const float* W;  // [n_alloc][ntaps][ldw]
  int32_t ldw;
  const float* bias;
  int32_t N;
  float* out;
  int64_t ldo;
  int32_t Ho, Wo, osy, osx, oy0, ox0;
  const float* res;  // optional, indexed like out
  int64_t ldr;
  int32_t act;
  float slope;
  int64_t P;  // B * Hc * Wc
  int32_t m_tiles, n_tiles;
  // X3 (split-f16 products): W holds per 4 channels (wh[4], wl[4]) f16 of w * 2^k (the same 16
  // bytes as 4 fp32 weights), yscale = 2^-k; flag: bit 0 set when an input value is NaN or
  // |x| >= 32768 (the f16 pairs' range; the caller recomputes in fp32)
  float yscale;
  uint32_t* flag;
};

// f(integral_constant<int, T>) for T = 0 .. N - 1 in order
template <int N, typename F, int... T>
__device__ __forceinline__ void dx_taps_unroll_impl(F&& f, std::integer_sequence<int, T...>) {
  (f(std::integral_constant<int, T>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void dx_taps_unroll(F&& f) {
  dx_taps_unroll_impl<N>(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ float vq_act(float v, int act, float slope) {
  if (act == IDF_ACT_RELU) return v > 0.0f ? v : 0.0f;
  if (act == IDF_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  if (act == IDF_ACT_TANH) return tanhf(v);
  return v;
}

// X3 = true: the same GEMM with every fp32 product as three f16 products on
// v_mfma_f32_16x16x16_f16 (x = xh + xl split when the tile is staged, the weights pre-split on
// the host): xh.wh + xl.wh + xh.wl per k-step, fp32 accumulation -- the split-f16 arithmetic of
// the flow's dx3 / wx3 convs, 1/16 of the MFMA cycles of the fp32 16x16x4 steps it replaces.
// R: k-chunks whose global loads are in flight in registers (R - 1 ahead of the chunk being
// multiplied; two LDS stages either way).  Which chunk meets which accumulator in which order
// does not depend on R: the outputs are bit-identical for every R.
#ifndef IDF_TAPS_PREFETCH
#define IDF_TAPS_PREFETCH 3
#endif
template <int BM, int BN, int WAVES_M, int WAVES_N, bool X3, int R>
__global__ void __launch_bounds__(256) conv_taps_kernel(ConvTapsArgs g) {
  constexpr int BK = 16;
  constexpr int LDS_LD = BK + 8;  // conflict-free b128 fragment reads
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int A_PER_T = BM * 4 / 256;
  constexpr int B_F4 = BN * 4;
  constexpr int B_PER_T = (B_F4 + 255) / 256;
  static_assert(WAVES_M * WAVES_N == 4 && FM >= 1 && FN >= 1, "tile");

  __shared__ __attribute__((aligned(16))) float As[2][BM][LDS_LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LDS_LD];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid = xcd_contiguous(blockIdx.x, gridDim.x);  // neighbouring row tiles on one XCD
  const int mt = bid / g.n_tiles, nt = bid % g.n_tiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int64_t hwc = (int64_t)g.Hc * g.Wc;

  int a_row[A_PER_T], a_kq[A_PER_T], a_b[A_PER_T], a_m[A_PER_T], a_n[A_PER_T];
  bool a_ok[A_PER_T];
#pragma unroll
  for (int j = 0; j < A_PER_T; ++j) {
    const int f = tid + 256 * j;
    a_row[j] = f >> 2;
    a_kq[j] = f & 3;
    const int64_t p = m0 + a_row[j];
    a_ok[j] = p < g.P;
    const int64_t pp = a_ok[j] ? p : 0;
    a_b[j] = (int)(pp / hwc);
    const int64_t rem = pp - (int64_t)a_b[j] * hwc;
    a_m[j] = (int)(rem / g.Wc);
    a_n[j] = (int)(rem - (int64_t)a_m[j] * g.Wc);
  }
  const int nslab = (g.C + BK - 1) / BK;
  const int nk = nslab * g.ntaps;
  f4 ra_s[R][A_PER_T], rb_s[R][B_PER_T];

  auto load_chunk = [&](int kc, f4 (&ra)[A_PER_T], f4 (&rb)[B_PER_T]) {
    const int slab = kc / g.ntaps, tap = kc - slab * g.ntaps, c0 = slab * BK;
    const int dy = g.dy[tap], dx = g.dx[tap];
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
      const int c = c0 + 4 * a_kq[j];
      const int iy = a_m[j] * g.isy + dy, ix = a_n[j] * g.isx + dx;
      const bool ok = a_ok[j] && c < g.C && iy >= 0 && iy < g.Hi && ix >= 0 && ix < g.Wi;
      ra[j] = ok ? *(const f4*)(g.X + (((int64_t)a_b[j] * g.Hi + iy) * g.Wi + ix) * g.ldx + c)
                 : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      const int f = tid + 256 * j;
      if (f < B_F4) {
        const int n = f >> 2, kq = f & 3;
        rb[j] = *(const f4*)(g.W + ((int64_t)(n0 + n) * g.ntaps + tap) * g.ldw + c0 + 4 * kq);
      }
    }
  };
  bool in_ok = true;
  auto store_chunk = [&](int buf, const f4 (&ra)[A_PER_T], const f4 (&rb)[B_PER_T]) {
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
      if constexpr (X3) {  // (xh[4], xl[4]) in the 16 bytes of the 4 fp32 values
        const f4 v = ra[j];
        in_ok = in_ok && fabsf(v[0]) < 32768.0f && fabsf(v[1]) < 32768.0f &&
                fabsf(v[2]) < 32768.0f && fabsf(v[3]) < 32768.0f;
        const h4 hi = __builtin_convertvector(v, h4);
        const h4 lo = __builtin_convertvector(v - __builtin_convertvector(hi, f4), h4);
        typedef _Float16 h8 __attribute__((ext_vector_type(8)));
        *(h8*)&As[buf][a_row[j]][4 * a_kq[j]] =
            h8{hi[0], hi[1], hi[2], hi[3], lo[0], lo[1], lo[2], lo[3]};
      } else {
        *(f4*)&As[buf][a_row[j]][4 * a_kq[j]] = ra[j];
      }
    }
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      const int f = tid + 256 * j;
      if (f < B_F4) *(f4*)&Bs[buf][f >> 2][4 * (f & 3)] = rb[j];
    }
  };

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int j = 0; j < R - 1; ++j)
    if (j < nk) load_chunk(j, ra_s[j], rb_s[j]);
  store_chunk(0, ra_s[0], rb_s[0]);
  __syncthreads();
  const int lr = lane & 15, lk = 4 * (lane >> 4);
  auto step = [&](int kc, f4 (&ra_next)[A_PER_T], f4 (&rb_next)[B_PER_T],
                  const f4 (&ra_st)[A_PER_T], const f4 (&rb_st)[B_PER_T]) {
    const int buf = kc & 1;
    if (kc + R - 1 < nk) load_chunk(kc + R - 1, ra_next, rb_next);
    f4 fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = *(const f4*)&As[buf][wm * WTM + i * 16 + lr][lk];
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = *(const f4*)&Bs[buf][wn * WTN + j * 16 + lr][lk];
    if constexpr (X3) {
      // lane: row lr, k = lk .. lk + 3 -- the A / B layout of v_mfma_f32_16x16x16_f16
      typedef _Float16 h8 __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const h8 a8 = __builtin_bit_cast(h8, fa[i]);
        const h4 ah = h4{a8[0], a8[1], a8[2], a8[3]}, al = h4{a8[4], a8[5], a8[6], a8[7]};
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const h8 b8 = __builtin_bit_cast(h8, fb[j]);
          const h4 bh = h4{b8[0], b8[1], b8[2], b8[3]}, bl = h4{b8[4], b8[5], b8[6], b8[7]};
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(al, bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bl, acc[i][j], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][t], fb[j][t], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) store_chunk(buf ^ 1, ra_st, rb_st);
    __syncthreads();
  };
  for (int kc0 = 0; kc0 < nk; kc0 += R) {
    // chunk kc0 + t: loads chunk kc0 + t + R - 1 into set (t + R - 1) % R, stages chunk
    // kc0 + t + 1 from set (t + 1) % R (kc0 is a multiple of R)
    dx_taps_unroll<R>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if (kc0 + t < nk)
        step(kc0 + t, ra_s[(t + R - 1) % R], rb_s[(t + R - 1) % R], ra_s[(t + 1) % R],
             rb_s[(t + 1) % R]);
    });
  }

  // bias loads first (a load after a store to a possibly aliasing pointer would wait for it),
  // then one pixel decomposition per output row (32-bit: the host caps P below 2^31)
  float bv[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * WTN + j * 16 + lr;
    bv[j] = g.bias && n < g.N ? g.bias[n] : 0.0f;
  }
  const uint32_t hwc32 = (uint32_t)hwc, wc32 = (uint32_t)g.Wc;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t p = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
      if (p >= g.P) continue;
      const uint32_t p32 = (uint32_t)p;
      const uint32_t b = p32 / hwc32, rem = p32 - b * hwc32;
      const uint32_t m = rem / wc32, nn = rem - m * wc32;
      const int64_t o = ((int64_t)b * g.Ho + (int64_t)m * g.osy + g.oy0) * g.Wo +
                        (int64_t)nn * g.osx + g.ox0;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + lr;
        if (n >= g.N) continue;
        float v = (X3 ? acc[i][j][r] * g.yscale : acc[i][j][r]) + bv[j];
        if (g.res) v = g.res[o * g.ldr + n] + v;  // ResBlock: x + resblock(x) (nnblock.py:81-82)
        g.out[o * g.ldo + n] = vq_act(v, g.act, g.slope);
      }
    }
  if (X3 && !in_ok && g.flag) atomicOr(g.flag, 1u);
}

template <int BN, bool X3>
static int launch_taps(ConvTapsArgs a, hipStream_t s) {
  constexpr int WN = BN >= 64 ? 2 : 1;
  constexpr int WM = 4 / WN;
  constexpr int BM = 64;
  a.m_tiles = (int)((a.P + BM - 1) / BM);
  a.n_tiles = (a.N + BN - 1) / BN;
  hipLaunchKernelGGL((conv_taps_kernel<BM, BN, WM, WN, X3, IDF_TAPS_PREFETCH>),
                     dim3((unsigned)(a.m_tiles * a.n_tiles)),
                     dim3(256), 0, s, a);
  return idf_last_error();
}

// ---------------------------------------------------------------- vector quantiser
// rows [P][ldx] (D columns), codebook E [K][lde], enorm[k] = |e_k|^2 (fp32, sum in index
// order).  idx[p] = argmin_k ((|x|^2 + enorm[k]) - 2 x.e_k), lowest k on ties.
//
// Block = 4 waves over 64 rows x 128 codes per code tile (wave: 32 rows x 64 codes, 2 x 4
// accumulator fragments of v_mfma_f32_16x16x4_f32); rows and codes stream through LDS in
// 16-deep k-chunks (two stages, the next chunk's global loads in flight during the current
// chunk's 32 MFMAs), so three blocks share a CU.  Blocks split the codebook into S slices:
// block b takes slice b % S (consecutive blocks land on different XCDs, so an XCD keeps its
// slice of E in its own L2) and row tile b / S; slices' (distance, index) minima are merged
// in slice order by vq_argmin_merge_kernel.  Per (row, code) the MFMA chain is the same for
// every S: k-chunk c, step t, lane group g multiplying k = 16c + 4g + t -- the index is
// independent of the launch shape.
constexpr int kVqBM = 64, kVqBN = 128, kVqBK = 16, kVqPitch = kVqBK + 8;
constexpr int kVqMaxSlices = 8;

__device__ __forceinline__ bool vq_better(float d, int k, float bd, int bk) {
  return d < bd || (d == bd && k < bk);  // NaN never wins
}

// X3 = true: x.e with split-f16 products (xh.eh + xl.eh + xh.el on v_mfma_f32_16x16x16_f16, fp32
// accumulation; E pre-split on the host as (eh[4], el[4]) per 4 channels of E * 2^k, yscale =
// 2^-k), |x|^2 and |e|^2 still fp32 in index order; an input value past the f16 pairs' range
// (NaN or |x| >= 32768) ORs bit 0 into flag (the caller searches again in fp32).
template <bool X3>
__global__ void __launch_bounds__(256) vq_argmin_kernel(int64_t P, int32_t D, const float* __restrict__ X,
                                                        int64_t ldx, const float* __restrict__ E,
                                                        int32_t lde, int32_t K,
                                                        const float* __restrict__ enorm, int32_t S,
                                                        int32_t slice_codes,
                                                        float* __restrict__ part_d,
                                                        int32_t* __restrict__ part_i,
                                                        int32_t* __restrict__ idx, float yscale,
                                                        uint32_t* __restrict__ flag) {
  __shared__ __attribute__((aligned(16))) float As[2][kVqBM][kVqPitch];
  __shared__ __attribute__((aligned(16))) float Bs[2][kVqBN][kVqPitch];
  __shared__ float x2s[kVqBM];
  __shared__ float red_d[kVqBM];
  __shared__ int red_i[kVqBM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave & 1, wc = wave >> 1;
  const int slice = (int)(blockIdx.x % (unsigned)S);
  const int64_t m0 = (int64_t)(blockIdx.x / (unsigned)S) * kVqBM;
  const int kb = slice * slice_codes;
  const int ke = kb + slice_codes < K ? kb + slice_codes : K;
  const int lr = lane & 15, lk = 4 * (lane >> 4);
  const int nkc = (D + kVqBK - 1) / kVqBK;
  // staging: A chunk 64 x 16 = one f4 per thread, B chunk 128 x 16 = two
  const int ar = tid >> 2, aq = 4 * (tid & 3);
  f4 ra, rb0, rb1;
  auto load = [&](int k0, int kc) {
    const int c = kc * kVqBK + aq;
    const int64_t p = m0 + ar;
    ra = (p < P && c < D) ? *(const f4*)(X + p * ldx + c) : f4{0.f, 0.f, 0.f, 0.f};
    const int n0 = k0 + ar, n1 = k0 + 64 + ar;
    rb0 = (n0 < ke && c < D) ? *(const f4*)(E + (int64_t)n0 * lde + c) : f4{0.f, 0.f, 0.f, 0.f};
    rb1 = (n1 < ke && c < D) ? *(const f4*)(E + (int64_t)n1 * lde + c) : f4{0.f, 0.f, 0.f, 0.f};
  };
  bool in_ok = true;
  auto store = [&](int buf) {
    if constexpr (X3) {  // (xh[4], xl[4]) in the 16 bytes of the 4 fp32 values
      typedef _Float16 h8 __attribute__((ext_vector_type(8)));
      in_ok = in_ok && fabsf(ra[0]) < 32768.0f && fabsf(ra[1]) < 32768.0f &&
              fabsf(ra[2]) < 32768.0f && fabsf(ra[3]) < 32768.0f;
      const h4 hi = __builtin_convertvector(ra, h4);
      const h4 lo = __builtin_convertvector(ra - __builtin_convertvector(hi, f4), h4);
      *(h8*)&As[buf][ar][aq] = h8{hi[0], hi[1], hi[2], hi[3], lo[0], lo[1], lo[2], lo[3]};
    } else {
      *(f4*)&As[buf][ar][aq] = ra;
    }
    *(f4*)&Bs[buf][ar][aq] = rb0;
    *(f4*)&Bs[buf][64 + ar][aq] = rb1;
  };
  float best[2][4];
  int bidx[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      best[i][r] = __builtin_inff();
      bidx[i][r] = 0x7fffffff;
    }
  float x2acc = 0.0f;  // thread tid < 64: |x_row|^2 in index order, formed on the first tile
  bool first = true;
  if constexpr (X3) {  // (the staged tile holds halves): from the rows themselves, same order
    if (tid < kVqBM && m0 + tid < P) {
      const float* xr = X + (m0 + tid) * ldx;
      for (int c = 0; c < D; ++c) x2acc = __builtin_fmaf(xr[c], xr[c], x2acc);
    }
  }
  for (int k0 = kb; k0 < ke; k0 += kVqBN) {
    f4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    load(k0, 0);
    store(0);
    __syncthreads();
    for (int kc = 0; kc < nkc; ++kc) {
      const int buf = kc & 1;
      if (kc + 1 < nkc) load(k0, kc + 1);
      f4 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *(const f4*)&As[buf][wr * 32 + i * 16 + lr][lk];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *(const f4*)&Bs[buf][wc * 64 + j * 16 + lr][lk];
      if (!X3 && first && tid < kVqBM) {
        const int cn = D - kc * kVqBK < kVqBK ? D - kc * kVqBK : kVqBK;
        for (int c = 0; c < cn; ++c) x2acc = __builtin_fmaf(As[buf][tid][c], As[buf][tid][c], x2acc);
      }
      if constexpr (X3) {
        typedef _Float16 h8 __attribute__((ext_vector_type(8)));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const h8 a8 = __builtin_bit_cast(h8, fa[i]);
          const h4 ah = h4{a8[0], a8[1], a8[2], a8[3]}, al = h4{a8[4], a8[5], a8[6], a8[7]};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const h8 b8 = __builtin_bit_cast(h8, fb[j]);
            const h4 bh = h4{b8[0], b8[1], b8[2], b8[3]}, bl = h4{b8[4], b8[5], b8[6], b8[7]};
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bh, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(al, bh, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bl, acc[i][j], 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][t], fb[j][t], acc[i][j], 0, 0, 0);
      }
      if (kc + 1 < nkc) store(buf ^ 1);
      __syncthreads();
    }
    if (first) {
      if (tid < kVqBM) x2s[tid] = x2acc;
      __syncthreads();
      first = false;
    }
    // lane holds rows wr*32 + i*16 + (lane>>4)*4 + r, code k0 + wc*64 + j*16 + (lane&15)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wc * 64 + j * 16 + lr;
      if (k >= ke) continue;
      const float en = enorm[k];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x2 = x2s[wr * 32 + i * 16 + (lane >> 4) * 4 + r];
          const float d = (x2 + en) - 2.0f * (X3 ? acc[i][j][r] * yscale : acc[i][j][r]);
          if (vq_better(d, k, best[i][r], bidx[i][r])) {
            best[i][r] = d;
            bidx[i][r] = k;
          }
        }
    }
  }
  if (X3 && !in_ok && flag) atomicOr(flag, 1u);
  // reduce over the 16 lanes sharing each row (lanes differ in code column), then the two
  // waves sharing each row (code halves)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float ov = __shfl_xor(best[i][r], o);
        const int oi = __shfl_xor(bidx[i][r], o);
        if (vq_better(ov, oi, best[i][r], bidx[i][r])) {
          best[i][r] = ov;
          bidx[i][r] = oi;
        }
      }
  if (wc == 1 && lr == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + i * 16 + (lane >> 4) * 4 + r;
        red_d[row] = best[i][r];
        red_i[row] = bidx[i][r];
      }
  }
  __syncthreads();
  if (wc == 0 && lr == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + i * 16 + (lane >> 4) * 4 + r;
        float bd = best[i][r];
        int bk = bidx[i][r];
        if (vq_better(red_d[row], red_i[row], bd, bk)) {
          bd = red_d[row];
          bk = red_i[row];
        }
        const int64_t p = m0 + row;
        if (p >= P) continue;
        if (S == 1) {
          idx[p] = bk;
        } else {
          part_d[(int64_t)slice * P + p] = bd;
          part_i[(int64_t)slice * P + p] = bk;
        }
      }
  }
}

// the slices' minima in slice order (lowest index on equal distances)
__global__ void vq_argmin_merge_kernel(int64_t P, int32_t S, const float* __restrict__ part_d,
                                       const int32_t* __restrict__ part_i, int32_t* __restrict__ idx) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  float bd = part_d[p];
  int bk = part_i[p];
  for (int s = 1; s < S; ++s) {
    const float d = part_d[(int64_t)s * P + p];
    const int k = part_i[(int64_t)s * P + p];
    if (vq_better(d, k, bd, bk)) {
      bd = d;
      bk = k;
    }
  }
  idx[p] = bk;
}

// |e_k|^2 in index order (the reference's torch.sum(weight**2, dim=1) up to summation order)
__global__ void vq_norms_kernel(int32_t K, int32_t D, const float* __restrict__ E, int32_t lde,
                                float* __restrict__ enorm) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float s = 0.0f;
  for (int c = 0; c < D; ++c) s = __builtin_fmaf(E[(int64_t)k * lde + c], E[(int64_t)k * lde + c], s);
  enorm[k] = s;
}

// out[p, c] = E[idx[p], c] (nn.Embedding lookup, vqvae.py:58 / roundlib.py:63)
__global__ void vq_gather_kernel(int64_t P, int32_t D, const int32_t* __restrict__ idx,
                                 const float* __restrict__ E, int32_t lde, float* __restrict__ out,
                                 int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * D) return;
  const int64_t p = i / D;
  const int c = (int)(i - p * D);
  out[p * ldo + c] = E[(int64_t)idx[p] * lde + c];
}

// y[p, c] = op(x[p, c]) on pixel-major buffers:
// 0: (x - 0.5) / 0.5            (trainer.py:606 input scaling)
// 1: rint((x * 0.5 + 0.5) * 256) / 256   (trainer.py:606-607: rescale + model.round)
// 2: x - z                      (trainer.py:608: res = data - rec)
// 3: x + z                      (decode: data = res + rec)
__global__ void vq_pointwise_kernel(int64_t P, int32_t C, int32_t op, const float* __restrict__ x,
                                    int64_t ldx, const float* __restrict__ z, int64_t ldz,
                                    float* __restrict__ y, int64_t ldy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * C) return;
  const int64_t p = i / C;
  const int c = (int)(i - p * C);
  const float v = x[p * ldx + c];
  float r;
  if (op == 0) r = (v - 0.5f) / 0.5f;
  else if (op == 1) r = __builtin_rintf((v * 0.5f + 0.5f) * 256.0f) / 256.0f;
  else if (op == 2) r = v - z[p * ldz + c];
  else r = v + z[p * ldz + c];
  y[p * ldy + c] = r;
}

// Patching.forward (extenddim.py:52-58) on NCHW: [B, C, H, W] -> [B*(H/h)*(W/w), C, h, w];
// inverse = backward (extenddim.py:60-67).
__global__ void patch_kernel(int32_t B, int32_t C, int32_t H, int32_t W, int32_t h, int32_t w,
                             int32_t inverse, const float* __restrict__ src, float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)B * C * H * W;
  if (i >= total) return;
  // i indexes the image layout [B][C][H][W]
  const int x = (int)(i % W);
  int64_t t = i / W;
  const int y = (int)(t % H);
  t /= H;
  const int c = (int)(t % C);
  const int64_t b = t / C;
  const int hh = H / h, ww = W / w;
  const int64_t q = (b * hh + y / h) * ww + x / w;  // patch index
  const int64_t j = ((q * C + c) * h + (y % h)) * w + (x % w);
  if (inverse) dst[i] = src[j];
  else dst[j] = src[i];
}

// ReplicationPad2d(padding=(0, right, 0, bottom)) of uint8 NCHW images (trainer.py:62,69-70:
// the dataloader pads the right/bottom edges by replication before Round) when Ho >= Hi and
// Wo >= Wi; the same map with Ho <= Hi, Wo <= Wi is the crop that undoes it.
__global__ void pad_edge_u8_kernel(int64_t total, int32_t Hi, int32_t Wi, int32_t Ho, int32_t Wo,
                                   const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = (int)(i % Wo);
  const int64_t t = i / Wo;
  const int y = (int)(t % Ho);
  const int64_t bc = t / Ho;
  dst[i] = src[(bc * Hi + min(y, Hi - 1)) * Wi + min(x, Wi - 1)];
}

// Fixed-width index code (the VQ indices of the residual configs):
// indices come in groups (one image each) of `per` indices; group g starts at word
// g * wpg (wpg = ceil(per * bits / 32)), and its index j occupies bits
// [j*bits, (j+1)*bits) of that little-endian word run -- so shards concatenate.
__global__ void pack_bits_kernel(int64_t n, int64_t per, int64_t wpg, int32_t bits,
                                 const int32_t* __restrict__ idx, uint32_t* __restrict__ words) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = i / per, j = i - g * per;
  const uint64_t v = (uint64_t)(uint32_t)idx[i] & ((1ull << bits) - 1);
  const uint64_t b0 = (uint64_t)j * bits;
  const int64_t w = g * wpg + (int64_t)(b0 >> 5);
  const int sh = (int)(b0 & 31);
  atomicOr(&words[w], (uint32_t)(v << sh));
  if (sh + bits > 32) atomicOr(&words[w + 1], (uint32_t)(v >> (32 - sh)));
}

__global__ void unpack_bits_kernel(int64_t n, int64_t per, int64_t wpg, int32_t bits,
                                   const uint32_t* __restrict__ words, int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = i / per, j = i - g * per;
  const uint64_t b0 = (uint64_t)j * bits;
  const int64_t w = g * wpg + (int64_t)(b0 >> 5);
  const int sh = (int)(b0 & 31);
  uint64_t v = words[w] >> sh;
  if (sh + bits > 32) v |= (uint64_t)words[w + 1] << (32 - sh);
  idx[i] = (int32_t)(v & ((1ull << bits) - 1));
}

}  // namespace idf

using namespace idf;

extern "C" {

static int conv_taps_run(bool x3, void* stream, int32_t B, int32_t Hi, int32_t Wi, int32_t C,
                         const float* x, int64_t ld_x, int32_t Hc, int32_t Wc, int32_t isy,
                         int32_t isx, int32_t ntaps, const int32_t* dy, const int32_t* dx,
                         const float* w, int32_t ldw, int32_t n_alloc, const float* bias, int32_t N,
                         float* out, int64_t ld_out, int32_t Ho, int32_t Wo, int32_t osy,
                         int32_t osx, int32_t oy0, int32_t ox0, const float* res, int64_t ld_res,
                         int32_t act, float slope, float yscale, uint32_t* d_flag) {
  if (B <= 0 || Hc <= 0 || Wc <= 0 || N <= 0) return IDF_OK;
  if (ntaps < 1 || ntaps > kMaxTaps || C <= 0 || (C & 3) || (ld_x & 3) || (ldw & 15) ||
      ldw < ((C + 15) / 16) * 16 || !dy || !dx || !x || !w || !out)
    return IDF_ERR_ARG;
  ConvTapsArgs a = {};
  a.X = x; a.ldx = ld_x; a.B = B; a.Hi = Hi; a.Wi = Wi; a.C = C; a.Hc = Hc; a.Wc = Wc;
  a.isy = isy; a.isx = isx; a.ntaps = ntaps;
  for (int t = 0; t < ntaps; ++t) {
    a.dy[t] = dy[t];
    a.dx[t] = dx[t];
  }
  a.W = w; a.ldw = ldw; a.bias = bias; a.N = N; a.out = out; a.ldo = ld_out;
  a.Ho = Ho; a.Wo = Wo; a.osy = osy; a.osx = osx; a.oy0 = oy0; a.ox0 = ox0;
  a.res = res; a.ldr = ld_res; a.act = act; a.slope = slope;
  a.yscale = yscale; a.flag = d_flag;
  a.P = (int64_t)B * Hc * Wc;
  if (a.P >= ((int64_t)1 << 31)) return IDF_ERR_UNSUPPORTED;  // 32-bit pixel decomposition
  const int bn = N <= 32 ? 32 : (N <= 64 ? 64 : 128);
  if (n_alloc < ((N + bn - 1) / bn) * bn) return IDF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (x3) {
    if (bn == 32) return launch_taps<32, true>(a, s);
    if (bn == 64) return launch_taps<64, true>(a, s);
    return launch_taps<128, true>(a, s);
  }
  if (bn == 32) return launch_taps<32, false>(a, s);
  if (bn == 64) return launch_taps<64, false>(a, s);
  return launch_taps<128, false>(a, s);
}

int idf_conv_taps_f32(void* stream, int32_t B, int32_t Hi, int32_t Wi, int32_t C, const float* x,
                      int64_t ld_x, int32_t Hc, int32_t Wc, int32_t isy, int32_t isx, int32_t ntaps,
                      const int32_t* dy, const int32_t* dx, const float* w, int32_t ldw,
                      int32_t n_alloc, const float* bias, int32_t N, float* out, int64_t ld_out,
                      int32_t Ho, int32_t Wo, int32_t osy, int32_t osx, int32_t oy0, int32_t ox0,
                      const float* res, int64_t ld_res, int32_t act, float slope) {
  return conv_taps_run(false, stream, B, Hi, Wi, C, x, ld_x, Hc, Wc, isy, isx, ntaps, dy, dx, w,
                       ldw, n_alloc, bias, N, out, ld_out, Ho, Wo, osy, osx, oy0, ox0, res, ld_res,
                       act, slope, 1.0f, nullptr);
}

int idf_conv_taps_x3(void* stream, int32_t B, int32_t Hi, int32_t Wi, int32_t C, const float* x,
                     int64_t ld_x, int32_t Hc, int32_t Wc, int32_t isy, int32_t isx, int32_t ntaps,
                     const int32_t* dy, const int32_t* dx, const uint16_t* w, int32_t ldw,
                     int32_t n_alloc, float yscale, const float* bias, int32_t N, float* out,
                     int64_t ld_out, int32_t Ho, int32_t Wo, int32_t osy, int32_t osx, int32_t oy0,
                     int32_t ox0, const float* res, int64_t ld_res, int32_t act, float slope,
                     uint32_t* d_flag) {
  return conv_taps_run(true, stream, B, Hi, Wi, C, x, ld_x, Hc, Wc, isy, isx, ntaps, dy, dx,
                       (const float*)w, ldw, n_alloc, bias, N, out, ld_out, Ho, Wo, osy, osx, oy0,
                       ox0, res, ld_res, act, slope, yscale, d_flag);
}

int idf_conv_taps_n_alloc(int32_t N) {
  const int bn = N <= 32 ? 32 : (N <= 64 ? 64 : 128);
  return ((N + bn - 1) / bn) * bn;
}

int idf_vq_norms(void* stream, int32_t K, int32_t D, const float* e, int32_t lde, float* enorm) {
  if (K <= 0) return IDF_OK;
  hipLaunchKernelGGL(vq_norms_kernel, dim3((K + 255) / 256), dim3(256), 0, (hipStream_t)stream, K, D,
                     e, lde, enorm);
  return idf_last_error();
}

static int vq_slices(int64_t P, int32_t K) {
  // enough blocks for ~3 per CU on 256 CUs, each slice at least two code tiles
  const int64_t tiles = (P + kVqBM - 1) / kVqBM;
  int S = 1;
  while (S < kVqMaxSlices && tiles * S < 768 && (int64_t)K >= (int64_t)(2 * S) * 2 * kVqBN) S *= 2;
  return S;
}

int64_t idf_vq_argmin_workspace_bytes(int64_t P, int32_t K) {
  const int S = P > 0 && K > 0 ? vq_slices(P, K) : 1;
  return S > 1 ? (int64_t)S * P * 8 : 0;
}

static int vq_argmin_run(bool x3, void* stream, int64_t P, int32_t D, const float* x, int64_t ld_x,
                         const float* e, int32_t lde, int32_t K, const float* enorm, int32_t* idx,
                         void* ws, int64_t ws_bytes, float yscale, uint32_t* d_flag) {
  if (P <= 0) return IDF_OK;
  if (D <= 0 || (D & 3) || (ld_x & 3) || (lde & 3) || K <= 0 || !x || !e || !enorm || !idx)
    return IDF_ERR_ARG;
  int S = vq_slices(P, K);
  if (!ws || ws_bytes < (int64_t)S * P * 8) S = 1;  // no room for the slices' minima
  // codes per slice, whole code tiles (the last slice may be short or empty)
  const int sc = S == 1 ? K : ((K + S - 1) / S + kVqBN - 1) / kVqBN * kVqBN;
  float* pd = (float*)ws;
  int32_t* pi = (int32_t*)(pd + (S > 1 ? (int64_t)S * P : 0));
  const int64_t blocks = (P + kVqBM - 1) / kVqBM * S;
  if (x3)
    hipLaunchKernelGGL(vq_argmin_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       P, D, x, ld_x, e, lde, K, enorm, S, sc, pd, pi, idx, yscale, d_flag);
  else
    hipLaunchKernelGGL(vq_argmin_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       P, D, x, ld_x, e, lde, K, enorm, S, sc, pd, pi, idx, 1.0f, nullptr);
  if (S > 1)
    hipLaunchKernelGGL(vq_argmin_merge_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, P, S, pd, pi, idx);
  return idf_last_error();
}

int idf_vq_argmin_ws(void* stream, int64_t P, int32_t D, const float* x, int64_t ld_x, const float* e,
                     int32_t lde, int32_t K, const float* enorm, int32_t* idx, void* ws,
                     int64_t ws_bytes) {
  return vq_argmin_run(false, stream, P, D, x, ld_x, e, lde, K, enorm, idx, ws, ws_bytes, 1.0f,
                       nullptr);
}

int idf_vq_argmin_x3_ws(void* stream, int64_t P, int32_t D, const float* x, int64_t ld_x,
                        const uint16_t* ex, int32_t lde, float yscale, int32_t K, const float* enorm,
                        int32_t* idx, void* ws, int64_t ws_bytes, uint32_t* d_flag) {
  return vq_argmin_run(true, stream, P, D, x, ld_x, (const float*)ex, lde, K, enorm, idx, ws,
                       ws_bytes, yscale, d_flag);
}

int idf_vq_argmin(void* stream, int64_t P, int32_t D, const float* x, int64_t ld_x, const float* e,
                  int32_t lde, int32_t K, const float* enorm, int32_t* idx) {
  return idf_vq_argmin_ws(stream, P, D, x, ld_x, e, lde, K, enorm, idx, nullptr, 0);
}

int idf_vq_gather(void* stream, int64_t P, int32_t D, const int32_t* idx, const float* e,
                  int32_t lde, float* out, int64_t ld_out) {
  const int64_t n = P * D;
  if (n <= 0) return IDF_OK;
  hipLaunchKernelGGL(vq_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P, D, idx, e, lde, out, ld_out);
  return idf_last_error();
}

int idf_vq_pointwise(void* stream, int64_t P, int32_t C, int32_t op, const float* x, int64_t ld_x,
                     const float* z, int64_t ld_z, float* y, int64_t ld_y) {
  const int64_t n = P * C;
  if (n <= 0) return IDF_OK;
  if (op < 0 || op > 3 || (op >= 2 && !z)) return IDF_ERR_ARG;
  hipLaunchKernelGGL(vq_pointwise_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P, C, op, x, ld_x, z, ld_z, y, ld_y);
  return idf_last_error();
}

int idf_patch(void* stream, int32_t B, int32_t C, int32_t H, int32_t W, int32_t h, int32_t w,
              int32_t inverse, const float* src, float* dst) {
  if (h <= 0 || w <= 0 || H % h || W % w) return IDF_ERR_ARG;
  const int64_t n = (int64_t)B * C * H * W;
  if (n <= 0) return IDF_OK;
  hipLaunchKernelGGL(patch_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, B, C, H, W, h, w, inverse, src, dst);
  return idf_last_error();
}

int idf_pad_edge_u8(void* stream, int32_t B, int32_t C, int32_t Hi, int32_t Wi, int32_t Ho,
                    int32_t Wo, const uint8_t* src, uint8_t* dst) {
  if (B < 0 || C < 0 || Hi <= 0 || Wi <= 0 || Ho <= 0 || Wo <= 0) return IDF_ERR_ARG;
  if ((Ho - Hi) * (long)(Wo - Wi) < 0) return IDF_ERR_ARG;  // pad both or crop both
  const int64_t n = (int64_t)B * C * Ho * Wo;
  if (n == 0) return IDF_OK;
  hipLaunchKernelGGL(pad_edge_u8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n, Hi, Wi, Ho, Wo, src, dst);
  return idf_last_error();
}

int64_t idf_pack_bits_words(int64_t groups, int64_t per, int32_t bits) {
  return groups * ((per * bits + 31) / 32);
}

int idf_pack_bits(void* stream, int64_t groups, int64_t per, int32_t bits, const int32_t* idx,
                  uint32_t* words) {
  if (bits < 1 || bits > 31 || groups < 0 || per < 0) return IDF_ERR_ARG;
  const int64_t n = groups * per;
  if (n == 0) return IDF_OK;
  if (hipMemsetAsync(words, 0, (size_t)idf_pack_bits_words(groups, per, bits) * 4,
                     (hipStream_t)stream) != hipSuccess)
    return IDF_ERR_HIP;
  hipLaunchKernelGGL(pack_bits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n, per, (per * bits + 31) / 32, bits, idx, words);
  return idf_last_error();
}

int idf_unpack_bits(void* stream, int64_t groups, int64_t per, int32_t bits, const uint32_t* words,
                    int32_t* idx) {
  if (bits < 1 || bits > 31 || groups < 0 || per < 0) return IDF_ERR_ARG;
  const int64_t n = groups * per;
  if (n == 0) return IDF_OK;
  hipLaunchKernelGGL(unpack_bits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n, per, (per * bits + 31) / 32, bits, words, idx);
  return idf_last_error();
}

}  // extern "C"
