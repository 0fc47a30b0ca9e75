// flow_kernels.hip -- CDNA4 (gfx950) fp32 kernels of the integer-discrete flow.
//
// The DenseBlock (nnblock.py:24-56, nnlayer.py:42-51) dominates the hot path:
// per layer a 1x1 conv (GEMM M=pixels, N=K=c) and a 3x3 conv (implicit GEMM
// M=pixels, N=growth, K=9c).  Both run on the f32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact fp32 fma chain, 64 FLOP/clk/SIMD = the fp32
// roofline of 157 TF/s).  Activations are pixel-major ("NHWC": one row of
// channels per pixel) so a GEMM row is one pixel and the DenseLayer concat is a
// column range of one preallocated feature buffer (no `cat`).
//
// GEMM tile: BM pixels x BN channels x BK=16, 4 waves.  Each wave owns a
// (BM/WAVES_M) x (BN/WAVES_N) sub-tile of 16x16 MFMA fragments.  A K-chunk of
// 16 is held per lane as one float4 of A (row lane&15, k = 4*(lane>>4)..+3) and
// one float4 of B; the 4 MFMAs of a chunk take element t of each float4 (the
// k <-> lane-group assignment is a bijection, so the sum is over all 16 k).
// LDS tiles are double-buffered, rows padded by 4 floats; the next chunk's
// global loads are in flight while the current chunk computes.  Blocks are
// remapped so that all N-tiles of one M-tile run on one XCD (shared A rows in
// that XCD's L2).
//
// Determinism: every output element is one fixed-order fma chain over k (chunk
// order, then t, then the MFMA's internal order) independent of the batch size
// or the tile's position, so encoder and decoder compute bit-identical coupling
// outputs -- the condition for an exact round trip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "idf_cdf.h"
#include "idf_codec_internal.h"

#pragma clang fp contract(off)

namespace idf {

typedef float floatx4 __attribute__((ext_vector_type(4)));

enum { MODE_DENSE = 0, MODE_CONV3 = 1 };
// EPI_ACT_FOLD: the 3x3 conv of a DenseLayer with its 1x1 conv folded in
// (W' = W3[tap] . W1 applied to the layer input directly).  The 1x1 bias b1 then
// enters as v[tap] = W3[tap] . b1 for every tap whose neighbour lies inside the
// image (the reference zero-pads the 1x1 OUTPUT, nnlayer.py:43-45), so the bias
// of pixel (y, x) is b3 + sum of v over its valid taps; `bfull` holds that sum for
// interior pixels, computed in the same fp32 order as the border loop.
enum { EPI_STORE = 0, EPI_ACT = 1, EPI_COUPLE_ADD = 2, EPI_COUPLE_SUB = 3, EPI_PRIOR = 4,
       EPI_ACT_FOLD = 5 };

struct GemmArgs {
  int64_t P;        // rows (pixels)
  int32_t K;        // DENSE: reduction length; CONV3: input channels C
  int32_t N;        // valid output columns
  const float* A;   // DENSE: [P][lda]; CONV3: T [P][lda]
  int64_t lda;
  const float* W;   // DENSE: [n_alloc][ldw]; CONV3: [n_alloc][9][ldw]
  int32_t ldw;
  const float* bias;
  float* out;
  int64_t ldo;
  const float* base;  // COUPLE
  int64_t ldb;
  float* mean;        // PRIOR
  float* logscale;
  float* scale;
  int32_t n_mean;
  int32_t B, H, Wd;   // image geometry (CONV3 neighbours, PRIOR NCHW)
  int32_t act;
  float slope;
  const float* vtap;  // ACT_FOLD: [9][ldv] per-tap folded 1x1 bias
  const float* bfull; // ACT_FOLD: interior bias b3 + sum_tap vtap
  int32_t ldv;
  int32_t m_tiles, n_tiles;
};

__device__ __forceinline__ float apply_act(float v, int act, float slope) {
  if (act == IDF_ACT_RELU) return v > 0.0f ? v : 0.0f;
  if (act == IDF_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  if (act == IDF_ACT_TANH) return tanhf(v);
  return v;
}

// round to the 1/256 grid exactly as roundlib.py:34-38 (torch.round = half to even)
__device__ __forceinline__ float round8(float v) { return __builtin_rintf(v * 256.0f) / 256.0f; }

// bijective XCD-grouping remap (cdna_hip_programming.md T1): blocks that share
// bid % 8 get consecutive tile ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  int q = nwg / 8, r = nwg % 8;
  int xcd = bid % 8, idx = bid / 8;
  int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + idx;
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE, int EPI>
__global__ void __launch_bounds__(256) gemm_f32_kernel(GemmArgs g) {
  constexpr int BK = 16;
  constexpr int LDS_LD = BK + 8;  // 96-B rows: b128 fragment reads are bank-conflict free
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int A_F4 = BM * 4;                    // float4s per A chunk
  constexpr int B_F4 = BN * 4;
  constexpr int A_PER_T = A_F4 / 256;             // BM multiple of 64
  constexpr int B_PER_T = (B_F4 + 255) / 256;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert(FM >= 1 && FN >= 1 && WTM % 16 == 0 && WTN % 16 == 0, "tile");
  static_assert(A_F4 % 256 == 0, "BM multiple of 64");

  __shared__ __attribute__((aligned(16))) float As[2][BM][LDS_LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LDS_LD];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;

  const int nwg = g.m_tiles * g.n_tiles;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int mt = tile / g.n_tiles, nt = tile % g.n_tiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;

  // ---- per-thread A rows (fixed over the K loop)
  int a_row[A_PER_T], a_kq[A_PER_T];
  int64_t a_pix[A_PER_T];
  int a_y[A_PER_T], a_x[A_PER_T];
  bool a_ok[A_PER_T];
#pragma unroll
  for (int j = 0; j < A_PER_T; ++j) {
    int f = tid + 256 * j;
    a_row[j] = f >> 2;
    a_kq[j] = f & 3;
    int64_t p = m0 + a_row[j];
    a_ok[j] = p < g.P;
    a_pix[j] = p;
    if (MODE == MODE_CONV3) {
      int64_t hw = (int64_t)g.H * g.Wd;
      int64_t rem = p % hw;
      a_y[j] = (int)(rem / g.Wd);
      a_x[j] = (int)(rem % g.Wd);
    } else {
      a_y[j] = a_x[j] = 0;
    }
  }

  const int nkc = (g.K + BK - 1) / BK;               // chunks per tap (CONV3) or total
  const int nk = (MODE == MODE_CONV3) ? 9 * nkc : nkc;

  floatx4 ra[A_PER_T], rb[B_PER_T];

  auto load_chunk = [&](int kc) {
    int tap = 0, c0 = kc * BK;
    if (MODE == MODE_CONV3) {
      // channel-major, tap-minor: the 9 taps of one 16-channel slab are consecutive
      // chunks, so a slab's 9 shifted re-reads hit L1/L2 instead of HBM
      const int slab = kc / 9;
      tap = kc - slab * 9;
      c0 = slab * BK;
    }
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
      int c = c0 + 4 * a_kq[j];
      bool ok = a_ok[j] && c < g.K;
      const float* src = nullptr;
      if (MODE == MODE_CONV3) {
        int dy = tap / 3 - 1, dx = tap % 3 - 1;
        int ny = a_y[j] + dy, nx = a_x[j] + dx;
        ok = ok && ny >= 0 && ny < g.H && nx >= 0 && nx < g.Wd;
        src = g.A + (a_pix[j] + (int64_t)dy * g.Wd + dx) * g.lda + c;
      } else {
        src = g.A + a_pix[j] * g.lda + c;
      }
      ra[j] = ok ? *(const floatx4*)src : floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      int f = tid + 256 * j;
      if (f < B_F4) {
        int n = f >> 2, kq = f & 3;
        const float* src;
        if (MODE == MODE_CONV3)
          src = g.W + (int64_t)(n0 + n) * 9 * g.ldw + tap * g.ldw + c0 + 4 * kq;
        else
          src = g.W + (int64_t)(n0 + n) * g.ldw + c0 + 4 * kq;
        rb[j] = *(const floatx4*)src;
      }
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) *(floatx4*)&As[buf][a_row[j]][4 * a_kq[j]] = ra[j];
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      int f = tid + 256 * j;
      if (f < B_F4) *(floatx4*)&Bs[buf][f >> 2][4 * (f & 3)] = rb[j];
    }
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  const int lr = lane & 15, lk = 4 * (lane >> 4);
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < nk) load_chunk(kc + 1);
    floatx4 fa[FM], fb[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = *(const floatx4*)&As[buf][wm * WTM + i * 16 + lr][lk];
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = *(const floatx4*)&Bs[buf][wn * WTN + j * 16 + lr][lk];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][t], fb[j][t], acc[i][j], 0, 0, 0);
    if (kc + 1 < nk) store_chunk(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds rows (lane>>4)*4 + r, column lane&15 of each fragment
  const int64_t hw = (int64_t)g.H * g.Wd;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * WTN + j * 16 + lr;
    if (n >= g.N) continue;
    const float bv = g.bias[n];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t p = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
        if (p >= g.P) continue;
        float v = acc[i][j][r] + bv;
        if (EPI == EPI_STORE) {
          g.out[p * g.ldo + n] = v;
        } else if (EPI == EPI_ACT) {
          g.out[p * g.ldo + n] = apply_act(v, g.act, g.slope);
        } else if (EPI == EPI_ACT_FOLD) {
          const int64_t rem = p % hw;
          const int y = (int)(rem / g.Wd), x = (int)(rem % g.Wd);
          float bsum;
          if (y >= 1 && y <= g.H - 2 && x >= 1 && x <= g.Wd - 2) {
            bsum = g.bfull[n];
          } else {
            bsum = bv;  // b3, then + v[tap] for every in-image tap, fixed order
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
              const int ny = y + tap / 3 - 1, nx = x + tap % 3 - 1;
              if (ny >= 0 && ny < g.H && nx >= 0 && nx < g.Wd) bsum = bsum + g.vtap[tap * g.ldv + n];
            }
          }
          g.out[p * g.ldo + n] = apply_act(acc[i][j][r] + bsum, g.act, g.slope);
        } else if (EPI == EPI_COUPLE_ADD) {
          g.out[p * g.ldo + n] = g.base[p * g.ldb + n] + round8(v);
        } else if (EPI == EPI_COUPLE_SUB) {
          g.out[p * g.ldo + n] = g.base[p * g.ldb + n] - round8(v);
        } else {  // EPI_PRIOR -> NCHW mean / logscale / scale
          const int64_t b = p / hw, rem = p - b * hw;
          if (n < g.n_mean) {
            g.mean[(b * g.n_mean + n) * hw + rem] = v;
          } else {
            const int64_t o = (b * g.n_mean + (n - g.n_mean)) * hw + rem;
            g.logscale[o] = v;
            g.scale[o] = expf_glibc(v);
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ dispatch
template <int BM, int BN, int WM, int WN, int MODE, int EPI>
static int launch_one(GemmArgs a, hipStream_t s) {
  a.m_tiles = (int)((a.P + BM - 1) / BM);
  a.n_tiles = (a.N + BN - 1) / BN;
  dim3 grid((unsigned)(a.m_tiles * a.n_tiles));
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, MODE, EPI>), grid, dim3(256), 0, s, a);
  return idf_last_error();
}

// Row-tile height: the largest BM whose grid still has >= 4 blocks per CU (1024),
// else the smallest.  BM only changes how rows are grouped into blocks; every
// output's k-order (and so its bits) is identical for any BM.
template <int BN, int MODE, int EPI>
static int launch_bn(const GemmArgs& a, hipStream_t s) {
  const int64_t nt = (a.N + BN - 1) / BN;
  auto blocks = [&](int bm) { return ((a.P + bm - 1) / bm) * nt; };
  if (BN == 128) {
    if (blocks(128) >= 1024) return launch_one<128, 128, 2, 2, MODE, EPI>(a, s);
    return launch_one<64, 128, 1, 4, MODE, EPI>(a, s);
  }
  if (blocks(256) >= 1024) return launch_one<256, BN, 4, 1, MODE, EPI>(a, s);
  if (blocks(128) >= 1024) return launch_one<128, BN, 4, 1, MODE, EPI>(a, s);
  return launch_one<64, BN, 4, 1, MODE, EPI>(a, s);
}

template <int MODE, int EPI>
static int launch_epi(const GemmArgs& a, int bn, hipStream_t s) {
  switch (bn) {
    case 16: return launch_bn<16, MODE, EPI>(a, s);
    case 32: return launch_bn<32, MODE, EPI>(a, s);
    case 48: return launch_bn<48, MODE, EPI>(a, s);
    case 64: return launch_bn<64, MODE, EPI>(a, s);
    default: return launch_bn<128, MODE, EPI>(a, s);
  }
}

// Tile width for N output columns (shared with idfcodec/packing.py: tile_n()).
static int tile_n(int N) {
  if (N <= 16) return 16;
  if (N <= 32) return 32;
  if (N <= 48) return 48;
  if (N <= 64) return 64;
  int w64 = ((N + 63) / 64) * 64 - N, w128 = ((N + 127) / 128) * 128 - N;
  return (w128 <= w64 + 32) ? 128 : 64;
}

static int launch_gemm(const GemmArgs& a, int mode, int epi, int n_alloc, hipStream_t s) {
  if (a.P <= 0 || a.N <= 0) return IDF_OK;
  if (a.K <= 0 || (a.K & 3) || (a.lda & 3) || (a.ldw & 15) || a.ldw < ((a.K + 15) / 16) * 16)
    return IDF_ERR_ARG;
  int bn = tile_n(a.N);
  if (n_alloc < ((a.N + bn - 1) / bn) * bn) return IDF_ERR_ARG;
  if (mode == MODE_DENSE) {
    switch (epi) {
      case EPI_STORE: return launch_epi<MODE_DENSE, EPI_STORE>(a, bn, s);
      case EPI_COUPLE_ADD: return launch_epi<MODE_DENSE, EPI_COUPLE_ADD>(a, bn, s);
      case EPI_COUPLE_SUB: return launch_epi<MODE_DENSE, EPI_COUPLE_SUB>(a, bn, s);
      case EPI_PRIOR: return launch_epi<MODE_DENSE, EPI_PRIOR>(a, bn, s);
      default: return IDF_ERR_ARG;
    }
  }
  switch (epi) {
    case EPI_ACT: return launch_epi<MODE_CONV3, EPI_ACT>(a, bn, s);
    case EPI_ACT_FOLD: return launch_epi<MODE_CONV3, EPI_ACT_FOLD>(a, bn, s);
    default: return IDF_ERR_ARG;
  }
}

static void fill_head(GemmArgs& a, const IdfHeadOut* h, int* epi) {
  if (!h) {
    *epi = EPI_STORE;
    return;
  }
  switch (h->mode) {
    case IDF_EPI_COUPLE_ADD: *epi = EPI_COUPLE_ADD; break;
    case IDF_EPI_COUPLE_SUB: *epi = EPI_COUPLE_SUB; break;
    case IDF_EPI_PRIOR: *epi = EPI_PRIOR; break;
    default: *epi = EPI_STORE; break;
  }
  a.out = h->out ? h->out : a.out;
  a.ldo = h->out ? h->ld_out : a.ldo;
  a.base = h->base;
  a.ldb = h->ld_base;
  a.n_mean = h->n_mean;
  a.mean = h->mean;
  a.logscale = h->logscale;
  a.scale = h->scale;
}

// ------------------------------------------------------------------ index maps
__global__ void dequant_u8_kernel(int B, int C, int H, int W, const uint8_t* __restrict__ img,
                                  float* __restrict__ out, int64_t ld) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)B * C * H * W;
  if (i >= total) return;
  // i indexes NCHW (coalesced read); scatter to pixel-major
  int64_t hw = (int64_t)H * W;
  int64_t b = i / (C * hw), rem = i % (C * hw);
  int c = (int)(rem / hw);
  int64_t pix = rem % hw;
  int k = img[i];
  out[(b * hw + pix) * ld + c] = (float)(k + (k >= 128 ? 1 : 0)) * (1.0f / 256.0f);
}

// ------------------------------------------------------------------ log-likelihood
// DLogistic.log_prob (distlib.py:40-55) per symbol, with IDFlows.log_likelihood's per-image
// reduction (flows.py:154-169) fused: one block per (level, image) group reduces its
// group_len log-probabilities in a fixed order (per-thread strided f64 partials, then a fixed
// tree), so the sums are deterministic.  The per-symbol arithmetic follows torch's fp32 ops
// in the reference's order: scale = exp(logscale); x+- = ((x +- 0.5/bins) - mean) / scale;
// logsigmoid(v) = min(v, 0) - log1p(exp(-|v|)); logP = lp + log((1 - exp(ln - lp)) + eps).
__device__ __forceinline__ float idf_logsigmoid(float v) {
  return fminf(v, 0.0f) - log1pf(expf(-fabsf(v)));
}

__global__ void __launch_bounds__(256) log_prob_kernel(int64_t group_len,
                                                       const float* __restrict__ x,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ logscale,
                                                       float half_bin, float eps,
                                                       float* __restrict__ logp,
                                                       double* __restrict__ gsum) {
  const int64_t g0 = (int64_t)blockIdx.x * group_len;
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < group_len; i += 256) {
    const int64_t k = g0 + i;
    const float sc = expf(logscale[k]);
    const float xm = x[k], mu = mean[k];
    const float xp = ((xm + half_bin) - mu) / sc;
    const float xn = ((xm - half_bin) - mu) / sc;
    const float lp = idf_logsigmoid(xp), ln = idf_logsigmoid(xn);
    const float v = lp + logf((1.0f - expf(ln - lp)) + eps);
    if (logp) logp[k] = v;
    acc += (double)v;
  }
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0 && gsum) gsum[blockIdx.x] = red[0];
}

// Per-element logP only (no group sums): one element per thread over a grid-stride loop,
// the same arithmetic as log_prob_kernel so both paths agree bit for bit.
__global__ void __launch_bounds__(256) log_prob_elem_kernel(int64_t n, const float* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ logscale,
                                                            float half_bin, float eps,
                                                            float* __restrict__ logp) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const float sc = expf(logscale[k]);
    const float xm = x[k], mu = mean[k];
    const float xp = ((xm + half_bin) - mu) / sc;
    const float xn = ((xm - half_bin) - mu) / sc;
    const float lp = idf_logsigmoid(xp), ln = idf_logsigmoid(xn);
    logp[k] = lp + logf((1.0f - expf(ln - lp)) + eps);
  }
}

__global__ void quant_u8_kernel(int B, int C, int H, int W, const float* __restrict__ in, int64_t ld,
                                uint8_t* __restrict__ img, int32_t* __restrict__ bad) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)B * C * H * W;
  if (i >= total) return;
  int64_t hw = (int64_t)H * W;
  int64_t b = i / (C * hw), rem = i % (C * hw);
  int c = (int)(rem / hw);
  int64_t pix = rem % hw;
  float v = in[(b * hw + pix) * ld + c] * 256.0f;
  float m = __builtin_rintf(v);
  int mi = (int)m;
  int k = mi >= 129 ? mi - 1 : mi;
  bool ok = (m == v) && mi >= 0 && mi <= 256 && mi != 128;
  if (!ok) {
    atomicAdd(bad, 1);
    k = k < 0 ? 0 : (k > 255 ? 255 : k);
  }
  img[i] = (uint8_t)k;
}

__global__ void squeeze_kernel(int B, int H, int W, int C, int s, const float* __restrict__ src,
                               int64_t lds, float* __restrict__ dst, int64_t ldd, int inverse) {
  // one thread per element of the squeezed tensor [B, H/s, W/s, C*s*s]
  int Ho = H / s, Wo = W / s, Co = C * s * s;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)B * Ho * Wo * Co;
  if (i >= total) return;
  int oc = (int)(i % Co);
  int64_t op = i / Co;
  int ox = (int)(op % Wo);
  int64_t t = op / Wo;
  int oy = (int)(t % Ho);
  int64_t b = t / Ho;
  int c = oc / (s * s), ii = (oc / s) % s, jj = oc % s;
  int64_t ip = (b * H + (int64_t)oy * s + ii) * W + (int64_t)ox * s + jj;
  if (!inverse)
    dst[op * ldd + oc] = src[ip * lds + c];
  else
    dst[ip * ldd + c] = src[op * lds + oc];
}

__global__ void permute_couple_in_kernel(int64_t P, int C, const int32_t* __restrict__ ids,
                                         const float* __restrict__ src, int64_t lds,
                                         float* __restrict__ dst, int64_t ldd, int a, int a_pad,
                                         float* __restrict__ feat, int64_t ldf) {
  int W = C > a_pad ? C : a_pad;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * W) return;
  int64_t p = i / W;
  int c = (int)(i % W);
  float v = 0.0f;
  if (c < C) {
    v = src[p * lds + ids[c]];
    dst[p * ldd + c] = v;
  }
  if (feat && c < a_pad) feat[p * ldf + c] = c < a ? v : 0.0f;
}

__global__ void copy_cols_kernel(int64_t P, int n, int n_pad, const float* __restrict__ src,
                                 int64_t lds, float* __restrict__ dst, int64_t ldd) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * n_pad) return;
  int64_t p = i / n_pad;
  int c = (int)(i % n_pad);
  dst[p * ldd + c] = c < n ? src[p * lds + c] : 0.0f;
}

__global__ void pm_nchw_kernel(int B, int C, int H, int W, const float* __restrict__ src,
                               int64_t ld, float* __restrict__ dst, int to_nchw) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t hw = (int64_t)H * W;
  int64_t total = (int64_t)B * C * hw;
  if (i >= total) return;
  int64_t b = i / (C * hw), rem = i % (C * hw);
  int c = (int)(rem / hw);
  int64_t pix = rem % hw;
  if (to_nchw)
    dst[i] = src[(b * hw + pix) * ld + c];
  else
    dst[(b * hw + pix) * ld + c] = src[i];  // here src is NCHW, dst pixel-major
}

static inline dim3 grid1d(int64_t n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

}  // namespace idf

// ============================================================== C-ABI
using namespace idf;

extern "C" {

int idf_conv1x1_f32(void* stream, int64_t P, int32_t K, int32_t N, const float* a, int64_t lda,
                    const float* w, int32_t ldw, int32_t n_alloc, const float* bias, float* out,
                    int64_t ld_out, int32_t B, int32_t H, int32_t W, const IdfHeadOut* head) {
  GemmArgs g = {};
  g.P = P; g.K = K; g.N = N; g.A = a; g.lda = lda; g.W = w; g.ldw = ldw; g.bias = bias;
  g.out = out; g.ldo = ld_out; g.B = B; g.H = H; g.Wd = W; g.act = IDF_ACT_NONE;
  int epi = EPI_STORE;
  fill_head(g, head, &epi);
  return launch_gemm(g, MODE_DENSE, epi, n_alloc, (hipStream_t)stream);
}

int idf_conv3x3_f32(void* stream, int32_t B, int32_t H, int32_t W, int32_t C, const float* t,
                    int64_t ld_t, const float* w, int32_t ldw, int32_t n_alloc, const float* bias,
                    int32_t N, float* out, int64_t ld_out, int32_t act, float slope) {
  GemmArgs g = {};
  g.P = (int64_t)B * H * W; g.K = C; g.N = N; g.A = t; g.lda = ld_t; g.W = w; g.ldw = ldw;
  g.bias = bias; g.out = out; g.ldo = ld_out; g.B = B; g.H = H; g.Wd = W; g.act = act;
  g.slope = slope;
  return launch_gemm(g, MODE_CONV3, EPI_ACT, n_alloc, (hipStream_t)stream);
}

int idf_conv3x3_fold_f32(void* stream, int32_t B, int32_t H, int32_t W, int32_t C, const float* x,
                         int64_t ld_x, const float* w, int32_t ldw, int32_t n_alloc,
                         const float* b3, const float* vtap, int32_t ldv, const float* bfull,
                         int32_t N, float* out, int64_t ld_out, int32_t act, float slope) {
  if (!vtap || !bfull || ldv < N) return IDF_ERR_ARG;
  GemmArgs g = {};
  g.P = (int64_t)B * H * W; g.K = C; g.N = N; g.A = x; g.lda = ld_x; g.W = w; g.ldw = ldw;
  g.bias = b3; g.out = out; g.ldo = ld_out; g.B = B; g.H = H; g.Wd = W; g.act = act;
  g.slope = slope; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv;
  return launch_gemm(g, MODE_CONV3, EPI_ACT_FOLD, n_alloc, (hipStream_t)stream);
}

}  // extern "C"

// ------------------------------------------------------------------ timer
struct IdfTimer {
  struct Rec {
    hipEvent_t a, b;
    int tag;
    double flops;
  };
  std::vector<Rec> recs;
  size_t used = 0;
};

static void timer_mark(IdfTimer* t, hipStream_t s, int tag, double flops, bool begin) {
  if (!t) return;
  if (begin) {
    if (t->used >= t->recs.size()) return;  // capacity reached: stop sampling
    IdfTimer::Rec& r = t->recs[t->used];
    r.tag = tag;
    r.flops = flops;
    (void)hipEventRecord(r.a, s);
  } else {
    if (t->used >= t->recs.size()) return;
    (void)hipEventRecord(t->recs[t->used].b, s);
    t->used++;
  }
}

// The dx3 / dxb layers' part of a DenseBlock's tmp (dense_block_run): the block's split (dx3) or
// bf16 (dxb) feature copy at the front, its layers' split-K workspace after it (256-B aligned),
// and -- when the head is fused (IdfDenseBlock.fuse_head, by the geometry alone: every layer on
// the direct conv, one output group, n_head <= 16, a block input of <= 64 channels) -- the head's
// running sums [P][16] f32 after that.  Whether the head is fused depends on the block and the
// geometry only, never on the room in tmp: a caller's tmp too small for the sums is an error
// (IDF_ERR_WORKSPACE), not a silent switch to the head GEMM, whose sums run in another order.
struct Dx3TmpPlan {
  bool dx3, dxb, fuse;
  int n_dx3, nslab_xs;
  int64_t xs_bytes, off, need, hoff, bytes;  // bytes: the whole part (0 without dx3 / dxb)
};

static int dx3_tmp_plan(const IdfDenseBlock* blk, int32_t B, int32_t H, int32_t W, bool head,
                        Dx3TmpPlan* pl) {
  *pl = {};
  const int64_t P = (int64_t)B * H * W;
  pl->dxb = blk->bf16 && blk->fold && blk->dxb && blk->depth > 0 &&
            idf_conv3x3_dxb_supported(H, W, blk->g_pad);
  // the layers with dx3 weights are a prefix (the narrow ones, packing.py pack_dense_block
  // dx3_cmax); the rest run on wx3, whose workspace then reuses the copy
  bool dx3 = blk->fold && blk->wx3 && blk->dx3 && !blk->bf16 &&
             idf_conv3x3_dx3_supported(H, W, blk->g_pad);
  int n_dx3 = 0;
  while (dx3 && n_dx3 < blk->depth && blk->dx3_w[n_dx3]) ++n_dx3;
  for (int i = n_dx3; dx3 && i < blk->depth; ++i)
    if (blk->dx3_w[i]) return IDF_ERR_ARG;  // not a prefix
  pl->dx3 = dx3 && n_dx3 > 0;
  if (pl->dxb) n_dx3 = blk->depth;  // below: "dx3" setup for either direct conv
  pl->n_dx3 = n_dx3;
  if (!pl->dx3 && !pl->dxb) return IDF_OK;
  const int nft = (blk->g_pad + 15) / 16, nf = nft < 4 ? nft : 4;
  const int dx3_nft = (nft + nf - 1) / nf * nf;  // fragments the dx3 weights hold
  // the slabs the dx3 layers read: up to the last one's input (its own outputs are read by
  // no dx3 layer, so they are split only into the slab it reads)
  pl->nslab_xs = (blk->k_in[n_dx3 - 1] + 15) / 16;
  pl->xs_bytes = pl->dxb ? idf_dxb_bytes(P, 16 * pl->nslab_xs) : idf_dx3_split_bytes(P, 16 * pl->nslab_xs);
  pl->off = (pl->xs_bytes + 255) / 256 * 256;
  pl->need = idf_conv3x3_dx3_workspace(B, H, W, blk->k_in[n_dx3 - 1], blk->g_pad);
  if (pl->need < 0) return IDF_ERR_UNSUPPORTED;
  pl->bytes = pl->off + pl->need;
  pl->fuse = head && blk->fuse_head && n_dx3 == blk->depth && blk->n_head <= 16 && dx3_nft <= 4 &&
             blk->k_in[0] <= 64 && blk->depth > 0;
  if (pl->fuse) {
    pl->hoff = (pl->off + pl->need + 255) / 256 * 256;
    pl->bytes = pl->hoff + P * 64;
  }
  return IDF_OK;
}

extern "C" int64_t idf_dense_block_dx3_tmp_bytes(const IdfDenseBlock* blk, int32_t B, int32_t H,
                                                  int32_t W) {
  if (!blk || blk->depth < 0 || blk->depth > IDF_MAX_DEPTH || B < 0 || H < 1 || W < 1) return -1;
  Dx3TmpPlan pl;
  if (dx3_tmp_plan(blk, B, H, W, true, &pl)) return -1;
  return pl.bytes;
}

static int dense_block_run(void* stream, const IdfDenseBlock* blk, int32_t B, int32_t H, int32_t W,
                           float* feat, int64_t ld_feat, float* tmp, int64_t ld_tmp,
                           const IdfHeadOut* head, IdfTimer* timer) {
  if (!blk || blk->depth < 0 || blk->depth > IDF_MAX_DEPTH) return IDF_ERR_ARG;
  const int64_t P = (int64_t)B * H * W;
  if (ld_feat < blk->k_in[blk->depth] || ld_tmp < blk->k_in[blk->depth]) return IDF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  // bf16 blocks keep a bf16 shadow of the feature columns at the front of tmp (each layer
  // writes its output in both precisions; conv3_bf16.hip DMAs its halos from the shadow),
  // followed by the split-K partials
  uint16_t* f16 = nullptr;
  int64_t ld16 = 0;
  float* ws = tmp;
  int64_t ws_floats = P * ld_tmp;
  // bf16 blocks on the bf16 direct conv (IdfDenseBlock.dxb, conv3_dx3.hip) -- every layer, by
  // the level geometry alone -- keep a slab-major bf16 copy of their features instead, set up
  // with the dx3 split copy below
  Dx3TmpPlan pl;
  if (int rc = dx3_tmp_plan(blk, B, H, W, head != nullptr, &pl)) return rc;
  const bool dxb = pl.dxb;
  if (blk->bf16) {
    if (!blk->fold) return IDF_ERR_ARG;
    for (int i = 0; i < blk->depth; ++i) {
      if (!blk->wb16[i]) return IDF_ERR_ARG;
      if (dxb && !blk->dxb_w[i]) return IDF_ERR_ARG;
    }
  }
  if (blk->bf16 && !dxb) {
    // pitch a multiple of 64 channels: a pixel's 32-channel slab is one aligned 64-B run
    ld16 = ((int64_t)blk->k_in[blk->depth] + 63) / 64 * 64;
    const int64_t sh = (P * ld16 / 2 + 3) / 4 * 4;  // floats
    if (sh > ws_floats) return IDF_ERR_WORKSPACE;
    f16 = (uint16_t*)tmp;
    ws = tmp + sh;
    ws_floats -= sh;
    const int c0 = blk->k_in[0];
    int rc = idf_f32_to_bf16_cols(stream, P, c0, (c0 + 7) / 8 * 8, feat, ld_feat, f16, ld16);
    if (rc) return rc;
  }
  // dx3 blocks keep the split copy of their feature columns (conv3_dx3.hip) at the front of
  // tmp: the block input is split once here, every dx3 layer writes its outputs in both
  // forms (dx3_tmp_plan: the layout)
  const bool dx3 = pl.dx3;
  const int n_dx3 = pl.n_dx3;
  uint16_t* xs = nullptr;
  int32_t nslab_xs = 0;
  char* dws = nullptr;  // the dx3 layers' split-K counters and partial sums, after the copy
  int64_t dws_bytes = 0;
  float* hacc = nullptr;  // the fused head's running sums (nullptr: the head GEMM runs)
  const int dx3_nft = [&] {  // fragments the dx3 weights hold (packing.dx3_groups)
    const int nft = (blk->g_pad + 15) / 16, nf = nft < 4 ? nft : 4;
    return (nft + nf - 1) / nf * nf;
  }();
  // the fused DenseBlock (IdfDenseBlock.fuse_layers): every layer in one launch, one workgroup
  // per tile, where the tiles hold whole images (conv3_dx3.hip conv3_dx3_block_kernel) -- the
  // per-layer launches' bits, with the fused head's sums in registers (no head init launch)
  const bool fused = blk->fuse_layers && (dx3 || dxb) && n_dx3 == blk->depth && blk->depth >= 1 &&
                     blk->depth <= 16 && idf_dx3_block_supported(H, W, blk->g_pad, dxb ? 1 : 0);
  if (dx3 || dxb) {
    const int64_t avail = ws_floats * 4;
    if (pl.bytes > avail || (uintptr_t)tmp % 256) return IDF_ERR_WORKSPACE;
    nslab_xs = pl.nslab_xs;
    const int64_t need = pl.need;
    xs = (uint16_t*)tmp;
    dws = (char*)tmp + pl.off;
    dws_bytes = need;
    if (pl.fuse) hacc = (float*)((char*)tmp + pl.hoff);
    const int64_t ctr = idf_conv3x3_dx3_counter_bytes(B, H, W, blk->g_pad);
    // the head init rides in the split's launch where it can (same bits, one launch fewer)
    const bool head_in_split = !dxb && hacc && !fused && blk->k_in[0] > 0 && blk->k_in[0] <= 64;
    int rc = dxb ? idf_dxb_cols(stream, P, 0, blk->k_in[0], feat, ld_feat, xs, nslab_xs,
                                need > 0 ? (uint32_t*)dws : nullptr,
                                need > 0 ? (int32_t)(ctr / 4) : 0)
           : head_in_split
               ? idf_dx3_split_cols_head(stream, P, blk->k_in[0], feat, ld_feat, xs, nslab_xs,
                                         blk->range_flag, need > 0 ? (uint32_t*)dws : nullptr,
                                         need > 0 ? (int32_t)(ctr / 4) : 0, blk->wh, blk->ldwh,
                                         blk->bh, blk->n_head, hacc)
               : idf_dx3_split_cols(stream, P, 0, blk->k_in[0], feat, ld_feat, xs, nslab_xs,
                                    blk->range_flag, need > 0 ? (uint32_t*)dws : nullptr,
                                    need > 0 ? (int32_t)(ctr / 4) : 0);
    if (rc) return rc;
    if (hacc && !fused && !head_in_split) {
      rc = idf_dx3_head_init(stream, P, blk->k_in[0], feat, ld_feat, blk->wh, blk->ldwh, blk->bh,
                             blk->n_head, hacc);
      if (rc) return rc;
    }
  }
  if (fused) {
    int32_t C[16];
    const uint16_t* w[16];
    float ys[16];
    const float *b3[16], *vt[16], *bfu[16];
    double fl = 0.0;
    for (int i = 0; i < blk->depth; ++i) {
      C[i] = blk->k_in[i];
      w[i] = dxb ? blk->dxb_w[i] : blk->dx3_w[i];
      ys[i] = dxb ? 1.0f : blk->dx3_yscale[i];
      b3[i] = blk->b3[i];
      vt[i] = blk->vtap[i];
      bfu[i] = blk->bfull[i];
      fl += 2.0 * P * 9.0 * blk->c_real[i] * blk->g_real[i];
    }
    IdfDx3Head hd = {};
    if (hacc) {
      hd.w = blk->wh; hd.ldw = blk->ldwh; hd.n_head = blk->n_head; hd.acc = nullptr;
      hd.last = 1;
      hd.skip_f32 = blk->keep_feat ? 0 : 1;
      hd.out = *head;
    }
    IdfDx3BlockDesc d = {};
    d.bf = dxb ? 1 : 0;
    d.B = B; d.H = H; d.W = W; d.nlayers = blk->depth; d.N = blk->g_pad; d.nft = dx3_nft;
    d.ldv = blk->ldv; d.act = blk->act; d.nslab_xs = nslab_xs; d.slope = blk->slope;
    d.xs = xs; d.C = C; d.w = w; d.yscale = ys; d.b3 = b3;
    d.vtap = blk->vtap[0] ? vt : nullptr; d.bfull = blk->vtap[0] ? bfu : nullptr;
    d.feat = feat; d.ld_feat = ld_feat; d.flag = dxb ? nullptr : blk->range_flag;
    d.head = hacc ? &hd : nullptr;
    d.hx = feat; d.hld_x = ld_feat; d.hc0 = blk->k_in[0]; d.hb = blk->bh;
    timer_mark(timer, s, IDF_TAG_CONV3X3, fl, true);
    const int rc = idf_dx3_block_launch(stream, &d);
    timer_mark(timer, s, 0, 0, false);
    if (rc) return rc;
  }
  for (int i = 0; i < (fused ? 0 : blk->depth); ++i) {
    const int c = blk->k_in[i];
    IdfDx3Head hd = {};
    if (hacc) {
      hd.w = blk->wh; hd.ldw = blk->ldwh; hd.n_head = blk->n_head; hd.acc = hacc;
      hd.last = i == blk->depth - 1;
      hd.skip_f32 = blk->keep_feat ? 0 : 1;
      hd.out = *head;
    }
    const double cr = blk->c_real[i], gr = blk->g_real[i];
    if (blk->fold) {  // one launch per layer: 3x3 over the layer input, 1x1 folded in
      timer_mark(timer, s, IDF_TAG_CONV3X3, 2.0 * P * 9.0 * cr * gr, true);
      const bool wino = blk->wino && blk->wino_u[i] && idf_conv3x3_wino_supported(H, W);
      const bool bf = blk->bf16 != 0;
      const int n16 = (c + blk->g_pad + 7) / 8 * 8 - c;
      int rc = dxb
                   ? idf_conv3x3_dxb(stream, B, H, W, c, xs, nslab_xs, blk->dxb_w[i], dx3_nft,
                                     blk->b3[i], blk->vtap[i], blk->ldv, blk->bfull[i], blk->g_pad,
                                     feat + c, ld_feat, blk->act, blk->slope, dws, dws_bytes,
                                     hacc ? &hd : nullptr)
               : bf
                   ? idf_conv3x3_bf16(stream, B, H, W, c, f16, ld16, blk->wb16[i], blk->g_alloc,
                                      blk->b3[i], blk->vtap[i], blk->ldv, blk->bfull[i],
                                      blk->g_pad, feat + c, ld_feat, f16 + c, ld16, n16,
                                      blk->act, blk->slope, ws, ws_floats)
               : (dx3 && i < n_dx3)
                   ? idf_conv3x3_dx3(stream, B, H, W, c, xs, nslab_xs, blk->dx3_w[i], dx3_nft,
                                     blk->dx3_yscale[i], blk->b3[i], blk->vtap[i], blk->ldv,
                                     blk->bfull[i], blk->g_pad, feat + c, ld_feat, blk->act,
                                     blk->slope, blk->range_flag, dws, dws_bytes,
                                     hacc ? &hd : nullptr)
               : (wino && blk->wx3 && blk->wx3_u[i])
                   ? idf_conv3x3_wx3(stream, B, H, W, c, feat, ld_feat, blk->wx3_u[i],
                                     blk->wino_nft, blk->wx3_yscale[i], blk->b3[i], blk->vtap[i],
                                     blk->ldv, blk->bfull[i], blk->g_pad, feat + c, ld_feat,
                                     blk->act, blk->slope, blk->range_flag,
                                     (i == 0 || (dx3 && i == n_dx3)) ? 1 : 0, tmp,
                                     P * ld_tmp)
               : wino
                   ? idf_conv3x3_wino(stream, B, H, W, c, feat, ld_feat, blk->wino_u[i],
                                      blk->wino_nft, blk->b3[i], blk->vtap[i], blk->ldv,
                                      blk->bfull[i], blk->g_pad, feat + c, ld_feat, blk->act,
                                      blk->slope, tmp, P * ld_tmp)
               : blk->halo
                   ? idf_conv3x3_halo(stream, B, H, W, c, feat, ld_feat, blk->w3[i], blk->ldw3[i],
                                      blk->g_alloc, blk->b3[i], blk->vtap[i], blk->ldv,
                                      blk->bfull[i], blk->g_pad, feat + c, ld_feat, blk->act,
                                      blk->slope, tmp, P * ld_tmp)
                   : idf_conv3x3_fold_f32(stream, B, H, W, c, feat, ld_feat, blk->w3[i],
                                          blk->ldw3[i], blk->g_alloc, blk->b3[i], blk->vtap[i],
                                          blk->ldv, blk->bfull[i], blk->g_pad, feat + c, ld_feat,
                                          blk->act, blk->slope);
      timer_mark(timer, s, 0, 0, false);
      if (rc) return rc;
      continue;
    }
    timer_mark(timer, s, IDF_TAG_CONV1X1, 2.0 * P * cr * cr, true);
    int rc = idf_conv1x1_f32(stream, P, c, c, feat, ld_feat, blk->w1[i], blk->ldw1[i],
                             blk->n1_alloc[i], blk->b1[i], tmp, ld_tmp, B, H, W, nullptr);
    timer_mark(timer, s, 0, 0, false);
    if (rc) return rc;
    timer_mark(timer, s, IDF_TAG_CONV3X3, 2.0 * P * 9.0 * cr * gr, true);
    rc = idf_conv3x3_f32(stream, B, H, W, c, tmp, ld_tmp, blk->w3[i], blk->ldw3[i], blk->g_alloc,
                         blk->b3[i], blk->g_pad, feat + c, ld_feat, blk->act, blk->slope);
    timer_mark(timer, s, 0, 0, false);
    if (rc) return rc;
  }
  if (!head || hacc) return IDF_OK;  // caller runs the head itself / fused into the last layer
  timer_mark(timer, s, IDF_TAG_HEAD, 2.0 * P * blk->c_real[blk->depth] * blk->n_head, true);
  int rc = idf_conv1x1_f32(stream, P, blk->k_in[blk->depth], blk->n_head, feat, ld_feat, blk->wh,
                           blk->ldwh, blk->nh_alloc, blk->bh, nullptr, 0, B, H, W, head);
  timer_mark(timer, s, 0, 0, false);
  return rc;
}

extern "C" {

int idf_dense_block_f32(void* stream, const IdfDenseBlock* blk, int32_t B, int32_t H, int32_t W,
                        float* feat, int64_t ld_feat, float* tmp, int64_t ld_tmp,
                        const IdfHeadOut* head) {
  return dense_block_run(stream, blk, B, H, W, feat, ld_feat, tmp, ld_tmp, head, nullptr);
}

int idf_dense_block_f32_timed(void* stream, const IdfDenseBlock* blk, int32_t B, int32_t H,
                              int32_t W, float* feat, int64_t ld_feat, float* tmp, int64_t ld_tmp,
                              const IdfHeadOut* head, IdfTimer* timer) {
  return dense_block_run(stream, blk, B, H, W, feat, ld_feat, tmp, ld_tmp, head, timer);
}

IdfTimer* idf_timer_create(int32_t capacity) {
  IdfTimer* t = new IdfTimer();
  t->recs.resize(capacity > 0 ? capacity : 0);
  for (auto& r : t->recs) {
    if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) {
      delete t;
      return nullptr;
    }
  }
  return t;
}

void idf_timer_destroy(IdfTimer* t) {
  if (!t) return;
  for (auto& r : t->recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  delete t;
}

void idf_timer_reset(IdfTimer* t) {
  if (t) t->used = 0;
}

int idf_timer_summary(IdfTimer* t, int32_t tag, double* total_ms, int64_t* count, double* flops) {
  if (!t) return IDF_ERR_ARG;
  double ms = 0, fl = 0;
  int64_t n = 0;
  for (size_t i = 0; i < t->used; ++i) {
    const IdfTimer::Rec& r = t->recs[i];
    if (r.tag != tag) continue;
    float e = 0.f;
    if (hipEventElapsedTime(&e, r.a, r.b) != hipSuccess) return IDF_ERR_HIP;
    ms += e;
    fl += r.flops;
    ++n;
  }
  if (total_ms) *total_ms = ms;
  if (count) *count = n;
  if (flops) *flops = fl;
  return IDF_OK;
}

int idf_dequant_u8(void* stream, int32_t B, int32_t C, int32_t H, int32_t W, const uint8_t* img,
                   float* out, int64_t ld_out) {
  int64_t n = (int64_t)B * C * H * W;
  if (n <= 0) return n < 0 ? IDF_ERR_ARG : IDF_OK;
  hipLaunchKernelGGL(dequant_u8_kernel, grid1d(n), dim3(256), 0, (hipStream_t)stream, B, C, H, W,
                     img, out, ld_out);
  return idf_last_error();
}

int idf_log_prob(void* stream, int64_t n_groups, int64_t group_len, const float* x,
                 const float* mean, const float* logscale, int32_t nbits, float eps,
                 float* logp, double* group_sum) {
  if (n_groups < 0 || group_len < 0 || nbits < 0 || nbits > 30) return IDF_ERR_ARG;
  if (n_groups == 0) return IDF_OK;
  if (n_groups > 0x7fffffff || !x || !mean || !logscale) return IDF_ERR_ARG;
  const float half_bin = 0.5f / (float)(1 << nbits);
  if (!group_sum) {
    if (!logp) return IDF_OK;
    const int64_t n = n_groups * group_len;
    if (n == 0) return IDF_OK;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(log_prob_elem_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, n, x, mean, logscale, half_bin, eps, logp);
    return idf_last_error();
  }
  hipLaunchKernelGGL(log_prob_kernel, dim3((unsigned)n_groups), dim3(256), 0,
                     (hipStream_t)stream, group_len, x, mean, logscale, half_bin, eps, logp,
                     group_sum);
  return idf_last_error();
}

int idf_quant_u8(void* stream, int32_t B, int32_t C, int32_t H, int32_t W, const float* in,
                 int64_t ld_in, uint8_t* img, int32_t* bad) {
  int64_t n = (int64_t)B * C * H * W;
  if (n <= 0) return n < 0 ? IDF_ERR_ARG : IDF_OK;
  hipLaunchKernelGGL(quant_u8_kernel, grid1d(n), dim3(256), 0, (hipStream_t)stream, B, C, H, W,
                     in, ld_in, img, bad);
  return idf_last_error();
}

int idf_squeeze(void* stream, int32_t B, int32_t H, int32_t W, int32_t C, int32_t s,
                const float* src, int64_t ld_src, float* dst, int64_t ld_dst) {
  if (s <= 0 || H % s || W % s) return IDF_ERR_ARG;
  int64_t n = (int64_t)B * H * W * C;
  if (n <= 0) return IDF_OK;
  hipLaunchKernelGGL(squeeze_kernel, grid1d(n), dim3(256), 0, (hipStream_t)stream, B, H, W, C, s,
                     src, ld_src, dst, ld_dst, 0);
  return idf_last_error();
}

int idf_unsqueeze(void* stream, int32_t B, int32_t H, int32_t W, int32_t C, int32_t s,
                  const float* src, int64_t ld_src, float* dst, int64_t ld_dst) {
  // (H, W, C) describe the UNSQUEEZED (output) tensor, as in idf_squeeze
  if (s <= 0 || H % s || W % s) return IDF_ERR_ARG;
  int64_t n = (int64_t)B * H * W * C;
  if (n <= 0) return IDF_OK;
  hipLaunchKernelGGL(squeeze_kernel, grid1d(n), dim3(256), 0, (hipStream_t)stream, B, H, W, C, s,
                     src, ld_src, dst, ld_dst, 1);
  return idf_last_error();
}

int idf_permute_couple_in(void* stream, int64_t P, int32_t C, const int32_t* ids, const float* src,
                          int64_t ld_src, float* dst, int64_t ld_dst, int32_t a, int32_t a_pad,
                          float* feat, int64_t ld_feat) {
  int Wd = C > a_pad ? C : a_pad;
  int64_t n = P * Wd;
  if (n <= 0) return IDF_OK;
  hipLaunchKernelGGL(permute_couple_in_kernel, grid1d(n), dim3(256), 0, (hipStream_t)stream, P, C,
                     ids, src, ld_src, dst, ld_dst, a, a_pad, feat, ld_feat);
  return idf_last_error();
}

int idf_copy_cols(void* stream, int64_t P, int32_t n, int32_t n_pad, const float* src,
                  int64_t ld_src, float* dst, int64_t ld_dst) {
  int64_t tot = P * n_pad;
  if (tot <= 0) return IDF_OK;
  hipLaunchKernelGGL(copy_cols_kernel, grid1d(tot), dim3(256), 0, (hipStream_t)stream, P, n, n_pad,
                     src, ld_src, dst, ld_dst);
  return idf_last_error();
}

int idf_pm_to_nchw(void* stream, int32_t B, int32_t C, int32_t H, int32_t W, const float* src,
                   int64_t ld_src, float* dst) {
  int64_t n = (int64_t)B * C * H * W;
  if (n <= 0) return IDF_OK;
  hipLaunchKernelGGL(pm_nchw_kernel, grid1d(n), dim3(256), 0, (hipStream_t)stream, B, C, H, W, src,
                     ld_src, dst, 1);
  return idf_last_error();
}

int idf_nchw_to_pm(void* stream, int32_t B, int32_t C, int32_t H, int32_t W, const float* src,
                   float* dst, int64_t ld_dst) {
  int64_t n = (int64_t)B * C * H * W;
  if (n <= 0) return IDF_OK;
  hipLaunchKernelGGL(pm_nchw_kernel, grid1d(n), dim3(256), 0, (hipStream_t)stream, B, C, H, W, src,
                     ld_dst, dst, 0);
  return idf_last_error();
}

const char* idf_version(void) { return "idfcodec 0.1.0 (gfx950)"; }

int idf_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
