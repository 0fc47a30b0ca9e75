// conv3_halo.hip -- the DenseLayer 3x3 convolution on gfx950 (the hot kernel).
//
// out[p, n] = act(bias(p, n) + sum_{tap, c} X[nbr(p, tap), c] * W[n, tap, c])
// with X pixel-major (the DenseBlock feature buffer, or the 1x1 output T when the
// 1x1 is not folded) and W packed [n][tap][c] (idfcodec/packing.py).
//
// Block = 8 waves, one spatial tile of up to 256 output pixels (IMGS images x TH
// rows x TW columns), all NF*16 output channels of one n-tile.  The K loop runs
// over 16-channel slabs.  For each slab the tile's (TH+2) x (TW+2) halo of X is
// staged in LDS ONCE and read by all 9 taps at shifted offsets (9x less load
// traffic than an implicit GEMM that re-gathers A per tap), together with the
// slab's 9 x BN weights.  Slabs are double buffered: the global loads of slab
// s+1 are in flight (in registers) while slab s computes; one barrier per slab.
// Per tap each lane reads one float4 of A per m-fragment and one of B per
// n-fragment (k = 4*(lane>>4) .. +3) and issues 4 f32 MFMAs (v_mfma_f32_16x16x4_f32)
// per fragment pair taking element t of the float4s -- a bijective k assignment.
//
// Split-K (ksplit > 1, chosen from the image geometry only, never the batch):
// block group s reduces slabs [s*nslab/S, (s+1)*nslab/S) and writes a partial
// tile; conv3_reduce_kernel adds the S partials in fixed order, then bias + act.
// Every output is thus a fixed-order sum that depends on the image geometry and
// channel count only: deterministic and batch-invariant.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "idf_codec_internal.h"

#pragma clang fp contract(off)

namespace idf {

typedef float f4 __attribute__((ext_vector_type(4)));

struct HaloArgs {
  const float* X;     // [P][ldx]
  int64_t ldx;
  int32_t C;          // input channels (multiple of 4)
  const float* W;     // [n_alloc][9][ldw]
  int32_t ldw;
  int32_t N;          // valid output channels
  int32_t B, H, Wd;   // images
  int32_t IMGS, TH, TW;
  int32_t tiles_b, tiles_y, tiles_x, n_tiles, ksplit;
  int32_t nslab;      // ceil(C / 16)
  // epilogue
  const float* b3;    // [n_alloc]
  const float* vtap;  // fold: [9][ldv]  (null = plain bias)
  const float* bfull; // fold: interior bias
  int32_t ldv;
  int32_t act;
  float slope;
  float* out;         // [P][ldo]  (ksplit == 1)
  int64_t ldo;
  float* part;        // [ksplit][P][ldp] (ksplit > 1)
  int32_t ldp;
};

constexpr int kThreads = 512;
constexpr int kApitch = 24;  // floats per halo pixel (16 data + 8 pad: conflict-free b128)
constexpr int kBpitch = 16;  // floats per (tap, n) weight row
constexpr int kLdsFloats = 163840 / 4;
// halo pixels per A stage that fit (double buffered) next to the NF-fragment B stage
constexpr int max_halo(int nf) { return (kLdsFloats / 2 - 9 * nf * 16 * kBpitch) / kApitch; }

__device__ __forceinline__ float act_fn(float v, int act, float slope) {
  if (act == IDF_ACT_RELU) return v > 0.0f ? v : 0.0f;
  if (act == IDF_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  if (act == IDF_ACT_TANH) return tanhf(v);
  return v;
}

__device__ __forceinline__ float tap_bias(const HaloArgs& g, int n, int y, int x) {
  float bsum;
  if (!g.vtap) return g.b3[n];
  if (y >= 1 && y <= g.H - 2 && x >= 1 && x <= g.Wd - 2) return g.bfull[n];
  bsum = g.b3[n];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int ny = y + tap / 3 - 1, nx = x + tap % 3 - 1;
    if (ny >= 0 && ny < g.H && nx >= 0 && nx < g.Wd) bsum = bsum + g.vtap[tap * g.ldv + n];
  }
  return bsum;
}

template <int NF>
__global__ void __launch_bounds__(kThreads) conv3_halo_kernel(HaloArgs g) {
  constexpr int BN = NF * 16;
  constexpr int FM = 2;                      // m-fragments per wave (8 waves x 32 px = 256)
  constexpr int B_F4 = 9 * BN * 4;           // float4 per B stage
  constexpr int B_PER_T = (B_F4 + kThreads - 1) / kThreads;
  constexpr int MAXH = max_halo(NF);
  constexpr int A_PER_T = (MAXH * 4 + kThreads - 1) / kThreads;
  constexpr int B_STAGE = 9 * BN * kBpitch;  // floats
  constexpr int A_STAGE = MAXH * kApitch;
  static_assert(2 * (A_STAGE + B_STAGE) <= kLdsFloats, "LDS budget");

  __shared__ __attribute__((aligned(16))) float lds[kLdsFloats];
  auto Abuf = [&](int buf) { return lds + buf * A_STAGE; };
  auto Bbuf = [&](int buf) { return lds + 2 * A_STAGE + buf * B_STAGE; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // tile decomposition; blocks share only the layer's weights (L2-resident everywhere)
  int bid = blockIdx.x;
  const int ks = bid % g.ksplit;
  bid /= g.ksplit;
  const int nt = bid % g.n_tiles;
  bid /= g.n_tiles;
  const int tx = bid % g.tiles_x;
  bid /= g.tiles_x;
  const int ty = bid % g.tiles_y;
  const int tb = bid / g.tiles_y;
  const int b0 = tb * g.IMGS, y0 = ty * g.TH, x0 = tx * g.TW;
  const int n0 = nt * BN;
  const int HW_ = g.TW + 2, HH = g.TH + 2;
  const int NH = g.IMGS * HH * HW_;          // halo pixels of this tile
  const int s_lo = (int)((int64_t)ks * g.nslab / g.ksplit);
  const int s_hi = (int)((int64_t)(ks + 1) * g.nslab / g.ksplit);

  // ---- staging map (fixed over slabs)
  int64_t a_src[A_PER_T];
  int a_dst[A_PER_T];
#pragma unroll
  for (int j = 0; j < A_PER_T; ++j) {
    const int f = tid + kThreads * j;
    const int hp = f >> 2, q = f & 3;
    a_src[j] = -1;
    a_dst[j] = -1;
    if (hp < NH) {
      const int img = hp / (HH * HW_);
      const int rem = hp - img * HH * HW_;
      const int hy = rem / HW_, hx = rem - hy * HW_;
      const int b = b0 + img, y = y0 + hy - 1, x = x0 + hx - 1;
      a_dst[j] = hp * kApitch + 4 * q;
      if (b < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd)
        a_src[j] = (((int64_t)b * g.H + y) * g.Wd + x) * g.ldx + 4 * q;
    }
  }
  f4 ra[A_PER_T], rb[B_PER_T];
  auto load = [&](int slab) {
    const int c0 = slab * 16;
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
      const bool ok = a_src[j] >= 0 && c0 + 4 * ((tid + kThreads * j) & 3) < g.C;
      ra[j] = ok ? *(const f4*)(g.X + a_src[j] + c0) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      const int f = tid + kThreads * j;
      if (f < B_F4) {
        const int row = f >> 2, q = f & 3;  // row = n * 9 + tap
        const int n = row / 9, tap = row - n * 9;
        rb[j] = *(const f4*)(g.W + ((int64_t)(n0 + n) * 9 + tap) * g.ldw + c0 + 4 * q);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j)
      if (a_dst[j] >= 0) *(f4*)(Abuf(buf) + a_dst[j]) = ra[j];
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      const int f = tid + kThreads * j;
      if (f < B_F4) {
        const int row = f >> 2, q = f & 3;
        const int n = row / 9, tap = row - n * 9;
        *(f4*)(Bbuf(buf) + (tap * BN + n) * kBpitch + 4 * q) = rb[j];
      }
    }
  };

  // ---- per-lane fragment addresses
  const int lr = lane & 15, lk = 4 * (lane >> 4);
  int a_off[FM];
  int m_img[FM], m_y[FM], m_x[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = wave * 32 + i * 16 + lr;
    const int img = m / (g.TH * g.TW);
    const int rem = m - img * g.TH * g.TW;
    const int r = rem / g.TW, c = rem - r * g.TW;
    m_img[i] = img;
    m_y[i] = r;
    m_x[i] = c;
    const int im = img < g.IMGS ? img : 0;  // idle slots read a valid address
    a_off[i] = ((im * HH + r + 1) * HW_ + c + 1) * kApitch + lk;
  }
  const int b_off = lr * kBpitch + lk;

  f4 acc[FM][NF];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  if (s_lo < s_hi) {
    load(s_lo);
    store(0);
  }
  __syncthreads();
  for (int s = s_lo; s < s_hi; ++s) {
    const int buf = (s - s_lo) & 1;
    if (s + 1 < s_hi) load(s + 1);
    const float* A = Abuf(buf);
    const float* Bw = Bbuf(buf);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = ((tap / 3 - 1) * HW_ + (tap % 3 - 1)) * kApitch;
      f4 fa[FM], fb[NF];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = *(const f4*)(A + a_off[i] + toff);
#pragma unroll
      for (int j = 0; j < NF; ++j) fb[j] = *(const f4*)(Bw + (tap * BN + j * 16) * kBpitch + b_off);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][t], fb[j][t], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < s_hi) store(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds rows (lane>>4)*4 + r of each 16x16 fragment, column lane&15
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = wave * 32 + i * 16 + (lane >> 4) * 4 + r;
      const int img = m / (g.TH * g.TW);
      const int rem = m - img * g.TH * g.TW;
      const int ry = rem / g.TW, rx = rem - ry * g.TW;
      const int b = b0 + img, y = y0 + ry, x = x0 + rx;
      if (img >= g.IMGS || b >= g.B || y >= g.H || x >= g.Wd) continue;
      const int64_t p = ((int64_t)b * g.H + y) * g.Wd + x;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int n = n0 + j * 16 + lr;
        if (n >= g.N) continue;
        if (g.ksplit == 1) {
          g.out[p * g.ldo + n] = act_fn(acc[i][j][r] + tap_bias(g, n, y, x), g.act, g.slope);
        } else {
          g.part[((int64_t)ks * ((int64_t)g.B * g.H * g.Wd) + p) * g.ldp + n] = acc[i][j][r];
        }
      }
    }
  }
  (void)m_img;
  (void)m_y;
  (void)m_x;
}

// fixed-order sum of the split-K partials, then bias + activation
__global__ void __launch_bounds__(256) conv3_reduce_kernel(HaloArgs g) {
  const int64_t P = (int64_t)g.B * g.H * g.Wd;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * g.N) return;
  const int64_t p = i / g.N;
  const int n = (int)(i - p * g.N);
  float s = g.part[p * g.ldp + n];
  for (int k = 1; k < g.ksplit; ++k) s = s + g.part[((int64_t)k * P + p) * g.ldp + n];
  const int64_t rem = p % ((int64_t)g.H * g.Wd);
  const int y = (int)(rem / g.Wd), x = (int)(rem % g.Wd);
  g.out[p * g.ldo + n] = act_fn(s + tap_bias(g, n, y, x), g.act, g.slope);
}

// Tile shape and split for an image geometry (never the batch size).
struct HaloPlan {
  int IMGS, TH, TW, ksplit;
};

static HaloPlan halo_plan(int H, int W, int nslab, int nf) {
  const int kMaxHalo = max_halo(nf);
  HaloPlan pl;
  pl.TW = W < 32 ? W : 32;
  pl.TH = 256 / pl.TW;
  if (pl.TH > H) pl.TH = H;
  pl.IMGS = 1;
  if (pl.TH == H) {
    pl.IMGS = 256 / (pl.TH * pl.TW);
    if (pl.IMGS < 1) pl.IMGS = 1;
  }
  while (pl.IMGS > 1 && pl.IMGS * (pl.TH + 2) * (pl.TW + 2) > kMaxHalo) --pl.IMGS;
  while (pl.IMGS == 1 && (pl.TH + 2) * (pl.TW + 2) > kMaxHalo && pl.TH > 1) --pl.TH;
  // small images: split K so that a batch still spreads over the CUs
  const int px = H * W;
  pl.ksplit = px <= 64 ? 4 : (px <= 144 ? 2 : 1);
  if (pl.ksplit > nslab) pl.ksplit = nslab > 0 ? nslab : 1;
  return pl;
}

}  // namespace idf

using namespace idf;

// workspace floats needed by idf_conv3x3_halo for the split-K partials
extern "C" int64_t idf_conv3x3_halo_workspace(int32_t B, int32_t H, int32_t W, int32_t C,
                                              int32_t N) {
  const int nslab = (C + 15) / 16;
  const int nft = (N + 15) / 16;
  HaloPlan pl = halo_plan(H, W, nslab, nft <= 4 ? nft : 4);
  if (pl.ksplit <= 1) return 0;
  return (int64_t)pl.ksplit * B * H * W * ((N + 3) / 4 * 4);
}

extern "C" int idf_conv3x3_halo(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                                const float* x, int64_t ld_x, const float* w, int32_t ldw,
                                int32_t n_alloc, const float* b3, const float* vtap, int32_t ldv,
                                const float* bfull, int32_t N, float* out, int64_t ld_out,
                                int32_t act, float slope, float* workspace,
                                int64_t workspace_floats) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || (ld_x & 3) || (ldw & 15) || ldw < ((C + 15) / 16) * 16) return IDF_ERR_ARG;
  const int nf_total = (N + 15) / 16;
  const int NF = nf_total <= 4 ? nf_total : 4;
  const int n_tiles = (nf_total + NF - 1) / NF;
  if (n_alloc < n_tiles * NF * 16) return IDF_ERR_ARG;
  HaloArgs g = {};
  g.X = x; g.ldx = ld_x; g.C = C; g.W = w; g.ldw = ldw; g.N = N;
  g.B = B; g.H = H; g.Wd = W;
  g.nslab = (C + 15) / 16;
  HaloPlan pl = halo_plan(H, W, g.nslab, NF);
  g.IMGS = pl.IMGS; g.TH = pl.TH; g.TW = pl.TW; g.ksplit = pl.ksplit;
  g.tiles_b = (B + pl.IMGS - 1) / pl.IMGS;
  g.tiles_y = (H + pl.TH - 1) / pl.TH;
  g.tiles_x = (W + pl.TW - 1) / pl.TW;
  g.n_tiles = n_tiles;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out;
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  if (pl.ksplit > 1) {
    g.ldp = (N + 3) / 4 * 4;
    if (!workspace || workspace_floats < (int64_t)pl.ksplit * B * H * W * g.ldp)
      return IDF_ERR_WORKSPACE;
    g.part = workspace;
  }
  const int64_t blocks = (int64_t)g.tiles_b * g.tiles_y * g.tiles_x * n_tiles * pl.ksplit;
  hipStream_t s = (hipStream_t)stream;
  switch (NF) {
    case 1: hipLaunchKernelGGL(conv3_halo_kernel<1>, dim3((unsigned)blocks), dim3(kThreads), 0, s, g); break;
    case 2: hipLaunchKernelGGL(conv3_halo_kernel<2>, dim3((unsigned)blocks), dim3(kThreads), 0, s, g); break;
    case 3: hipLaunchKernelGGL(conv3_halo_kernel<3>, dim3((unsigned)blocks), dim3(kThreads), 0, s, g); break;
    default: hipLaunchKernelGGL(conv3_halo_kernel<4>, dim3((unsigned)blocks), dim3(kThreads), 0, s, g); break;
  }
  if (pl.ksplit > 1) {
    const int64_t n = (int64_t)B * H * W * N;
    hipLaunchKernelGGL(conv3_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
  }
  return idf_last_error();
}
