// conv3_bf16.hip -- the DenseLayer 3x3 convolution (1x1 folded in) on bf16 MFMA, for the
// configs that name bf16 coupling convolutions (BASELINE configs[2]: resflow-cond-imagenet64).
//
// out[p, n] = act(bias(p, n) + sum_{tap, c} bf16(X[nbr(p, tap), c]) * Wb[n, tap, c])
// with fp32 accumulation (v_mfma_f32_16x16x32_bf16).  X stays fp32 in HBM (the DenseBlock
// feature buffer); the halo of each 32-channel slab is converted to bf16 (round to nearest
// even, v_cvt_pk_bf16_f32) on its way into LDS.  Wb is packed on the host
// (idfcodec/packing.py bf16_weights) in MFMA fragment order
// [slab][tap][4 k-blocks of 8 channels][n_alloc][8 bf16], so a wave's B operand for one
// (tap, n-fragment) is one conflict-free 1 KiB ds_read_b128.
//
// Block = 8 waves, a tile of up to 512 output pixels (32 row-fragments) x 48 outputs; wave w
// owns row-fragments w, w+8, w+16, w+24 and all NF n-fragments (4 x NF accumulators).  Per
// slab: the (TH+2) x (TW+2) halo (IMGS images) in a k-block-major image [4][kMaxSlots][8 bf16]
// (16 B per (k-block, pixel); 16 consecutive pixels of a row-fragment = one 256-B run: no bank
// conflicts), and the slab's 9 x 4 x n_alloc x 16 B of weights.  Both are staged through
// registers one slab ahead (double-buffered LDS), one barrier per slab.
// The sum order (slab-major, tap-minor, 32 channels per MFMA) depends on the weights' shape
// only; small images split the slabs (from H, W -- never the batch) with a fixed-order reduce:
// deterministic and batch-invariant, so the decoder reproduces the encoder exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "idf_codec_internal.h"

#pragma clang fp contract(off)

namespace idf {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4b __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

constexpr int kBThreads = 512;
constexpr int kBMaxSlots = 800;      // halo pixels per stage
constexpr int kBMaxNF = 3;           // n-fragments (48 outputs) per block

struct Bf16Args {
  const float* X;
  int64_t ldx;
  int32_t C;
  const uint16_t* Wb;  // [nslab][9][4][n_alloc][8]
  int32_t nslab, n_alloc;
  int32_t N;
  int32_t B, H, Wd;
  int32_t IMGS, TH, TW;
  int32_t tiles_b, tiles_y, tiles_x, ksplit;
  const float* b3;
  const float* vtap;
  const float* bfull;
  int32_t ldv;
  int32_t act;
  float slope;
  float* out;
  int64_t ldo;
  float* part;
  int32_t ldp;
};

__device__ __forceinline__ float bact(float v, int act, float slope) {
  if (act == IDF_ACT_RELU) return v > 0.0f ? v : 0.0f;
  if (act == IDF_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  if (act == IDF_ACT_TANH) return tanhf(v);
  return v;
}

__device__ __forceinline__ float bbias(const Bf16Args& g, int n, int y, int x) {
  if (!g.vtap) return g.b3[n];
  if (y >= 1 && y <= g.H - 2 && x >= 1 && x <= g.Wd - 2) return g.bfull[n];
  float bsum = g.b3[n];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int ny = y + tap / 3 - 1, nx = x + tap % 3 - 1;
    if (ny >= 0 && ny < g.H && nx >= 0 && nx < g.Wd) bsum = bsum + g.vtap[tap * g.ldv + n];
  }
  return bsum;
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const __bf16 x = (__bf16)a, y = (__bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

template <int NF>
__global__ void __launch_bounds__(kBThreads) conv3_bf16_kernel(Bf16Args g) {
  constexpr int A_STAGE = 4 * kBMaxSlots * 8;     // bf16 elements
  constexpr int B_STAGE = 9 * 4 * NF * 16 * 8;    // bf16 elements
  constexpr int A_PER_T = (kBMaxSlots * 4 + kBThreads - 1) / kBThreads;  // 8-channel chunks
  constexpr int B_PER_T = (B_STAGE / 8 + kBThreads - 1) / kBThreads;     // 16-B chunks
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * (A_STAGE + B_STAGE)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid = blockIdx.x;
  const int ks = bid % g.ksplit;
  bid /= g.ksplit;
  const int tx_ = bid % g.tiles_x;
  bid /= g.tiles_x;
  const int ty_ = bid % g.tiles_y;
  const int tb = bid / g.tiles_y;
  const int b0 = tb * g.IMGS, y0 = ty_ * g.TH, x0 = tx_ * g.TW;
  const int HWp = g.TW + 2, HH = g.TH + 2;
  const int NH = g.IMGS * HH * HWp;
  const int TPX = g.TH * g.TW;  // output pixels per image in the tile
  const int s_lo = (int)((int64_t)ks * g.nslab / g.ksplit);
  const int s_hi = (int)((int64_t)(ks + 1) * g.nslab / g.ksplit);

  // ---- halo staging map: chunk f = slot * 4 + kb (8 channels of one halo pixel)
  int64_t a_src[A_PER_T];  // float offset of channel 8*kb of the pixel (slab 0), -1 = zero
  int a_dst[A_PER_T];      // bf16 offset in the stage, -1 = none
#pragma unroll
  for (int j = 0; j < A_PER_T; ++j) {
    const int f = tid + kBThreads * j;
    const int slot = f >> 2, kb = f & 3;
    a_src[j] = -1;
    a_dst[j] = -1;
    if (slot < NH) {
      a_dst[j] = (kb * kBMaxSlots + slot) * 8;
      const int img = slot / (HH * HWp);
      const int rem = slot - img * HH * HWp;
      const int hy = rem / HWp, hx = rem - hy * HWp;
      const int y = y0 + hy - 1, x = x0 + hx - 1;
      if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd)
        a_src[j] = (((int64_t)(b0 + img) * g.H + y) * g.Wd + x) * g.ldx + 8 * kb;
    }
  }
  u4 ra[A_PER_T];
  u4 rb[B_PER_T];
  auto load = [&](int slab) {
    const int c0 = slab * 32;
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
      const int kb = (tid + kBThreads * j) & 3;
      const int c = c0 + 8 * kb;
      f4b v0 = f4b{0.f, 0.f, 0.f, 0.f}, v1 = v0;
      if (a_src[j] >= 0) {
        const float* p = g.X + a_src[j] + c0;
        if (c < g.C) v0 = *(const f4b*)p;
        if (c + 4 < g.C) v1 = *(const f4b*)(p + 4);
      }
      ra[j] = u4{pack2(v0[0], v0[1]), pack2(v0[2], v0[3]), pack2(v1[0], v1[1]), pack2(v1[2], v1[3])};
    }
    const uint16_t* wsrc = g.Wb + (int64_t)slab * B_STAGE;
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      const int f = tid + kBThreads * j;
      if (f < B_STAGE / 8) rb[j] = *(const u4*)(wsrc + f * 8);
    }
  };
  auto store = [&](int buf) {
    uint16_t* As = lds + buf * (A_STAGE + B_STAGE);
    uint16_t* Bs = As + A_STAGE;
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j)
      if (a_dst[j] >= 0) *(u4*)(As + a_dst[j]) = ra[j];
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
      const int f = tid + kBThreads * j;
      if (f < B_STAGE / 8) *(u4*)(Bs + f * 8) = rb[j];
    }
  };

  // ---- per-lane row-fragment bases (slot of the output pixel's halo centre)
  const int lr = lane & 15, kb = lane >> 4;
  int cslot[4];
  bool rvalid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = 16 * (wave + 8 * i) + lr;
    int img = t / TPX;
    const int rem = t - img * TPX;
    const int ty = rem / g.TW, tx = rem - ty * g.TW;
    rvalid[i] = img < g.IMGS;
    if (!rvalid[i]) img = 0;
    cslot[i] = (img * HH + ty + 1) * HWp + tx + 1;
  }

  f4b acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f4b{0.f, 0.f, 0.f, 0.f};

  if (s_lo < s_hi) {
    load(s_lo);
    store(0);
  }
  __syncthreads();
  for (int s = s_lo; s < s_hi; ++s) {
    const int buf = (s - s_lo) & 1;
    const bool more = s + 1 < s_hi;
    if (more) load(s + 1);
    const uint16_t* As = lds + buf * (A_STAGE + B_STAGE) + kb * kBMaxSlots * 8;
    const uint16_t* Bs = lds + buf * (A_STAGE + B_STAGE) + A_STAGE;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int off = (tap / 3 - 1) * HWp + (tap % 3 - 1);
      bf8 a[4], b[NF];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *(const bf8*)(As + (cslot[i] + off) * 8);
#pragma unroll
      for (int j = 0; j < NF; ++j)
        b[j] = *(const bf8*)(Bs + (((tap * 4 + kb) * (NF * 16)) + j * 16 + lr) * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds rows (lane>>4)*4 + r of each row-fragment, column lane&15
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int n = j * 16 + lr;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 16 * (wave + 8 * i) + (lane >> 4) * 4 + r;
        const int img = t / TPX;
        if (img >= g.IMGS) continue;
        const int rem = t - img * TPX;
        const int ty = rem / g.TW, tx = rem - ty * g.TW;
        const int b = b0 + img, y = y0 + ty, x = x0 + tx;
        if (b >= g.B || y >= g.H || x >= g.Wd) continue;
        const int64_t p = ((int64_t)b * g.H + y) * g.Wd + x;
        if (g.ksplit == 1)
          g.out[p * g.ldo + n] = bact(acc[i][j][r] + bbias(g, n, y, x), g.act, g.slope);
        else
          g.part[((int64_t)ks * ((int64_t)g.B * g.H * g.Wd) + p) * g.ldp + n] = acc[i][j][r];
      }
    }
  }
}

__global__ void __launch_bounds__(256) conv3_bf16_reduce_kernel(Bf16Args g) {
  const int64_t P = (int64_t)g.B * g.H * g.Wd;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * g.N) return;
  const int64_t p = i / g.N;
  const int n = (int)(i - p * g.N);
  float s = g.part[p * g.ldp + n];
  for (int k = 1; k < g.ksplit; ++k) s = s + g.part[((int64_t)k * P + p) * g.ldp + n];
  const int64_t rem = p % ((int64_t)g.H * g.Wd);
  const int y = (int)(rem / g.Wd), x = (int)(rem % g.Wd);
  g.out[p * g.ldo + n] = bact(s + bbias(g, n, y, x), g.act, g.slope);
}

struct Bf16Plan {
  int IMGS, TH, TW, ksplit;
};

// Tile and split from the image geometry only (never the batch size).
static Bf16Plan bf16_plan(int H, int W, int nslab) {
  Bf16Plan pl;
  pl.TW = W < 32 ? W : 32;
  pl.TH = 512 / pl.TW;
  if (pl.TH > H) pl.TH = H;
  pl.IMGS = 1;
  if (pl.TH == H) {
    pl.IMGS = 512 / (pl.TH * pl.TW);
    if (pl.IMGS < 1) pl.IMGS = 1;
  }
  while (pl.IMGS > 1 && pl.IMGS * (pl.TH + 2) * (pl.TW + 2) > kBMaxSlots) --pl.IMGS;
  while (pl.IMGS == 1 && (pl.TH + 2) * (pl.TW + 2) > kBMaxSlots && pl.TH > 1) --pl.TH;
  const int px = H * W;
  pl.ksplit = px <= 64 ? 2 : 1;
  if (pl.ksplit > nslab) pl.ksplit = nslab > 0 ? nslab : 1;
  return pl;
}

}  // namespace idf

using namespace idf;

extern "C" int64_t idf_conv3x3_bf16_workspace(int32_t B, int32_t H, int32_t W, int32_t C,
                                              int32_t N) {
  Bf16Plan pl = bf16_plan(H, W, (C + 31) / 32);
  if (pl.ksplit <= 1) return 0;
  return (int64_t)pl.ksplit * B * H * W * ((N + 3) / 4 * 4);
}

extern "C" int idf_conv3x3_bf16(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                                const float* x, int64_t ld_x, const uint16_t* wb, int32_t n_alloc,
                                const float* b3, const float* vtap, int32_t ldv,
                                const float* bfull, int32_t N, float* out, int64_t ld_out,
                                int32_t act, float slope, float* workspace,
                                int64_t workspace_floats) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || (ld_x & 3) || !wb) return IDF_ERR_ARG;
  const int nf = (N + 15) / 16;
  if (nf > kBMaxNF || n_alloc != nf * 16) return IDF_ERR_ARG;
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  Bf16Args g = {};
  g.X = x; g.ldx = ld_x; g.C = C; g.Wb = wb; g.nslab = (C + 31) / 32; g.n_alloc = n_alloc;
  g.N = N; g.B = B; g.H = H; g.Wd = W;
  Bf16Plan pl = bf16_plan(H, W, g.nslab);
  g.IMGS = pl.IMGS; g.TH = pl.TH; g.TW = pl.TW; g.ksplit = pl.ksplit;
  g.tiles_b = (B + pl.IMGS - 1) / pl.IMGS;
  g.tiles_y = (H + pl.TH - 1) / pl.TH;
  g.tiles_x = (W + pl.TW - 1) / pl.TW;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out;
  if (pl.ksplit > 1) {
    g.ldp = (N + 3) / 4 * 4;
    if (!workspace || workspace_floats < (int64_t)pl.ksplit * B * H * W * g.ldp)
      return IDF_ERR_WORKSPACE;
    g.part = workspace;
  }
  const int64_t blocks = (int64_t)g.tiles_b * g.tiles_y * g.tiles_x * pl.ksplit;
  hipStream_t s = (hipStream_t)stream;
  switch (nf) {
    case 1: hipLaunchKernelGGL(conv3_bf16_kernel<1>, dim3((unsigned)blocks), dim3(kBThreads), 0, s, g); break;
    case 2: hipLaunchKernelGGL(conv3_bf16_kernel<2>, dim3((unsigned)blocks), dim3(kBThreads), 0, s, g); break;
    default: hipLaunchKernelGGL(conv3_bf16_kernel<3>, dim3((unsigned)blocks), dim3(kBThreads), 0, s, g); break;
  }
  if (pl.ksplit > 1) {
    const int64_t n = (int64_t)B * H * W * N;
    hipLaunchKernelGGL(conv3_bf16_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       g);
  }
  return idf_last_error();
}
