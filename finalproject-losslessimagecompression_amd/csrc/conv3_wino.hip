// conv3_wino.hip -- the DenseLayer 3x3 convolution as Winograd F(2x2, 3x3) on gfx950.
//
// out = act(bias + conv3x3(X, W)) computed per 2x2 output tile as
//   Y = A^T [ sum_c U_c (.) V_c ] A,  V_c = B^T d_c B (4x4 input patch),  U_c = G g_c G^T,
// i.e. 16 independent GEMMs (one per transform position) of [tiles x C] x [C x N]:
// 16 multiplies per 4 outputs instead of 36 -- 2.25x fewer MFMA FLOPs than the direct
// conv (conv3_halo.hip).  All transforms of F(2,3) have entries in {0, +-1, +-1/2}; U is
// formed in float64 on the host and rounded once (idfcodec/packing.py wino_weights), the
// V and Y transforms are +-1 sums evaluated in a fixed order: deterministic, and within
// the flow's 1e-5 parity tolerance (tests/test_gpu_wino.py).
//
// Block = 8 waves, one spatial tile of up to 64 Winograd tiles (e.g. 8x32 output pixels
// at 32x32, a whole 16x16 image, or four 8x8 images) x all N outputs of an n-tile.
// Wave w owns transform positions 2w and 2w+1 (of 16) for all 64 tiles.  Per
// 16-channel slab:
//   * the tile's (rows+2) x (cols+2) halo of X is staged into LDS once, columns
//     de-interleaved (even columns, then odd) so the stride-2 patch reads of 16
//     neighbouring tiles are unit-stride, conflict-free ds_read_b128s;
//   * each wave builds its V fragments on the fly (4 LDS reads + 3 vector adds per
//     16 tiles x 4 channels) -- V never touches LDS;
//   * U fragments are pre-arranged on the host in MFMA fragment order, so each wave
//     streams its 2 x NF fragments with coalesced 1-KiB loads straight into registers,
//     one slab ahead;
//   * 2 positions x 4 tile-frags x NF n-frags x 4 k-steps of v_mfma_f32_16x16x4_f32.
// After the last slab the accumulators (M) go through LDS one n-fragment at a time for
// the cross-position output transform, bias (incl. the folded 1x1 bias per valid tap),
// activation and store.  Small images split the slab range (ksplit, fixed by H, W, C)
// into partial Y tiles that conv3_wino_reduce_kernel sums in fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "idf_codec_internal.h"

#pragma clang fp contract(off)

namespace idf {

typedef float w4 __attribute__((ext_vector_type(4)));

struct WinoArgs {
  const float* X;
  int64_t ldx;
  int32_t C;
  const float* U;  // [16][nslab][nft][64 lanes][4]
  int32_t nslab, nft;
  int32_t N;
  int32_t B, H, Wd;
  int32_t IMGS, TH, TW;  // output tile (TH, TW even)
  int32_t tiles_b, tiles_y, tiles_x, n_tiles, ksplit;
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

constexpr int kWThreads = 512;
constexpr int kWPitch = 24;      // floats per halo pixel slot (16 channels + 8 pad)
constexpr int kWMaxHalo = 400;   // halo pixel slots per stage
constexpr int kWMsPitch = 17;    // M staging: floats per (position, tile) row of 16 n

__device__ __forceinline__ float wact(float v, int act, float slope) {
  if (act == IDF_ACT_RELU) return v > 0.0f ? v : 0.0f;
  if (act == IDF_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  if (act == IDF_ACT_TANH) return tanhf(v);
  return v;
}

__device__ __forceinline__ float wbias(const WinoArgs& g, int n, int y, int x) {
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

// B^T row a of F(2,3): V[a][.] = s0 * d[i0][.] + s1 * d[i1][.]
__device__ __forceinline__ void bt_row(int a, int& i0, int& i1, float& s0, float& s1) {
  i0 = a == 0 ? 0 : 1;
  i1 = a == 3 ? 3 : 2;
  s0 = a == 2 ? -1.0f : 1.0f;
  s1 = (a == 0 || a == 3) ? -1.0f : 1.0f;
}

template <int NF>
__global__ void __launch_bounds__(kWThreads) conv3_wino_kernel(WinoArgs g) {
  constexpr int A_STAGE = kWMaxHalo * kWPitch;
  constexpr int A_PER_T = (kWMaxHalo * 4 + kWThreads - 1) / kWThreads;
  static_assert(16 * 64 * kWMsPitch <= 2 * A_STAGE, "M staging aliases the halo buffers");
  __shared__ __attribute__((aligned(16))) float lds[2 * A_STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid = blockIdx.x;
  const int ks = bid % g.ksplit;
  bid /= g.ksplit;
  const int nt = bid % g.n_tiles;
  bid /= g.n_tiles;
  const int tx_ = bid % g.tiles_x;
  bid /= g.tiles_x;
  const int ty_ = bid % g.tiles_y;
  const int tb = bid / g.tiles_y;
  const int b0 = tb * g.IMGS, y0 = ty_ * g.TH, x0 = tx_ * g.TW;
  const int HWp = g.TW + 2, HH = g.TH + 2, EH = (HWp + 1) >> 1;
  const int NH = g.IMGS * HH * HWp;
  const int TTH = g.TH >> 1, TTW = g.TW >> 1, TPI = TTH * TTW;  // wino tiles per image
  const int s_lo = (int)((int64_t)ks * g.nslab / g.ksplit);
  const int s_hi = (int)((int64_t)(ks + 1) * g.nslab / g.ksplit);
  const int nf0 = nt * NF;  // first global n-fragment of this block

  // ---- halo staging map: pixel (img, hy, hx) -> de-interleaved slot
  int64_t a_src[A_PER_T];
  int a_dst[A_PER_T];
#pragma unroll
  for (int j = 0; j < A_PER_T; ++j) {
    const int f = tid + kWThreads * j;
    const int hp = f >> 2, q = f & 3;
    a_src[j] = -1;
    a_dst[j] = -1;
    if (hp < NH) {
      const int img = hp / (HH * HWp);
      const int rem = hp - img * HH * HWp;
      const int hy = rem / HWp, hx = rem - hy * HWp;
      const int slot = (img * HH + hy) * HWp + ((hx & 1) ? EH + (hx >> 1) : (hx >> 1));
      a_dst[j] = slot * kWPitch + 4 * q;
      const int b = b0 + img, y = y0 + hy - 1, x = x0 + hx - 1;
      if (b < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd)
        a_src[j] = (((int64_t)b * g.H + y) * g.Wd + x) * g.ldx + 4 * q;
    }
  }
  w4 ra[A_PER_T];
  auto load_halo = [&](int slab) {
    const int c0 = slab * 16;
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
      const bool ok = a_src[j] >= 0 && c0 + 4 * ((tid + kWThreads * j) & 3) < g.C;
      ra[j] = ok ? *(const w4*)(g.X + a_src[j] + c0) : w4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_halo = [&](int buf) {
    float* A = lds + buf * A_STAGE;
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j)
      if (a_dst[j] >= 0) *(w4*)(A + a_dst[j]) = ra[j];
  };
  // ---- U fragments (registers, one slab ahead)
  w4 ucur[2][NF], unxt[2][NF];
  auto load_u = [&](int slab, w4 (&u)[2][NF]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = 2 * wave + q;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int64_t o = ((((int64_t)p * g.nslab + slab) * g.nft + nf0 + j) * 64 + lane) * 4;
        u[q][j] = *(const w4*)(g.U + o);
      }
    }
  };

  // ---- per-lane tile bases (slot of the patch's top-left, even-column half)
  const int lr = lane & 15, lk = 4 * (lane >> 4);
  int tbase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = 16 * i + lr;
    int img = t / TPI;
    const int rem = t - img * TPI;
    const int ty = rem / TTW, tx = rem - ty * TTW;
    if (img >= g.IMGS) img = 0;  // idle rows read valid LDS
    tbase[i] = (img * HH + 2 * ty) * HWp + tx;
  }
  int pi0[2], pi1[2], pj0[2], pj1[2];
  float ps0[2], ps1[2], pt0[2], pt1[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = 2 * wave + q;
    bt_row(p >> 2, pi0[q], pi1[q], ps0[q], ps1[q]);
    bt_row(p & 3, pj0[q], pj1[q], pt0[q], pt1[q]);
  }
  auto col = [&](int j) { return (j & 1) ? EH + (j >> 1) : (j >> 1); };

  w4 acc[2][4][NF];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[q][i][j] = w4{0.f, 0.f, 0.f, 0.f};

  if (s_lo < s_hi) {
    load_halo(s_lo);
    load_u(s_lo, ucur);
    store_halo(0);
  }
  __syncthreads();
  for (int s = s_lo; s < s_hi; ++s) {
    const int buf = (s - s_lo) & 1;
    const bool more = s + 1 < s_hi;
    if (more) {
      load_halo(s + 1);
      load_u(s + 1, unxt);
    }
    const float* A = lds + buf * A_STAGE;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int o00 = (pi0[q] * HWp + col(pj0[q])) * kWPitch + lk;
      const int o01 = (pi0[q] * HWp + col(pj1[q])) * kWPitch + lk;
      const int o10 = (pi1[q] * HWp + col(pj0[q])) * kWPitch + lk;
      const int o11 = (pi1[q] * HWp + col(pj1[q])) * kWPitch + lk;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float* P = A + tbase[i] * kWPitch;
        const w4 d00 = *(const w4*)(P + o00), d01 = *(const w4*)(P + o01);
        const w4 d10 = *(const w4*)(P + o10), d11 = *(const w4*)(P + o11);
        const w4 r0 = d00 * pt0[q] + d01 * pt1[q];
        const w4 r1 = d10 * pt0[q] + d11 * pt1[q];
        const w4 v = r0 * ps0[q] + r1 * ps1[q];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < NF; ++j)
            acc[q][i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[t], ucur[q][j][t], acc[q][i][j], 0, 0, 0);
      }
    }
    if (more) {
      store_halo(buf ^ 1);
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < NF; ++j) ucur[q][j] = unxt[q][j];
    }
    __syncthreads();
  }

  // ---- output transform, one n-fragment at a time through LDS
  float* Ms = lds;  // [16 pos][64 tiles][kWMsPitch]
#pragma unroll
  for (int j = 0; j < NF; ++j) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = 2 * wave + q;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = 16 * i + (lane >> 4) * 4 + r;
          Ms[(p * 64 + t) * kWMsPitch + lr] = acc[q][i][j][r];
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int item = tid + kWThreads * it;
      const int t = item >> 4, nn = item & 15;
      int img = t / TPI;
      const int rem = t - img * TPI;
      const int ty = rem / TTW, tx = rem - ty * TTW;
      const int n = (nf0 + j) * 16 + nn;
      if (img < g.IMGS && n < g.N) {
        float m[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) m[a][b] = Ms[((a * 4 + b) * 64 + t) * kWMsPitch + nn];
        // A^T m: rows (m0 + m1 + m2), (m1 - m2 - m3); then the same over columns
        float u0[4], u1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          u0[b] = (m[0][b] + m[1][b]) + m[2][b];
          u1[b] = (m[1][b] - m[2][b]) - m[3][b];
        }
        float Y[2][2];
        Y[0][0] = (u0[0] + u0[1]) + u0[2];
        Y[0][1] = (u0[1] - u0[2]) - u0[3];
        Y[1][0] = (u1[0] + u1[1]) + u1[2];
        Y[1][1] = (u1[1] - u1[2]) - u1[3];
        const int b = b0 + img;
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int y = y0 + 2 * ty + r, x = x0 + 2 * tx + c;
            if (b >= g.B || y >= g.H || x >= g.Wd) continue;
            const int64_t p = ((int64_t)b * g.H + y) * g.Wd + x;
            if (g.ksplit == 1)
              g.out[p * g.ldo + n] = wact(Y[r][c] + wbias(g, n, y, x), g.act, g.slope);
            else
              g.part[((int64_t)ks * ((int64_t)g.B * g.H * g.Wd) + p) * g.ldp + n] = Y[r][c];
          }
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) conv3_wino_reduce_kernel(WinoArgs g) {
  const int64_t P = (int64_t)g.B * g.H * g.Wd;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * g.N) return;
  const int64_t p = i / g.N;
  const int n = (int)(i - p * g.N);
  float s = g.part[p * g.ldp + n];
  for (int k = 1; k < g.ksplit; ++k) s = s + g.part[((int64_t)k * P + p) * g.ldp + n];
  const int64_t rem = p % ((int64_t)g.H * g.Wd);
  const int y = (int)(rem / g.Wd), x = (int)(rem % g.Wd);
  g.out[p * g.ldo + n] = wact(s + wbias(g, n, y, x), g.act, g.slope);
}

struct WinoPlan {
  int ok, IMGS, TH, TW, ksplit;
};

// Output tile and split for an image geometry (never the batch size).
static WinoPlan wino_plan(int H, int W, int nslab) {
  WinoPlan pl = {0, 1, 0, 0, 1};
  if ((H & 1) || (W & 1) || H < 2 || W < 2) return pl;
  pl.TW = W < 32 ? W : 32;
  pl.TH = 256 / pl.TW;  // 64 wino tiles = 256 output pixels
  if (pl.TH > H) pl.TH = H;
  if (pl.TH & 1) pl.TH -= 1;
  if (pl.TH < 2) return pl;
  if (pl.TH == H) {
    pl.IMGS = 256 / (pl.TH * pl.TW);
    if (pl.IMGS < 1) pl.IMGS = 1;
  }
  while (pl.IMGS > 1 && pl.IMGS * (pl.TH + 2) * (pl.TW + 2) > kWMaxHalo) --pl.IMGS;
  if ((pl.TH + 2) * (pl.TW + 2) > kWMaxHalo) return pl;
  const int px = H * W;
  pl.ksplit = px <= 64 ? 4 : (px <= 144 ? 2 : 1);
  if (pl.ksplit > nslab) pl.ksplit = nslab > 0 ? nslab : 1;
  pl.ok = 1;
  return pl;
}

}  // namespace idf

using namespace idf;

extern "C" int idf_conv3x3_wino_supported(int32_t H, int32_t W) {
  return wino_plan(H, W, 1).ok;
}

extern "C" int64_t idf_conv3x3_wino_workspace(int32_t B, int32_t H, int32_t W, int32_t C,
                                              int32_t N) {
  WinoPlan pl = wino_plan(H, W, (C + 15) / 16);
  if (!pl.ok || pl.ksplit <= 1) return 0;
  return (int64_t)pl.ksplit * B * H * W * ((N + 3) / 4 * 4);
}

extern "C" int idf_conv3x3_wino(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                                const float* x, int64_t ld_x, const float* u, int32_t nft,
                                const float* b3, const float* vtap, int32_t ldv,
                                const float* bfull, int32_t N, float* out, int64_t ld_out,
                                int32_t act, float slope, float* workspace,
                                int64_t workspace_floats) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || (ld_x & 3) || !u) return IDF_ERR_ARG;
  const int nf_total = (N + 15) / 16;
  if (nft < nf_total) return IDF_ERR_ARG;
  const int NF = nf_total <= 2 ? nf_total : (nf_total % 3 == 0 ? 3 : (nf_total % 2 == 0 ? 2 : 1));
  WinoArgs g = {};
  g.X = x; g.ldx = ld_x; g.C = C; g.U = u; g.nslab = (C + 15) / 16; g.nft = nft; g.N = N;
  g.B = B; g.H = H; g.Wd = W;
  WinoPlan pl = wino_plan(H, W, g.nslab);
  if (!pl.ok) return IDF_ERR_UNSUPPORTED;
  g.IMGS = pl.IMGS; g.TH = pl.TH; g.TW = pl.TW; g.ksplit = pl.ksplit;
  g.tiles_b = (B + pl.IMGS - 1) / pl.IMGS;
  g.tiles_y = (H + pl.TH - 1) / pl.TH;
  g.tiles_x = (W + pl.TW - 1) / pl.TW;
  g.n_tiles = (nf_total + NF - 1) / NF;
  if (g.n_tiles * NF > nft) return IDF_ERR_ARG;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out;
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  if (pl.ksplit > 1) {
    g.ldp = (N + 3) / 4 * 4;
    if (!workspace || workspace_floats < (int64_t)pl.ksplit * B * H * W * g.ldp)
      return IDF_ERR_WORKSPACE;
    g.part = workspace;
  }
  const int64_t blocks = (int64_t)g.tiles_b * g.tiles_y * g.tiles_x * g.n_tiles * pl.ksplit;
  hipStream_t s = (hipStream_t)stream;
  switch (NF) {
    case 1: hipLaunchKernelGGL(conv3_wino_kernel<1>, dim3((unsigned)blocks), dim3(kWThreads), 0, s, g); break;
    case 2: hipLaunchKernelGGL(conv3_wino_kernel<2>, dim3((unsigned)blocks), dim3(kWThreads), 0, s, g); break;
    default: hipLaunchKernelGGL(conv3_wino_kernel<3>, dim3((unsigned)blocks), dim3(kWThreads), 0, s, g); break;
  }
  if (pl.ksplit > 1) {
    const int64_t n = (int64_t)B * H * W * N;
    hipLaunchKernelGGL(conv3_wino_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       s, g);
  }
  return idf_last_error();
}
