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
// Wave w owns transform positions (a, b) = (w/2, 2(w%2)) and (w/2, 2(w%2)+1) for all 64
// tiles; the pair shares its B^T row a, so each wave forms three row combinations
// R[j] = s0*d[i0][j] + s1*d[i1][j] and both V's from them (24 LDS reads + 5 vector
// add/subs per 16 tiles x 4 channels; the signs are compile-time per wave group).
// Per 16-channel slab:
//   * the tile's (rows+2) x (cols+2) halo of X is staged into LDS once through
//     range-checked buffer loads (out-of-image / out-of-channel elements read as 0,
//     branch-free), columns de-interleaved (even columns, then odd) so the stride-2
//     patch reads of 16 neighbouring tiles are unit-stride, conflict-free ds_read_b128s;
//   * U fragments are pre-arranged on the host in MFMA fragment order, so each wave
//     streams its 2 x NF fragments with coalesced 1-KiB loads straight into registers,
//     one slab ahead;
//   * 2 positions x 4 tile-frags x NF n-frags x 4 k-steps of v_mfma_f32_16x16x4_f32,
//     with the next tile-fragment's LDS reads issued ahead of each MFMA group.
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
constexpr int kWMaxHalo = 400;   // halo pixel slots per stage (+1 trash slot)
constexpr int kWMsPitch = 17;    // M staging: floats per (position, tile) row of 16 n
constexpr uint32_t kWInvalid = 0xFFFFFFF0u;  // buffer offset that always reads 0

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

// B^T of F(2,3): row a combines d[I0(a)] (sign S0(a)) and d[I1(a)] (sign S1(a)).
template <int a> struct BT {
  static constexpr int i0 = a == 0 ? 0 : 1;
  static constexpr int i1 = a == 3 ? 3 : 2;
  static constexpr bool neg0 = a == 2;
  static constexpr bool neg1 = a == 0 || a == 3;
};

template <bool NEG0, bool NEG1>
__device__ __forceinline__ w4 comb(w4 x0, w4 x1) {
  if (!NEG0 && !NEG1) return x0 + x1;
  if (!NEG0 && NEG1) return x0 - x1;
  if (NEG0 && !NEG1) return x1 - x0;
  return -(x0 + x1);
}

// Column slot of halo column j (0..3) relative to a tile's even-half base, de-interleaved.
__device__ __forceinline__ int colslot(int j, int EH) { return (j & 1) ? EH + (j >> 1) : (j >> 1); }

// One slab of MFMAs for a wave whose positions are (A, 2*BP) and (A, 2*BP + 1).
template <int NF, int A, int BP>
__device__ __forceinline__ void wino_slab(const float* __restrict__ lds_a, const int (&tbase)[4],
                                          int HWp, int EH, int lk, const w4 (&u)[2][NF],
                                          w4 (&acc)[2][4][NF]) {
  using RA = BT<A>;
  constexpr int b0 = 2 * BP, b1 = 2 * BP + 1;
  using C0 = BT<b0>;
  using C1 = BT<b1>;
  // the three halo columns the pair needs: {0,1,2} (BP=0) or {1,2,3} (BP=1)
  constexpr int j0 = BP, j1 = BP + 1, j2 = BP + 2;
  const int r0 = RA::i0 * HWp, r1 = RA::i1 * HWp;
  const int cs0 = colslot(j0, EH), cs1 = colslot(j1, EH), cs2 = colslot(j2, EH);
  const int o00 = (r0 + cs0) * kWPitch + lk, o01 = (r0 + cs1) * kWPitch + lk,
            o02 = (r0 + cs2) * kWPitch + lk;
  const int o10 = (r1 + cs0) * kWPitch + lk, o11 = (r1 + cs1) * kWPitch + lk,
            o12 = (r1 + cs2) * kWPitch + lk;
  w4 d[6];
  auto fetch = [&](int i) {
    const float* P = lds_a + tbase[i] * kWPitch;
    d[0] = *(const w4*)(P + o00);
    d[1] = *(const w4*)(P + o01);
    d[2] = *(const w4*)(P + o02);
    d[3] = *(const w4*)(P + o10);
    d[4] = *(const w4*)(P + o11);
    d[5] = *(const w4*)(P + o12);
  };
  fetch(0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // rows: R[j] = s0 d[i0][j] + s1 d[i1][j]
    const w4 R0 = comb<RA::neg0, RA::neg1>(d[0], d[3]);
    const w4 R1 = comb<RA::neg0, RA::neg1>(d[1], d[4]);
    const w4 R2 = comb<RA::neg0, RA::neg1>(d[2], d[5]);
    // columns of position b: its two columns among {j0, j1, j2}
    auto pick = [&](int j) -> w4 { return j == j0 ? R0 : (j == j1 ? R1 : R2); };
    const w4 v0 = comb<C0::neg0, C0::neg1>(pick(C0::i0), pick(C0::i1));
    const w4 v1 = comb<C1::neg0, C1::neg1>(pick(C1::i0), pick(C1::i1));
    if (i + 1 < 4) fetch(i + 1);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int jn = 0; jn < NF; ++jn) {
        acc[0][i][jn] = __builtin_amdgcn_mfma_f32_16x16x4f32(v0[t], u[0][jn][t], acc[0][i][jn], 0, 0, 0);
        acc[1][i][jn] = __builtin_amdgcn_mfma_f32_16x16x4f32(v1[t], u[1][jn][t], acc[1][i][jn], 0, 0, 0);
      }
  }
}

template <int NF>
__global__ void __launch_bounds__(kWThreads) conv3_wino_kernel(WinoArgs g) {
  constexpr int A_STAGE = (kWMaxHalo + 1) * kWPitch;
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
  const int nf0 = nt * NF;

  // ---- halo staging: buffer resource over the block's images; invalid -> reads 0
  const float* xbase = g.X + (int64_t)b0 * g.H * g.Wd * g.ldx;
  const int64_t xbytes = ((int64_t)g.B * g.H * g.Wd * g.ldx - (int64_t)b0 * g.H * g.Wd * g.ldx) * 4;
  const int nrec = (int)(xbytes < (int64_t)kWInvalid ? xbytes : (int64_t)kWInvalid);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)xbase, 0, nrec, 0x00020000);
  uint32_t a_src[A_PER_T];  // byte offset of the pixel's channel 4q (slab 0), or kWInvalid
  int a_dst[A_PER_T];       // LDS float offset (trash slot when beyond the halo)
#pragma unroll
  for (int j = 0; j < A_PER_T; ++j) {
    const int f = tid + kWThreads * j;
    const int hp = f >> 2, q = f & 3;
    a_src[j] = kWInvalid;
    a_dst[j] = kWMaxHalo * kWPitch;  // trash slot
    if (hp < NH) {
      const int img = hp / (HH * HWp);
      const int rem = hp - img * HH * HWp;
      const int hy = rem / HWp, hx = rem - hy * HWp;
      const int slot = (img * HH + hy) * HWp + ((hx & 1) ? EH + (hx >> 1) : (hx >> 1));
      a_dst[j] = slot * kWPitch + 4 * q;
      const int y = y0 + hy - 1, x = x0 + hx - 1;
      if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd)
        a_src[j] = (uint32_t)(((((int64_t)img * g.H + y) * g.Wd + x) * g.ldx + 4 * q) * 4);
    }
  }
  w4 ra[A_PER_T];
  auto load_halo = [&](int slab) {
    const int c0 = slab * 16;
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
      const bool ok = a_src[j] != kWInvalid && c0 + 4 * ((tid + kWThreads * j) & 3) < g.C;
      const uint32_t off = ok ? a_src[j] + (uint32_t)c0 * 4u : kWInvalid;
      ra[j] = __builtin_bit_cast(w4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto store_halo = [&](int buf) {
    float* Ab = lds + buf * A_STAGE;
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) *(w4*)(Ab + a_dst[j]) = ra[j];
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
  const int wg = wave;  // wave-uniform: selects (a, b-pair)
  for (int s = s_lo; s < s_hi; ++s) {
    const int buf = (s - s_lo) & 1;
    const bool more = s + 1 < s_hi;
    if (more) {
      load_halo(s + 1);
      load_u(s + 1, unxt);
    }
    const float* Ab = lds + buf * A_STAGE;
    switch (wg) {
      case 0: wino_slab<NF, 0, 0>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
      case 1: wino_slab<NF, 0, 1>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
      case 2: wino_slab<NF, 1, 0>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
      case 3: wino_slab<NF, 1, 1>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
      case 4: wino_slab<NF, 2, 0>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
      case 5: wino_slab<NF, 2, 1>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
      case 6: wino_slab<NF, 3, 0>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
      default: wino_slab<NF, 3, 1>(Ab, tbase, HWp, EH, lk, ucur, acc); break;
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
  // per-block buffer offsets are 32-bit: the block's images must span < 4 GiB
  if ((int64_t)pl.IMGS * H * W * ld_x * 4 >= (int64_t)kWInvalid) return IDF_ERR_UNSUPPORTED;
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
