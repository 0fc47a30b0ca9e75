// conv3_bf16.hip -- the DenseLayer 3x3 convolution (1x1 folded in) on bf16 MFMA, for the
// configs that name bf16 coupling convolutions (BASELINE configs[2]: resflow-cond-imagenet64).
//
// out[p, n] = act(bias(p, n) + sum_{tap, c} X16[nbr(p, tap), c] * Wb[n, tap, c])
// with fp32 accumulation (v_mfma_f32_16x16x32_bf16).  X16 is the bf16 shadow of the
// DenseBlock's fp32 feature buffer (every column rounded to nearest even, v_cvt_pk_bf16_f32,
// once, by the layer that produced it): each layer stores its activated output in fp32
// (the 1x1 head and the flow read those) AND in bf16 into the shadow, so the next layers'
// halos reach LDS by direct DMA (buffer_load ... lds, 16 B per lane) with no register staging
// or conversion.  Wb is packed on the host (idfcodec/packing.py bf16_weights) in MFMA
// fragment order [slab][tap][4 k-blocks of 8 channels][n_alloc][8 bf16], so a wave's B
// operand for one (tap, n-fragment) is one conflict-free 1 KiB ds_read_b128; it is DMA'd too.
//
// Block = 8 waves, a tile of up to 512 output pixels (32 row-fragments) x 48 outputs; wave w
// owns row-fragments w, w+8, w+16, w+24 and all NF n-fragments (4 x NF accumulators).  Per
// 32-channel slab: the (TH+2) x (TW+2) halo (IMGS images) in a k-block-major image
// [4][kBMaxSlots][8 bf16] (16 consecutive pixels of a row-fragment = one 256-B run: no bank
// conflicts) and the slab's 9 x 4 x n_alloc x 16 B of weights, double-buffered: slab s+1's
// DMA is in flight under slab s's 108 MFMAs per wave; one barrier per slab.  Within a slab
// the 9 taps are software-pipelined (tap t+1's 4 + NF fragment reads issued before tap t's
// MFMAs).  The shadow's pitch is a multiple of 64 channels (dense_block_run), so a pixel's
// 32-channel slab is one 64-B run inside one 128-B line: with an 8-channel pitch half the runs
// straddled two lines and the L0 c=496 launch took 806 instead of 650 us.
// The sum order (slab-major, tap-minor, 32 channels per MFMA) depends on the weights' shape
// only; small images split the slabs (from H, W -- never the batch) with a fixed-order reduce:
// deterministic and batch-invariant, so the decoder reproduces the encoder exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "idf_codec_internal.h"

#pragma clang fp contract(off)

// Timing-only ablations for tools/native/bf16_ablate (never set in the library build):
// bit 0 skips the per-slab DMA after the first, bit 1 the LDS fragment reads after the
// first tap, bit 2 the MFMAs, bit 3 the per-slab barrier.
#ifndef IDF_BF16_ABLATE
#define IDF_BF16_ABLATE 0
#endif

namespace idf {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4b __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_b;

constexpr int kBThreads = 512;
constexpr int kBMaxHalo = 800;       // halo pixels per stage the plan may use
constexpr int kBMaxSlots = 832;      // slots per k-block (13 DMA blocks of 64; 16-slot multiple)
constexpr int kBMaxNF = 3;           // n-fragments (48 outputs) per block
constexpr uint32_t kBInvalid = 0xFFFFFFF0u;  // buffer offset that always reads 0

struct Bf16Args {
  const uint16_t* X16;
  int64_t ldx16;
  int32_t C;
  const uint16_t* Wb;  // [nslab][9][4][n_alloc][8]
  int32_t nslab, n_alloc;
  int32_t N, N16;
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
  uint16_t* out16;
  int64_t ldo16;
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

__device__ __forceinline__ uint16_t bf16_bits(float v) {
  return __builtin_bit_cast(uint16_t, (__bf16)v);
}

template <int NF>
__global__ void __launch_bounds__(kBThreads) conv3_bf16_kernel(Bf16Args g) {
  constexpr int A_STAGE = 4 * kBMaxSlots * 8;     // bf16 elements
  constexpr int B_STAGE = 9 * 4 * NF * 16 * 8;    // bf16 elements
  constexpr int STAGE = A_STAGE + B_STAGE;
  constexpr int NBLK = kBMaxSlots / 64;
  constexpr int XA = (4 * NBLK + 7) / 8;          // halo DMA instructions per wave (max)
  constexpr int NXB = B_STAGE / (8 * 64);         // weight DMA instructions per slab
  constexpr int XB = (NXB + 7) / 8;
  static_assert(kBMaxSlots % 64 == 0 && kBMaxSlots >= kBMaxHalo, "DMA blocks of 64 slots");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = xcd_contiguous(blockIdx.x, gridDim.x);  // neighbouring tiles on one XCD
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

  // ---- halo DMA: instruction f = kb * nblk + blk stages slots [64 blk, 64 blk + 64) of
  // k-block kb; buffer resource over the block's images, out-of-range offsets read 0.
  const int nblk = (NH + 63) >> 6, nxa = 4 * nblk;
  const int64_t img_elems = (int64_t)g.H * g.Wd * g.ldx16;
  const uint16_t* xbase = g.X16 + (int64_t)b0 * img_elems;
  const int64_t xbytes = ((int64_t)g.B - b0) * img_elems * 2;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xbase, 0, (int)(xbytes < (int64_t)kBInvalid ? xbytes : (int64_t)kBInvalid), 0x00020000);
  const int64_t wbytes = (int64_t)g.nslab * B_STAGE * 2;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.Wb, 0, (int)(wbytes < (int64_t)kBInvalid ? wbytes : (int64_t)kBInvalid), 0x00020000);
  uint32_t a_off[XA];  // byte offset of this lane's slot pixel, k-block kb, slab 0
#pragma unroll
  for (int m = 0; m < XA; ++m) {
    const int f = wave + 8 * m;
    a_off[m] = kBInvalid;
    if (f < nxa) {
      const int kb = f / nblk, slot = (f - kb * nblk) * 64 + lane;
      if (slot < NH) {
        const int img = slot / (HH * HWp);
        const int rem = slot - img * HH * HWp;
        const int hy = rem / HWp, hx = rem - hy * HWp;
        const int y = y0 + hy - 1, x = x0 + hx - 1;
        if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd)
          a_off[m] = (uint32_t)(((((int64_t)img * g.H + y) * g.Wd + x) * g.ldx16 + 8 * kb) * 2);
      }
    }
  }
  auto issue = [&](int slab, int buf) {
    uint16_t* As = lds + buf * STAGE;
    uint16_t* Bs = As + A_STAGE;
    const int c0 = slab * 32;
#pragma unroll
    for (int m = 0; m < XA; ++m) {
      const int f = wave + 8 * m;
      if (f < nxa) {
        const int kb = f / nblk, blk = f - kb * nblk;
        const bool ok = a_off[m] != kBInvalid && c0 + 8 * kb < g.C;
        const uint32_t off = ok ? a_off[m] + (uint32_t)c0 * 2u : kBInvalid;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr, (lds_ptr_b)(As + (kb * kBMaxSlots + 64 * blk) * 8), 16, off, 0, 0, 0);
      }
    }
#pragma unroll
    for (int m = 0; m < XB; ++m) {
      const int f = wave + 8 * m;
      if (f < NXB)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            wr, (lds_ptr_b)(Bs + f * 64 * 8), 16,
            (uint32_t)(((int64_t)slab * B_STAGE + (f * 64 + lane) * 8) * 2), 0, 0, 0);
    }
  };

  // ---- per-lane row-fragment bases (slot of the output pixel's halo centre)
  const int lr = lane & 15, kb = lane >> 4;
  int cslot[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = 16 * (wave + 8 * i) + lr;
    int img = t / TPX;
    const int rem = t - img * TPX;
    const int ty = rem / g.TW, tx = rem - ty * g.TW;
    if (img >= g.IMGS) img = 0;  // idle rows read valid LDS
    cslot[i] = (img * HH + ty + 1) * HWp + tx + 1;
  }

  f4b acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f4b{0.f, 0.f, 0.f, 0.f};

  if (s_lo < s_hi) issue(s_lo, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int s = s_lo; s < s_hi; ++s) {
    const int buf = (s - s_lo) & 1;
    if (s + 1 < s_hi && !(IDF_BF16_ABLATE & 1)) issue(s + 1, buf ^ 1);
    const uint16_t* As = lds + buf * STAGE + kb * kBMaxSlots * 8;
    const uint16_t* Bs = lds + buf * STAGE + A_STAGE + (kb * (NF * 16) + lr) * 8;
    bf8 a[2][4], b[2][NF];
    auto fetch = [&](int tap, bf8 (&av)[4], bf8 (&bv)[NF]) {
      const int off = (tap / 3 - 1) * HWp + (tap % 3 - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = *(const bf8*)(As + (cslot[i] + off) * 8);
#pragma unroll
      for (int j = 0; j < NF; ++j) bv[j] = *(const bf8*)(Bs + (tap * 4 * NF * 16 + j * 16) * 8);
    };
    fetch(0, a[0], b[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap < 8 && !(IDF_BF16_ABLATE & 2)) fetch(tap + 1, a[(tap + 1) & 1], b[(tap + 1) & 1]);
      if (tap < 8 && (IDF_BF16_ABLATE & 2)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[(tap + 1) & 1][i] = a[tap & 1][i];
#pragma unroll
        for (int j = 0; j < NF; ++j) b[(tap + 1) & 1][j] = b[tap & 1][j];
      }
      __builtin_amdgcn_sched_barrier(0);  // keep tap t+1's reads ahead of tap t's MFMAs
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j)
          if (!(IDF_BF16_ABLATE & 4))
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tap & 1][i], b[tap & 1][j],
                                                                acc[i][j], 0, 0, 0);
          else
            acc[i][j][0] += (float)a[tap & 1][i][0] * (float)b[tap & 1][j][1];
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slab s+1 has landed
    if (!(IDF_BF16_ABLATE & 8)) __syncthreads();       // and every wave is done with slab s
  }

  // ---- epilogue: lane holds rows (lane>>4)*4 + r of each row-fragment, column lane&15.
  // The bias table goes through LDS (the stages are free after the last barrier).
  float* btab = (float*)lds;
  if (g.ksplit == 1) {
    stage_bias(btab, NF * 16, 0, g.N, g.b3, g.vtap, g.bfull, g.ldv, tid, kBThreads);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
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
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int n = j * 16 + lr;
        if (n >= g.N) continue;
        if (g.ksplit == 1) {
          const float v = bact(acc[i][j][r] + btab[bias_class(y, x, g.H, g.Wd) * (NF * 16) + n],
                               g.act, g.slope);
          g.out[p * g.ldo + n] = v;
          g.out16[p * g.ldo16 + n] = bf16_bits(v);
        } else {
          g.part[((int64_t)ks * ((int64_t)g.B * g.H * g.Wd) + p) * g.ldp + n] = acc[i][j][r];
        }
      }
      // shadow columns [N, N16): zeros, so the next layer's partial 8-channel k-block
      // multiplies zero weights by zeros
      if (ks == 0 && lr < g.N16 - g.N) g.out16[p * g.ldo16 + g.N + lr] = 0;
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
  const float v = bact(s + bbias(g, n, y, x), g.act, g.slope);
  g.out[p * g.ldo + n] = v;
  g.out16[p * g.ldo16 + n] = bf16_bits(v);
}

// fp32 columns -> bf16 shadow columns (round to nearest even); zeros for [n, n_zero).
__global__ void f32_to_bf16_cols_kernel(int64_t P, int32_t n, int32_t nz, const float* __restrict__ src,
                                        int64_t lds_, uint16_t* __restrict__ dst, int64_t ldd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * nz) return;
  const int64_t p = i / nz;
  const int c = (int)(i - p * nz);
  dst[p * ldd + c] = c < n ? bf16_bits(src[p * lds_ + c]) : (uint16_t)0;
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
  while (pl.IMGS > 1 && pl.IMGS * (pl.TH + 2) * (pl.TW + 2) > kBMaxHalo) --pl.IMGS;
  while (pl.IMGS == 1 && (pl.TH + 2) * (pl.TW + 2) > kBMaxHalo && pl.TH > 1) --pl.TH;
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

extern "C" int idf_f32_to_bf16_cols(void* stream, int64_t P, int32_t n, int32_t n_zero,
                                    const float* src, int64_t ld_src, uint16_t* dst,
                                    int64_t ld_dst) {
  if (P < 0 || n < 0 || n_zero < n || (n > 0 && !src) || !dst) return IDF_ERR_ARG;
  const int64_t total = P * n_zero;
  if (total == 0) return IDF_OK;
  hipLaunchKernelGGL(f32_to_bf16_cols_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P, n, n_zero, src, ld_src, dst, ld_dst);
  return idf_last_error();
}

extern "C" int idf_conv3x3_bf16(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                                const uint16_t* x16, int64_t ld_x16, const uint16_t* wb,
                                int32_t n_alloc, const float* b3, const float* vtap, int32_t ldv,
                                const float* bfull, int32_t N, float* out, int64_t ld_out,
                                uint16_t* out16, int64_t ld_out16, int32_t n16, int32_t act,
                                float slope, float* workspace, int64_t workspace_floats) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || (ld_x16 & 7) || !wb || !x16 || !out || !out16) return IDF_ERR_ARG;
  if (((uintptr_t)x16 & 15) || ((uintptr_t)wb & 15)) return IDF_ERR_ARG;
  const int nf = (N + 15) / 16;
  if (nf > kBMaxNF || n_alloc != nf * 16) return IDF_ERR_ARG;
  if (n16 < N || n16 > N + 15) return IDF_ERR_ARG;
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  Bf16Args g = {};
  g.X16 = x16; g.ldx16 = ld_x16; g.C = C; g.Wb = wb; g.nslab = (C + 31) / 32; g.n_alloc = n_alloc;
  g.N = N; g.N16 = n16; g.B = B; g.H = H; g.Wd = W;
  Bf16Plan pl = bf16_plan(H, W, g.nslab);
  // per-block buffer offsets are 32-bit: the block's images must span < 4 GiB
  if ((int64_t)pl.IMGS * H * W * ld_x16 * 2 >= (int64_t)kBInvalid) return IDF_ERR_UNSUPPORTED;
  if ((int64_t)g.nslab * 9 * 4 * nf * 16 * 8 * 2 >= (int64_t)kBInvalid) return IDF_ERR_UNSUPPORTED;
  g.IMGS = pl.IMGS; g.TH = pl.TH; g.TW = pl.TW; g.ksplit = pl.ksplit;
  g.tiles_b = (B + pl.IMGS - 1) / pl.IMGS;
  g.tiles_y = (H + pl.TH - 1) / pl.TH;
  g.tiles_x = (W + pl.TW - 1) / pl.TW;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out; g.out16 = out16; g.ldo16 = ld_out16;
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
