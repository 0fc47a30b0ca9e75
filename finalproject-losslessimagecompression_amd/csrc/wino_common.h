// wino_common.h -- helpers shared by the 3x3 conv kernels (conv3_wino.hip, conv3_dx3.hip):
// tile planning, halo pitch, B^T rows, fast index division, activations.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "idf_codec_internal.h"

namespace idf {

constexpr int kWMaxHalo = 400;   // halo pixel slots used per stage
// Small images packed many to a block (config 4's 4x4 / 2x2 levels: 16 or 64 images of
// 36 or 16 halo pixels) use a 1024-slot stage instead: 2 x 64 KiB of LDS, which costs no
// occupancy (the kernel is VGPR-limited to one 8-wave block per CU either way).
constexpr int kWSlotsBig = 1024;

__device__ __forceinline__ float wact(float v, int act, float slope) {
  if (act == IDF_ACT_RELU) return v > 0.0f ? v : 0.0f;
  if (act == IDF_ACT_LEAKY) return v > 0.0f ? v : v * slope;
  if (act == IDF_ACT_TANH) return tanhf(v);
  return v;
}

// wact without a branch per value (the epilogue's ReLU / LeakyReLU / identity): the same bits
// as wact for those three -- v > 0 keeps v; else ReLU gives +0, LeakyReLU v * slope, identity
// v * 1 = v (NaN: +0 for ReLU, NaN otherwise, as wact).  Tanh layers take wact.
struct WAct {
  float mul;   // v <= 0: v * mul (LeakyReLU slope, identity 1)
  bool zero;   // ReLU
  bool tanh_;
  __device__ explicit WAct(int act, float slope)
      : mul(act == IDF_ACT_LEAKY ? slope : 1.0f), zero(act == IDF_ACT_RELU),
        tanh_(act == IDF_ACT_TANH) {}
  __device__ __forceinline__ float operator()(float v) const {
    const float neg = zero ? 0.0f : v * mul;
    return v > 0.0f ? v : neg;
  }
};

// a / b for 0 <= a < 2^20, 1 <= b < 2^20, exact: the float estimate is within 0.25 of a / b,
// one remainder step corrects its truncation.  ~6 instructions instead of the ~35 of a
// general 32-bit division: the kernel's index maps (halo slots, tiles, the block index) take
// a dozen or more per thread, all before its first load.
__device__ __forceinline__ int udiv_s(int a, int b) {
  int q = (int)((float)a * __builtin_amdgcn_rcpf((float)b));
  const int r = a - q * b;
  return q + (r >= b) - (r < 0);
}

// XCD-aware block order of the Winograd kernels (idf_codec_internal.h xcd_contiguous): the
// neighbouring tiles of an image run on one XCD and read their shared halo rows through its L2.
__device__ __forceinline__ int wino_xcd_remap(int bid, int nwg) { return xcd_contiguous(bid, nwg); }

// B^T of F(2,3): row a combines d[I0(a)] (sign S0(a)) and d[I1(a)] (sign S1(a)).
template <int a> struct BT {
  static constexpr int i0 = a == 0 ? 0 : 1;
  static constexpr int i1 = a == 3 ? 3 : 2;
  static constexpr bool neg0 = a == 2;
  static constexpr bool neg1 = a == 0 || a == 3;
};

// Halo row pitch (slots) for an output tile TW wide: TW + 2, plus 2 when a 16-tile MFMA
// fragment spans two rows of 8 tiles (TW = 16).  Its two rows' slots then differ by 8 mod 16
// and every ds_read_b128 lane group of the halo reads hits 16 distinct bank quads; at 18 they
// differed by 36 = 4 mod 16 and half of the group collided (SQ_LDS_BANK_CONFLICT 2x the LDS
// cycles of the 16x16 level).  TW = 32 fragments lie in one tile row; TW = 8 rows land 0/4/8/12.
__host__ __device__ constexpr int halo_pitch(int tw) { return tw + 2 + (tw == 16 ? 2 : 0); }

struct WinoPlan {
  int ok, IMGS, TH, TW, ksplit, big;
};

// Output tile and split for an image geometry (never the batch size).  Odd H or W are
// tiled as the next even size: the extra row/column of 2x2 tiles reads zero padding
// (out-of-image halo) and its outputs are never stored, so every stored pixel sees the
// same 3x3 neighbourhood as in the direct conv.
// Output tile width of images exactly 32 wide (imagenet64's 32x32 level): 16 (16x16 blocks, 4 per
// image; bench +0.7% same-box over 32x8 strips, profiles/r03/session2/tw_ab.txt) unless
// IDF_WINO_TW32=32.  The tiling never changes a tile's arithmetic: the outputs are the same
// bits either way.
static inline int wino_tw_32() {
  static const int tw = [] {
    const char* e = getenv("IDF_WINO_TW32");
    return e && atoi(e) == 32 ? 32 : 16;
  }();
  return tw;
}

// Output tile width of images wider than 32 (the VQ-VAE's convs): 32 unless IDF_WINO_TWW=16.
static inline int wino_tw_wide() {
  static const int tw = [] {
    const char* e = getenv("IDF_WINO_TWW");
    return e && atoi(e) == 16 ? 16 : 32;
  }();
  return tw;
}

static inline WinoPlan wino_plan(int H, int W, int nslab, int N) {
  WinoPlan pl = {0, 1, 0, 0, 1, 0};
  if (H < 1 || W < 1) return pl;
  const int He = (H + 1) & ~1, We = (W + 1) & ~1;
  pl.TW = We < 32 ? We : (We == 32 ? wino_tw_32() : wino_tw_wide());
  pl.TH = 256 / pl.TW;  // 64 wino tiles = 256 output pixels
  if (pl.TH > He) pl.TH = He;
  if (pl.TH & 1) pl.TH -= 1;
  if (pl.TH < 2) return pl;
  if (pl.TH < He) {
    // balance the row tiles: same tile count, least overhang below the image
    const int nty = (He + pl.TH - 1) / pl.TH;
    pl.TH = ((He + nty - 1) / nty + 1) & ~1;
  }
  if (pl.TH == He) {
    pl.IMGS = 256 / (pl.TH * pl.TW);
    if (pl.IMGS < 1) pl.IMGS = 1;
  }
  const int want = pl.IMGS, halo = (pl.TH + 2) * halo_pitch(pl.TW);
  while (pl.IMGS > 1 && pl.IMGS * halo > kWMaxHalo) --pl.IMGS;
  if (pl.IMGS < want) {  // whole small images: pack up to 64 tiles in the big stage
    pl.big = 1;
    pl.IMGS = want;
    while (pl.IMGS > 1 && pl.IMGS * halo > kWSlotsBig) --pl.IMGS;
  }
  if (halo > kWMaxHalo) return pl;
  const int px = H * W;
  pl.ksplit = px <= 64 ? 4 : (px <= 144 ? 2 : 1);
  // Blocks come from the pixels, the n-tiles and the split.  Packed small images (64 tiles of
  // whole images per block) and wide outputs (several n-tiles: the VQ-VAE's 384/512-channel
  // convs) have enough blocks without splitting K, and the split's partial-sum round trip
  // and reduce then cost more than they gain (measured: config 4 5.4 -> 8.3 Mpx/s, config 3's
  // VQ-VAE 67 -> 54 ms; imagenet64's 8x8 level keeps 4: 10.2 vs 9.6 Mpx/s with 1).
  if (pl.big || N > 64) pl.ksplit = 1;
  if (pl.ksplit > nslab) pl.ksplit = nslab > 0 ? nslab : 1;
  pl.ok = 1;
  return pl;
}

}  // namespace idf
