// idf_codec_internal.h -- shared internals of libidfcodec (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/idf_codec.h"

// The fused DenseBlock launch on the direct convs (conv3_dx3.hip conv3_dx3_block_kernel; used
// by flow_kernels.hip dense_block_run): every layer of a block in one launch, one workgroup per
// tile, for geometries whose tiles hold whole images.  Bit for bit the same outputs, split
// copy, fused-head results and range-guard flag as one idf_conv3x3_dx3 / dxb launch per layer.
struct IdfDx3BlockDesc {
  int32_t bf;                    // 0: split-f16 (dx3), 1: bf16 (dxb)
  int32_t B, H, W, nlayers, N, nft, ldv, act, nslab_xs;
  float slope;
  uint16_t* xs;                  // the block's split (bf16) feature copy
  const int32_t* C;              // [nlayers] input channels
  const uint16_t* const* w;      // [nlayers] dx3 / dxb weights
  const float* yscale;           // [nlayers] (dx3)
  const float* const* b3;
  const float* const* vtap;
  const float* const* bfull;
  float* feat;                   // layer i's fp32 outputs at feat + C[i] (rows of ld_feat)
  int64_t ld_feat;
  uint32_t* flag;                // range guard (dx3)
  const IdfDx3Head* head;        // fused head: w / ldw / n_head / skip_f32 / out (acc unused),
                                 // the sums kept in registers; nullptr: none
  const float* hx;               // the head init's block input (fp32 rows of hld_x), hc0 channels
  int64_t hld_x;
  int32_t hc0;
  const float* hb;               // the head bias
};
int idf_dx3_block_launch(void* stream, const IdfDx3BlockDesc* d);

// marker written by rans_cdf_freq for scale == 0 (freq can never be INT32_MIN)
#define IDF_FREQ_SCALE_ZERO ((int32_t)0x80000000)

static inline int idf_last_error() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? IDF_OK : IDF_ERR_HIP;
}

namespace idf {

// XCD-aware block order: the dispatcher deals blocks round-robin over the 8 XCDs (block b on
// XCD b % 8); this bijection gives XCD x a contiguous range of tile indices instead, so tiles
// that share input rows (conv halos) run on one XCD and share its L2.  Which block computes a
// tile changes, never the tile's arithmetic.
__device__ __forceinline__ int xcd_contiguous(int bid, int nwg) {
#ifdef IDF_XCD_OFF  // timing-only A/B builds (tools/gpu_xcd_res_ab.sh): the dispatcher's order
  return bid;
#endif
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + idx;
}

// Border class of an output pixel for the folded 1x1 bias: bit 0 y == 0, bit 1 y == H-1,
// bit 2 x == 0, bit 3 x == W-1 (class 0 = interior).
__device__ __forceinline__ int bias_class(int y, int x, int H, int W) {
  return (y == 0) | ((y == H - 1) << 1) | ((x == 0) << 2) | ((x == W - 1) << 3);
}

// Stage the epilogue's bias table in LDS: tab[cls * nn + k] for output column n0 + k (k < nn)
// = b3 (no fold), bfull (interior) or b3 + the vtap of every in-image tap, summed in tap
// order -- the same values, bit for bit, as evaluating the bias per pixel.  Reading the
// table from LDS keeps the epilogue's global stores free of (possibly aliasing) global bias
// loads, which the compiler would otherwise serialise one round trip per store.
__device__ __forceinline__ void stage_bias(float* tab, int nn, int n0, int N, const float* b3,
                                           const float* vtap, const float* bfull, int ldv,
                                           int tid, int nthreads) {
  for (int e = tid; e < 16 * nn; e += nthreads) {
    const int cls = e / nn, k = e - cls * nn, n = n0 + k;
    float v = 0.0f;
    if (n < N) {
      // every load unconditional and issued together (one round trip), then combined
      v = b3[n];
      if (vtap) {
        float t[9];
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) t[tap] = vtap[tap * ldv + n];
        const float full = bfull[n];
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int dy = tap / 3 - 1, dx = tap % 3 - 1;
          const bool ok = !((dy < 0 && (cls & 1)) || (dy > 0 && (cls & 2)) ||
                            (dx < 0 && (cls & 4)) || (dx > 0 && (cls & 8)));
          v = ok ? v + t[tap] : v;
        }
        v = cls == 0 ? full : v;
      }
    }
    tab[e] = v;
  }
}

}  // namespace idf
