// conv3_dx3.hip -- the DenseLayer 3x3 convolution ("dx3"): direct form, fp32-class products
// as split-f16 pairs on the K=32 f16 MFMA of gfx950.
//
// out = act(bias + conv3x3(X, W)) with the 1x1 folded in (packing.fold_layer).  Each fp32
// operand is an f16 pair, x = xh + xl and w' = w * 2^k = wh + wl (k per layer, host float64),
// and x.w' ~= xh.wh + xl.wh + xh.wl: every f16 x f16 product is exact in f32, the dropped
// xl.wl is ~2^-22 of the product (the same arithmetic as the split-f16 Winograd kernel, wx3,
// conv3_wino.hip -- but with no transform, so the split happens once per staged value, not
// once per transformed value in the loop).  All three products run on
// v_mfma_f32_16x16x32_f16 (A = weights: 16 outputs x 32 k, B = pixels: 32 k x 16 pixels):
//   [wh ; wh] . [xh | xl]           one K=32 MFMA per tap and 16 channels (hi.hi + hi.lo)
//   [wl_t ; wl_t'] . [xh_t | xh_t'] xh.wl of two taps per K=32 MFMA (4 pairs per 16 channels;
//                                   the ninth tap pairs with zeros), so 14 MFMAs cover 16
//                                   channels x 9 taps x 3 products (13.5 is the floor).
// There is no VALU in the loop: the k-loop is LDS reads and MFMAs.
//
// Block = 4 waves = one 16x16 output tile x NF*16 outputs.  Wave w owns output rows
// 4w .. 4w+3 (four 16-pixel B fragments of the MFMA) x all outputs: 4 x NF accumulators.
// Per 16-channel slab the block stages into LDS (through registers: loads issued a slab
// ahead, split, written after the slab's reads are done):
//   * the 18x18 halo as two planes, xh [324 slots][16] and xl [324 slots][16] (32 B per
//     slot: every ds_read_b128 lane group of the fragment reads is bank-conflict-free);
//   * the slab's weights in A-fragment order, wh [9 taps][NF][16 out][16 ch] then wl.
// A pixel fragment (16 pixels of one halo row, one tap column) is read once and feeds the
// 3 output rows x NF fragments that use it (rows share halo rows across kernel rows).
// Each output is one fixed-order sum (slabs, then the tap/product order below) whose order
// depends on C only: batch- and tile-invariant, so encoder and decoder agree bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "idf_codec_internal.h"
#include "wino_common.h"

#pragma clang fp contract(off)

namespace idf {

typedef float d4 __attribute__((ext_vector_type(4)));
typedef _Float16 e4 __attribute__((ext_vector_type(4)));
typedef _Float16 e8 __attribute__((ext_vector_type(8)));

struct Dx3Args {
  const float* X;
  int64_t ldx;
  int32_t C;
  const uint16_t* Wt;  // [nslab][2: hi, lo][9 taps][nft][16 out][16 ch] f16 bits of w * 2^k
  int32_t nslab, nft;
  int32_t N;
  int32_t B, H, Wd;
  int32_t tiles_y, tiles_x;
  const float* b3;
  const float* vtap;
  const float* bfull;
  int32_t ldv;
  int32_t act;
  float slope;
  float* out;
  int64_t ldo;
  float yscale;
  uint32_t* flag;  // bit 0: range guard tripped
};

// timing-only ablations (tools/dx3_ablate.sh builds; never set in the library build):
// 1 no halo loads, 2 no halo split/writes, 4 no weight DMA, 8 no slab barrier, 16 no MFMAs,
// 32 no pixel-fragment LDS reads, 64 no weight-fragment LDS reads
#ifndef IDF_DX3_ABLATE
#define IDF_DX3_ABLATE 0
#endif

constexpr int kDxThreads = 256;
constexpr int kDxCW = 18;                 // halo canvas width (slots) = tile width 16 + 2
constexpr int kDxSlots = kDxCW * kDxCW;   // 324
constexpr int kDxPlane = kDxSlots * 32;   // bytes of one (xh or xl) plane
constexpr uint32_t kDxInvalid = 0xFFFFFFF0u;
// the split-f16 range guards of wx3 (conv3_wino.hip): block inputs |x| < 32768 (f16 max
// 65504), layer outputs |y| < 8192 -- the same bound wx3 puts on its outputs, so a pass may
// mix the two kernels (by geometry) under one guard
constexpr float kDxInGuard = 32768.0f;
constexpr float kDxOutGuard = 8192.0f;

template <int NF>
struct Dx3Lds {
  // one stage = a slab's halo planes and weights; three stages (see the schedule below)
  static constexpr int HI = 0, LO = kDxPlane;
  static constexpr int WOFF = 2 * kDxPlane;       // 20736, 16-B aligned
  static constexpr int WPART = 9 * NF * 512;      // one part (wh or wl) of a slab's weights
  static constexpr int WST = 2 * WPART;           // a multiple of 1 KiB: whole DMA pieces
  static constexpr int STAGE = WOFF + WST;
  static constexpr int NSTAGE = 3;
  static constexpr int ZOFF = NSTAGE * STAGE;     // NF * 512 B of zeros (the odd tap's pair)
  static constexpr int BOFF = ZOFF + NF * 512;    // bias table [16 classes][NF * 16] f32
  static constexpr int BYTES = BOFF + 16 * NF * 16 * 4;
  static constexpr int HU = (kDxSlots * 4 + kDxThreads - 1) / kDxThreads;  // halo loads / thread
  static constexpr int WPIECES = WST / 1024;                                // weight DMA pieces
  static constexpr int WPW = (WPIECES + 3) / 4;                             // ... per wave (max)
};

typedef __attribute__((address_space(3))) void* dx_lds_ptr_t;

// f(integral_constant<int, T>) for T = 0, 1, ... in order: a compile-time unrolled schedule
template <typename F, int... T>
__device__ __forceinline__ void dx_unroll(F&& f, std::integer_sequence<int, T...>) {
  (f(std::integral_constant<int, T>{}), ...);
}

template <int NF, bool CHK>
__global__ void __launch_bounds__(kDxThreads, 1) conv3_dx3_kernel(Dx3Args g) {
  using L = Dx3Lds<NF>;
  static_assert(L::WST % 1024 == 0, "weight stage must be whole 1-KiB DMA pieces");
  static_assert(L::BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char lds[L::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = xcd_contiguous(blockIdx.x, gridDim.x);
  const int tx = bid - udiv_s(bid, g.tiles_x) * g.tiles_x;
  bid = udiv_s(bid, g.tiles_x);
  const int ty = bid - udiv_s(bid, g.tiles_y) * g.tiles_y;
  const int b = udiv_s(bid, g.tiles_y);
  const int x0 = tx * 16, y0 = ty * 16;

  // ---- staging maps.  Halo unit u = tid + 256 i: slot u >> 2, channel quad u & 3 (a load's
  // 64 lanes cover 16 slots x 64 B); its split lands at byte 8u of each plane.
  const int64_t img_f = (int64_t)g.H * g.Wd * g.ldx;  // floats per image
  const float* xbase = g.X + (int64_t)b * img_f;
  const int64_t xbytes = ((int64_t)(g.B - b) * img_f) * 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xbase, 0, (int)(xbytes < (int64_t)kDxInvalid ? xbytes : (int64_t)kDxInvalid), 0x00020000);
  uint32_t hoff[L::HU];
  int hq4[L::HU];
#pragma unroll
  for (int i = 0; i < L::HU; ++i) {
    const int u = tid + kDxThreads * i, slot = u >> 2;
    hq4[i] = 4 * (u & 3);
    hoff[i] = kDxInvalid;
    if (slot < kDxSlots) {
      const int hy = udiv_s(slot, kDxCW), cx = slot - hy * kDxCW;
      const int y = y0 + hy - 1, x = x0 + cx - 1;
      if (y >= 0 && y < g.H && x >= 0 && x < g.Wd)
        hoff[i] = (uint32_t)((((int64_t)y * g.Wd + x) * g.ldx + hq4[i]) * 4);
    }
  }
  const int64_t wbytes = (int64_t)g.nslab * L::WST;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.Wt, 0, (int)(wbytes < (int64_t)kDxInvalid ? wbytes : (int64_t)kDxInvalid), 0x00020000);

  // halo of slab s -> registers; weights of slab s -> stage `buf` by LDS-DMA (1 KiB pieces)
  d4 hraw[L::HU];
  auto load_halo = [&](int s) {
    const int c0 = 16 * s;
#pragma unroll
    for (int i = 0; i < L::HU; ++i) {
      const uint32_t off = (hoff[i] != kDxInvalid && c0 + hq4[i] < g.C) ? hoff[i] + (uint32_t)c0 * 4u
                                                                         : kDxInvalid;
      if (IDF_DX3_ABLATE & 1) hraw[i] = d4{(float)off, 1.f, 2.f, 3.f};
      else hraw[i] = __builtin_bit_cast(d4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto load_w = [&](int s, int buf) {
#pragma unroll
    for (int k = 0; k < L::WPW; ++k) {
      if (IDF_DX3_ABLATE & 4) break;
      const int pc = wave + 4 * k;
      if (pc < L::WPIECES)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            wr, (dx_lds_ptr_t)(lds + buf * L::STAGE + L::WOFF + pc * 1024), 16,
            (uint32_t)(s * L::WST + pc * 1024 + lane * 16), 0, 0, 0);
    }
  };
  float gmax = 0.0f;
  // split + write of staged halo unit i into stage `buf`
  auto store_halo = [&](int buf, int i) {
    if (IDF_DX3_ABLATE & 2) return;
    const int u = tid + kDxThreads * i;
    if (u < kDxSlots * 4) {
      const d4 v = hraw[i];
      const e4 h = __builtin_convertvector(v, e4);
      const e4 l = __builtin_convertvector(v - __builtin_convertvector(h, d4), e4);
      *(e4*)(lds + buf * L::STAGE + L::HI + 8 * u) = h;
      *(e4*)(lds + buf * L::STAGE + L::LO + 8 * u) = l;
      if constexpr (CHK) {
        const float m = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
        gmax = fmaxf(gmax, m);
      }
    }
  };

  // zeros for the odd tap's pair, and the epilogue's bias table (both outside the stages)
  for (int e = tid; e < NF * 512 / 16; e += kDxThreads) *(d4*)(lds + L::ZOFF + 16 * e) = d4{0.f, 0.f, 0.f, 0.f};
  stage_bias((float*)(lds + L::BOFF), NF * 16, 0, g.N, g.b3, g.vtap, g.bfull, g.ldv, tid, kDxThreads);

  // ---- fragment read offsets (bytes from a stage base).  B (pixels): lane (q = lane >> 4,
  // j = lane & 15) reads pixel j of a halo row, 8 channels.  A (weights): output j, 8 channels.
  const int j = lane & 15, q = lane >> 4;
  const int r0 = 4 * wave;
  const int slot0 = r0 * kDxCW + j;
  // [xh | xl] at (halo row r0 + h, column j + dx): q 0,1 hi plane chunk q, q 2,3 lo plane chunk q-2
  const int oP = (q >> 1) * L::LO + slot0 * 32 + (q & 1) * 16;
  // [xh(h, dx 0) | xh(h, dx 1)]
  const int oF = L::HI + slot0 * 32 + (q & 1) * 16 + (q >> 1) * 32;
  // [xh(h, dx 2) | xh(h + 1, dx 2)]
  const int oG = L::HI + slot0 * 32 + (q & 1) * 16 + 64 + (q >> 1) * kDxCW * 32;
  // [wh(tap) ; wh(tap)] at tap t, fragment n: + (t * NF + n) * 512
  const int oAH = L::WOFF + j * 32 + (q & 1) * 16;
  // [wl(dy, 0) ; wl(dy, 1)]: + (3 dy * NF + n) * 512
  const int oAF = L::WOFF + L::WPART + j * 32 + (q & 1) * 16 + (q >> 1) * NF * 512;
  // [wl(0, 2) ; wl(1, 2)]: + n * 512
  const int oAG = L::WOFF + L::WPART + 2 * NF * 512 + j * 32 + (q & 1) * 16 + (q >> 1) * 3 * NF * 512;
  // [0 ; wl(2, 2)]: + n * 512; lanes q < 2 read the zero block (outside the stages)
  const int oAO = L::WOFF + L::WPART + 8 * NF * 512 + j * 32 + (q & 1) * 16;
  const bool zlane = q < 2;
  const char* zO = lds + L::ZOFF + j * 32 + (q & 1) * 16;

  d4 acc[4][NF];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < NF; ++n) acc[m][n] = d4{0.f, 0.f, 0.f, 0.f};

  auto rd = [](const char* p) { return *(const e8*)p; };
  auto mma = [](const e8& a, const e8& bb, d4& c) {
    if (IDF_DX3_ABLATE & 16) c[0] += (float)(a[0] * bb[0]);
    else c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bb, c, 0, 0, 0);
  };
  auto rdB = [&](const char* p) -> e8 {
    if (IDF_DX3_ABLATE & 32) return e8{(_Float16)1, (_Float16)(lane & 7), 0, 0, 0, 0, 0, (_Float16)(p == nullptr)};
    return rd(p);
  };
  auto rdA = [&](const char* p) -> e8 {
    if (IDF_DX3_ABLATE & 64) return e8{(_Float16)2, (_Float16)(lane & 3), 0, 0, 0, 0, 0, (_Float16)(p == nullptr)};
    return rd(p);
  };

  // ---- the slab schedule: 29 steps, each one pixel fragment and the MFMAs that use it.
  //   steps 0-17  (P, dx = t / 6, h = t % 6): [wh ; wh] . [xh | xl](h, dx)
  //   steps 18-23 (F, h = t - 18):           [wl(dy,0) ; wl(dy,1)] . [xh(h,0) | xh(h,1)]
  //   steps 24-28 (G, h = t - 24):           [wl(0,2) ; wl(1,2)] and [0 ; wl(2,2)] . [xh(h,2) | xh(h+1,2)]
  // Pixel fragments are read four steps ahead (a ring of 5 that runs on into the next slab), a
  // phase's weight fragments in the three steps before it (per kernel row dy, so that one
  // phase's rows die as the next phase's arrive).  Three LDS stages: slab s reads stage s%3,
  // writes slab s+1's halo into stage (s+1)%3 (steps 8-13) and issues slab s+2's halo loads
  // into the freed registers (step 14), passes the block barrier at step 20 (so stage (s+1)%3
  // is complete, and every wave has finished slab s-1, i.e. stage (s+2)%3 is free) and then
  // DMAs slab s+2's weights into stage (s+2)%3 (step 22).  One barrier per slab, with MFMAs
  // queued on both sides of it.
  constexpr int RB = 5, DB = RB - 1;  // pixel-fragment ring, prefetch distance
  e8 Bq[RB];
  e8 AS[2][3][NF];  // weight sets: P0 / P2 in 0, P1 / F in 1
  e8 AZ[2][NF];     // G: [wl(0,2) ; wl(1,2)] and [0 ; wl(2,2)]
  auto read_B = [&](const char* st, int t) -> e8 {
    if (t < 18) return rdB(st + oP + ((t % 6) * kDxCW + t / 6) * 32);
    if (t < 24) return rdB(st + oF + (t - 18) * kDxCW * 32);
    return rdB(st + oG + (t - 24) * kDxCW * 32);
  };
  // weight fragments of phase p (0-2: P dx = p, 3: F), kernel row dy
  auto read_A = [&](const char* st, int p, int dy, e8 (&A)[NF]) {
#pragma unroll
    for (int n = 0; n < NF; ++n)
      A[n] = p < 3 ? rdA(st + oAH + ((dy * 3 + p) * NF + n) * 512)
                   : rdA(st + oAF + (3 * dy * NF + n) * 512);
  };
  auto mma_rows = [&](const e8 (&A)[3][NF], const e8& Bv, int h) {
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int m = h - dy;
      if (m < 0 || m > 3) continue;
#pragma unroll
      for (int n = 0; n < NF; ++n) mma(A[dy][n], Bv, acc[m][n]);
    }
  };
  // the block barrier: this wave's LDS writes and weight DMA done (the HU youngest vector-memory
  // operations, slab s+2's halo loads, may stay in flight when `halo_in_flight`), then s_barrier
  auto block_barrier = [](bool halo_in_flight) {
    static_assert(L::HU == 6, "vmcnt below counts the halo loads");
    if (halo_in_flight) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (!(IDF_DX3_ABLATE & 8)) asm volatile("s_barrier" ::: "memory");
  };

  const int nslab = g.nslab;
  if (nslab > 0) {
    load_halo(0);
    load_w(0, 0);
#pragma unroll
    for (int i = 0; i < L::HU; ++i) store_halo(0, i);
    if (nslab > 1) {
      load_halo(1);
      load_w(1, 1);
    }
    block_barrier(false);  // stage 0 complete (the DMA'd weights and every wave's halo writes)
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) read_A(lds, 0, dy, AS[0][dy]);
#pragma unroll
    for (int k = 0; k < DB; ++k) Bq[k] = read_B(lds, k);
  }
  int cs = 0;  // stage of slab s (s % 3)
  for (int s = 0; s < nslab; ++s) {
    const int ns = cs == 2 ? 0 : cs + 1, ns2 = ns == 2 ? 0 : ns + 1;
    const char* cur = lds + cs * L::STAGE;
    const char* nxt = lds + ns * L::STAGE;
    const bool more = s + 1 < nslab;
    auto step = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      __builtin_amdgcn_sched_barrier(0);  // keep the schedule: steps do not mix
      // weights of the next phase, one kernel row per step
      if constexpr (t >= 3 && t < 6) read_A(cur, 1, t - 3, AS[1][t - 3]);
      if constexpr (t >= 9 && t < 12) read_A(cur, 2, t - 9, AS[0][t - 9]);
      if constexpr (t >= 15 && t < 18) read_A(cur, 3, t - 15, AS[1][t - 15]);
      if constexpr (t == 21 || t == 22) {
#pragma unroll
        for (int n = 0; n < NF; ++n) {
          if (t == 21) AZ[0][n] = rdA(cur + oAG + n * 512);
          else AZ[1][n] = rdA(zlane ? zO + n * 512 : cur + oAO + n * 512);
        }
      }
      if constexpr (t == 14) {
        if (s + 2 < nslab) load_halo(s + 2);
      }
      if constexpr (t == 20) {
        if (more) block_barrier(s + 2 < nslab);
      }
      if constexpr (t == 22) {
        if (s + 2 < nslab) load_w(s + 2, ns2);
      }
      if constexpr (t >= 25 && t < 28) read_A(nxt, 0, t - 25, AS[0][t - 25]);
      // pixel fragment DB steps ahead (into the next slab from step 29 - DB, after the barrier)
      if constexpr (t + DB < 29) Bq[(t + DB) % RB] = read_B(cur, t + DB);
      else Bq[(t + DB) % RB] = read_B(nxt, t + DB - 29);
      // the next slab's halo: split + write, one unit per step
      if constexpr (t >= 8 && t < 8 + L::HU) {
        if (more) store_halo(ns, t - 8);
      }
      const e8& Bv = Bq[t % RB];
      if constexpr (t < 18) {
        mma_rows(AS[(t / 6) & 1], Bv, t % 6);
      } else if constexpr (t < 24) {
        mma_rows(AS[1], Bv, t - 18);
      } else {
        const int h = t - 24;
        if (h < 4) {
#pragma unroll
          for (int n = 0; n < NF; ++n) mma(AZ[0][n], Bv, acc[h][n]);
        }
        if (h > 0) {
#pragma unroll
          for (int n = 0; n < NF; ++n) mma(AZ[1][n], Bv, acc[h - 1][n]);
        }
      }
    };
    dx_unroll(step, std::make_integer_sequence<int, 29>{});
    // the ring ran 29 steps: re-align it for the next slab (its fragment k is in (29 + k) % RB)
    {
      e8 f[DB];
#pragma unroll
      for (int k = 0; k < DB; ++k) f[k] = Bq[(29 + k) % RB];
#pragma unroll
      for (int k = 0; k < DB; ++k) Bq[k] = f[k];
    }
    cs = ns;
  }

  // ---- guard: block inputs in range (CHK), NaN anywhere (through the accumulators)
  if constexpr (CHK) {
    float asum = 0.0f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < NF; ++n) asum += (acc[m][n][0] + acc[m][n][1]) + (acc[m][n][2] + acc[m][n][3]);
    if ((!(gmax < kDxInGuard) || !(asum - asum == 0.0f)) && g.flag) atomicOr(g.flag, 1u);
  }

  // ---- epilogue: lane holds outputs 16n + 4q .. +3 of pixel (row r0 + m, column j)
  const WAct act(g.act, g.slope);
  const float* btab = (const float*)(lds + L::BOFF);
  float* obase = g.out + (int64_t)b * g.H * g.Wd * g.ldo;
  bool out_ok = true;
  const int x = x0 + j;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int y = y0 + r0 + m;
    if (y >= g.H || x >= g.Wd) continue;
    const int cls = bias_class(y, x, g.H, g.Wd);
    float* dst = obase + ((int64_t)y * g.Wd + x) * g.ldo;
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int n0 = 16 * n + 4 * q;
      if (n0 >= g.N) continue;
      const d4 bv = *(const d4*)(btab + cls * (NF * 16) + n0);
      d4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float t = acc[m][n][k] * g.yscale + bv[k];
        v[k] = act.tanh_ ? wact(t, g.act, g.slope) : act(t);
        out_ok = out_ok && fabsf(v[k]) < kDxOutGuard;
      }
      if (n0 + 4 <= g.N) {
        *(d4*)(dst + n0) = v;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (n0 + k < g.N) dst[n0 + k] = v[k];
      }
    }
  }
  if (!out_ok && g.flag) atomicOr(g.flag, 1u);
}

}  // namespace idf

using namespace idf;

extern "C" int idf_conv3x3_dx3_supported(int32_t H, int32_t W, int32_t N) {
  return H >= 1 && W >= 16 && W % 16 == 0 && N >= 1 && N <= 48;
}

extern "C" int idf_conv3x3_dx3(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                               const float* x, int64_t ld_x, const uint16_t* w, int32_t nft,
                               float yscale, const float* b3, const float* vtap, int32_t ldv,
                               const float* bfull, int32_t N, float* out, int64_t ld_out,
                               int32_t act, float slope, uint32_t* d_flag, int32_t check_input) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || (ld_x & 3) || !w || !x || !out || !b3) return IDF_ERR_ARG;
  if (!idf_conv3x3_dx3_supported(H, W, N)) return IDF_ERR_UNSUPPORTED;
  const int nf = (N + 15) / 16;
  if (nft != nf) return IDF_ERR_ARG;  // the weights hold exactly the kernel's fragments
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  if ((uintptr_t)out % 16 || ld_out % 4) return IDF_ERR_ARG;  // 16-B output stores
  // 32-bit buffer offsets: one image's features must span < 4 GiB
  if ((int64_t)H * W * ld_x * 4 >= (int64_t)kDxInvalid) return IDF_ERR_UNSUPPORTED;
  Dx3Args g = {};
  g.X = x; g.ldx = ld_x; g.C = C; g.Wt = w; g.nslab = (C + 15) / 16; g.nft = nft; g.N = N;
  g.B = B; g.H = H; g.Wd = W;
  g.tiles_y = (H + 15) / 16;
  g.tiles_x = W / 16;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out; g.yscale = yscale; g.flag = d_flag;
  const int64_t blocks = (int64_t)B * g.tiles_y * g.tiles_x;
  if (blocks >= (1 << 20)) return IDF_ERR_UNSUPPORTED;  // udiv_s operands
  hipStream_t s = (hipStream_t)stream;
#define IDF_DX3_LAUNCH(nf_, chk)                                                                   \
  hipLaunchKernelGGL((conv3_dx3_kernel<nf_, chk>), dim3((unsigned)blocks), dim3(kDxThreads), 0, s, g)
  switch (nf) {
    case 1: if (check_input) IDF_DX3_LAUNCH(1, true); else IDF_DX3_LAUNCH(1, false); break;
    case 2: if (check_input) IDF_DX3_LAUNCH(2, true); else IDF_DX3_LAUNCH(2, false); break;
    default: if (check_input) IDF_DX3_LAUNCH(3, true); else IDF_DX3_LAUNCH(3, false); break;
  }
#undef IDF_DX3_LAUNCH
  return idf_last_error();
}
