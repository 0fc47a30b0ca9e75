// conv3_dx3.hip -- the DenseLayer 3x3 convolution ("dx3"): direct form, fp32-class products
// as split-f16 pairs on the K=32 f16 MFMA of gfx950, over PRE-SPLIT features.
//
// out = act(bias + conv3x3(X, W)) with the 1x1 folded in (packing.fold_layer).  Each fp32
// operand is an f16 pair, x = xh + xl and w' = w * 2^k = wh + wl (k per layer, host float64),
// and x.w' ~= xh.wh + xl.wh + xh.wl: every f16 x f16 product is exact in f32, the dropped
// xl.wl is ~2^-22 of the product (the arithmetic of the split-f16 Winograd kernel, wx3,
// conv3_wino.hip, without the transform).  All three products run on v_mfma_f32_16x16x32_f16
// (A = weights: 16 outputs x 32 k, B = pixels: 32 k x 16 pixels):
//   [wh ; wh] . [xh | xl]           one K=32 MFMA per tap and 16 channels (hi.hi + hi.lo)
//   [wl_t ; wl_t'] . [xh_t | xh_t'] xh.wl of two taps per K=32 MFMA (4 pairs per 16 channels;
//                                   the ninth tap pairs with zeros), so 14 MFMAs cover 16
//                                   channels x 9 taps x 3 products (13.5 is the floor).
//
// The features arrive split: the DenseBlock keeps, beside its fp32 feature rows, a split copy
// XS = [slab][hi, lo][pixel][16 channels] of f16 (64 B per pixel and 16 channels, the bytes
// of the fp32 values).  The block input is split once (idf_dx3_split_cols) and every dx3 layer
// writes its outputs in both forms.  So a slab's halo goes HBM -> LDS by LDS-DMA with no
// registers, no conversion and no VALU: the k-loop is LDS reads and MFMAs.
//
// Block = 8 waves (two per SIMD) = WR/2 16x16 output tiles x NF*16 outputs; a wave owns WR
// output rows (WR 16-pixel B fragments) of one tile x all outputs.  Per 16-channel slab the
// block stages into one of two LDS stages, by LDS-DMA issued a slab ahead:
//   * each tile's 18x18 halo as two planes, xh [324 slots][16] and xl [324 slots][16] (32 B
//     per slot: every ds_read_b128 lane group of the fragment reads is bank-conflict-free);
//   * the slab's weights in A-fragment order, wh [9 taps][NF][16 out][16 ch] then wl.
// One barrier per slab.  A pixel fragment (16 pixels of one halo row, one tap column) is read
// once and feeds the 3 output rows x NF fragments that use it.
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
  const uint16_t* xs;  // split features [nslab_xs][2: hi, lo][P][16] f16 bits
  int64_t P;           // pixels of the batch (B * H * W)
  int32_t nslab_xs;    // slabs the split buffer holds
  int32_t C;           // input channels (slabs read: ceil(C / 16))
  const uint16_t* Wt;  // [nslab][2: hi, lo][9 taps][nft][16 out][16 ch] f16 bits of w * 2^k
  int32_t nslab, nft;
  int32_t N;
  int32_t B, H, Wd;
  int32_t tiles_y, tiles_x, ntiles;
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

// timing-only ablations (tools/dx3_build_ablate.sh builds; never set in the library build):
// 1 no halo DMA, 4 no weight DMA, 8 no slab barrier, 16 no MFMAs, 32 no pixel-fragment LDS
// reads, 64 no weight-fragment LDS reads, 128 no split-output stores
#ifndef IDF_DX3_ABLATE
#define IDF_DX3_ABLATE 0
#endif
// schedule knobs (timing A/Bs; the defaults are the library's): pixel-fragment prefetch
// distance, a scheduling barrier between steps, the step of the slab's first DMA piece and the
// steps between pieces
#ifndef IDF_DX3_DB
#define IDF_DX3_DB 3
#endif
#ifndef IDF_DX3_SB
#define IDF_DX3_SB 1
#endif
#ifndef IDF_DX3_DMA0
#define IDF_DX3_DMA0 0
#endif
#ifndef IDF_DX3_DMAS
#define IDF_DX3_DMAS 1
#endif
// waves 4-7 (the second wave of each SIMD) start their DMA pieces this many steps later
#ifndef IDF_DX3_STAG
#define IDF_DX3_STAG 0
#endif
// timing-only s_memtime stamps (IDF_DX3_STAMPS=1 builds): per slab, for every wave of the block
// whose index is IDF_DX3_STAMP_BLOCK -- before the slab's wait, after its barrier, after step 9,
// at its end; read back with idf_dx3_stamps
#ifndef IDF_DX3_STAMPS
#define IDF_DX3_STAMPS 0
#endif
#ifndef IDF_DX3_STAMP_BLOCK
#define IDF_DX3_STAMP_BLOCK 100
#endif
#if IDF_DX3_STAMPS
__device__ unsigned long long g_dx3_stamp[8][40][4];
// per wave: kernel entry, after the bias table, loop end, kernel end (s_memtime), and
// s_memrealtime (100 MHz) at entry and end -- the clock the loop ran at
__device__ unsigned long long g_dx3_phase[8][6];
#define DX3_PHASE(j, v)                                                                      \
  do {                                                                                      \
    if (blockIdx.x == IDF_DX3_STAMP_BLOCK && lane == 0) g_dx3_phase[wave][(j)] = (v);       \
  } while (0)
#define DX3_STAMP(slab, j)                                                                 \
  do {                                                                                    \
    if (blockIdx.x == IDF_DX3_STAMP_BLOCK && (slab) < 40 && lane == 0)                    \
      g_dx3_stamp[wave][(slab)][(j)] = __builtin_amdgcn_s_memtime();                      \
  } while (0)
#else
#define DX3_STAMP(slab, j) do { } while (0)
#define DX3_PHASE(j, v) do { } while (0)
#endif
// the waves that issue the DMA pieces: IDF_DX3_DMAW of them from wave IDF_DX3_DMAW0
#ifndef IDF_DX3_DMAW
#define IDF_DX3_DMAW IDF_DX3_WAVES
#endif
#ifndef IDF_DX3_DMAW0
#define IDF_DX3_DMAW0 0
#endif
// 1: cross-slab prefetch -- two barriers per slab: one at its start (the stage slab s - 1 used
// may be refilled: slab s + 1's DMA is issued), one at step IDF_DX3_X (slab s + 1's stage is
// complete: the slab's last steps read slab s + 1's first fragments)
#ifndef IDF_DX3_XPF
#define IDF_DX3_XPF 0
#endif
#ifndef IDF_DX3_X
#define IDF_DX3_X 20
#endif
// 1: one tile per block at every geometry (timing A/B of the two block shapes)
#ifndef IDF_DX3_FORCE1
#define IDF_DX3_FORCE1 0
#endif

// waves per block (timing A/B: 16 = four per SIMD at 2 rows per wave)
#ifndef IDF_DX3_WAVES
#define IDF_DX3_WAVES 8
#endif
constexpr int kDxWaves = IDF_DX3_WAVES;
constexpr int kDxThreads = 64 * kDxWaves;
constexpr int kDxCW = 18;                 // halo canvas width (slots) = tile width 16 + 2
constexpr int kDxSlots = kDxCW * kDxCW;   // 324
constexpr int kDxPlane = 11 * 1024;       // one plane (xh or xl): 324 x 32 B in whole 1-KiB pieces
constexpr int kDxPlanePieces = kDxPlane / 1024;
constexpr uint32_t kDxInvalid = 0xFFFFFFF0u;
// the split-f16 range guard on stored outputs: |y| < 8192, as wx3 (|x| < 32768 on block inputs
// is checked where the inputs are split, idf_dx3_split_cols)
constexpr float kDxInGuard = 32768.0f;
constexpr float kDxOutGuard = 8192.0f;

template <int NF, int WR>
struct Dx3Lds {
  static constexpr int T = WR * kDxWaves / 16;     // 16x16 tiles per block
  static constexpr int HR = WR + 2;                // halo rows a wave reads
  static constexpr int NS = 5 * HR - 1;            // steps per slab (see the schedule)
  static constexpr int WOFF = T * 2 * kDxPlane;    // weights within a stage
  static constexpr int WPART = 9 * NF * 512;       // one part (wh or wl) of a slab's weights
  static constexpr int WST = 2 * WPART;            // a multiple of 1 KiB: whole DMA pieces
  static constexpr int STAGE = WOFF + WST;
  static constexpr int ZOFF = 2 * STAGE;           // NF * 512 B of zeros (the odd tap's pair)
  static constexpr int BOFF = ZOFF + NF * 512;     // bias table [16 classes][NF * 16] f32
  static constexpr int BYTES = BOFF + 16 * NF * 16 * 4;
  static constexpr int HPIECES = T * 2 * kDxPlanePieces;   // halo DMA pieces per slab
  static constexpr int NPIECES = HPIECES + WST / 1024;     // + weight pieces
  static constexpr int PPW = (NPIECES + IDF_DX3_DMAW - 1) / IDF_DX3_DMAW;  // pieces per wave (max)
};

typedef __attribute__((address_space(3))) void* dx_lds_ptr_t;

// f(integral_constant<int, T>) for T = 0, 1, ... in order: a compile-time unrolled schedule
template <typename F, int... T>
__device__ __forceinline__ void dx_unroll(F&& f, std::integer_sequence<int, T...>) {
  (f(std::integral_constant<int, T>{}), ...);
}

template <int NF, int WR>
__global__ void __launch_bounds__(kDxThreads, 1) conv3_dx3_kernel(Dx3Args g) {
  using L = Dx3Lds<NF, WR>;
  constexpr int T = L::T, HR = L::HR, NS = L::NS;
  static_assert(L::WST % 1024 == 0, "weight stage must be whole 1-KiB DMA pieces");
  static_assert(L::BYTES <= 160 * 1024, "LDS");
  static_assert(HR >= 3, "the A-fragment reads of a phase take its last three steps");
  __shared__ __attribute__((aligned(16))) char lds[L::BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = xcd_contiguous(blockIdx.x, gridDim.x);
  // the wave's tile and first output row
  const int tw = wave / (kDxWaves / T);
  const int r0 = WR * (wave % (kDxWaves / T));
  const int tile = bid * T + tw;

  // ---- DMA plan: piece k = wave + 8 i of each slab.  Halo pieces k < HPIECES: tile k / 22,
  // plane (k / 11) % 2, slots 32 (k % 11) .. +31 (lane: slot + lane / 2, 8 channels (lane & 1));
  // weight pieces: 1 KiB of the slab's weights each.
  const int64_t plane_b = g.P * 32;                      // bytes of one plane of one slab
  const uint32_t xs_stride = (uint32_t)(2 * plane_b);    // bytes per slab
  const int64_t xs_bytes = (int64_t)g.nslab_xs * 2 * plane_b;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.xs, 0, (int)(xs_bytes < (int64_t)kDxInvalid ? xs_bytes : (int64_t)kDxInvalid), 0x00020000);
  const int64_t wbytes = (int64_t)g.nslab * L::WST;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.Wt, 0, (int)(wbytes < (int64_t)kDxInvalid ? wbytes : (int64_t)kDxInvalid), 0x00020000);
  uint32_t pbase[L::PPW];  // per piece: source byte offset of slab 0 (halo) / within a slab (weights)
#pragma unroll
  for (int i = 0; i < L::PPW; ++i) {
    const int dw = wave - IDF_DX3_DMAW0;  // this wave's rank among the DMA-issuing waves
    const int k = (dw >= 0 && dw < IDF_DX3_DMAW) ? dw + IDF_DX3_DMAW * i : (1 << 20);
    pbase[i] = kDxInvalid;
    if (k < L::HPIECES) {
      const int t = k / (2 * kDxPlanePieces), pl = (k / kDxPlanePieces) % 2, pi = k % kDxPlanePieces;
      const int slot = 32 * pi + (lane >> 1);
      const int tt = bid * T + t;
      if (slot < kDxSlots && tt < g.ntiles) {
        int q = tt;
        const int tx = q - udiv_s(q, g.tiles_x) * g.tiles_x;
        q = udiv_s(q, g.tiles_x);
        const int ty = q - udiv_s(q, g.tiles_y) * g.tiles_y;
        const int b = udiv_s(q, g.tiles_y);
        const int hy = udiv_s(slot, kDxCW), cx = slot - hy * kDxCW;
        const int y = 16 * ty + hy - 1, x = 16 * tx + cx - 1;
        if (y >= 0 && y < g.H && x >= 0 && x < g.Wd)
          pbase[i] = (uint32_t)(pl * plane_b + ((((int64_t)b * g.H + y) * g.Wd + x) * 32) + (lane & 1) * 16);
      }
    } else if (k < L::NPIECES) {
      pbase[i] = (uint32_t)((k - L::HPIECES) * 1024 + lane * 16);
    }
  }
  // issue piece i of slab s into stage st
  auto dma = [&](int s, int st, int i) {
    const int dw = wave - IDF_DX3_DMAW0;
    const int k = (dw >= 0 && dw < IDF_DX3_DMAW) ? dw + IDF_DX3_DMAW * i : (1 << 20);
    if (k >= L::NPIECES) return;
    // one call site for both kinds of piece (the LDS address formed from the __shared__ array
    // itself): the host pass of hipcc drops the kernel's launch stub otherwise
    const bool halo = k < L::HPIECES;
    if (halo ? (IDF_DX3_ABLATE & 1) : (IDF_DX3_ABLATE & 4)) return;
    int lo;
    uint32_t off;
    if (halo) {
      const int t = k / (2 * kDxPlanePieces), pl = (k / kDxPlanePieces) % 2, pi = k % kDxPlanePieces;
      lo = (t * 2 + pl) * kDxPlane + pi * 1024;
      off = pbase[i] == kDxInvalid ? kDxInvalid : pbase[i] + (uint32_t)s * xs_stride;
    } else {
      lo = L::WOFF + (k - L::HPIECES) * 1024;
      off = pbase[i] + (uint32_t)(s * L::WST);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(halo ? xr : wr, (dx_lds_ptr_t)(lds + st * L::STAGE + lo),
                                             16, off, 0, 0, 0);
  };

  // zeros for the odd tap's pair, and the epilogue's bias table (both outside the stages)
  // slab 0's DMA first: the bias table's dependent global loads below then overlap its latency
  if (g.nslab > 0) {
#pragma unroll
    for (int i = 0; i < L::PPW; ++i) dma(0, 0, i);
  }
  for (int e = tid; e < NF * 512 / 16; e += kDxThreads) *(d4*)(lds + L::ZOFF + 16 * e) = d4{0.f, 0.f, 0.f, 0.f};
  DX3_PHASE(0, __builtin_amdgcn_s_memtime());
  DX3_PHASE(4, __builtin_amdgcn_s_memrealtime());
  stage_bias((float*)(lds + L::BOFF), NF * 16, 0, g.N, g.b3, g.vtap, g.bfull, g.ldv, tid, kDxThreads);
  DX3_PHASE(1, __builtin_amdgcn_s_memtime());

  // ---- fragment read offsets (bytes from a stage base).  B (pixels): lane (q = lane >> 4,
  // j = lane & 15) reads pixel j of a halo row, 8 channels.  A (weights): output j, 8 channels.
  const int j = lane & 15, q = lane >> 4;
  const int slot0 = r0 * kDxCW + j;
  const int tb = tw * 2 * kDxPlane;  // the wave's tile planes
  // [xh | xl] at (halo row r0 + h, column j + dx): q 0,1 hi plane chunk q, q 2,3 lo plane chunk q-2
  const int oP = tb + (q >> 1) * kDxPlane + slot0 * 32 + (q & 1) * 16;
  // [xh(h, dx 0) | xh(h, dx 1)]
  const int oF = tb + slot0 * 32 + (q & 1) * 16 + (q >> 1) * 32;
  // [xh(h, dx 2) | xh(h + 1, dx 2)]
  const int oG = tb + slot0 * 32 + (q & 1) * 16 + 64 + (q >> 1) * kDxCW * 32;
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

  d4 acc[WR][NF];
#pragma unroll
  for (int m = 0; m < WR; ++m)
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

  // ---- the slab schedule: NS = 5 HR - 1 steps, each one pixel fragment and the MFMAs using it.
  //   steps [0, 3 HR)     (P, dx = t / HR, h = t % HR): [wh ; wh] . [xh | xl](h, dx)
  //   steps [3 HR, 4 HR)  (F, h = t - 3 HR):            [wl(dy,0) ; wl(dy,1)] . [xh(h,0) | xh(h,1)]
  //   steps [4 HR, NS)    (G, h = t - 4 HR):            [wl(0,2) ; wl(1,2)] and [0 ; wl(2,2)]
  //                                                      . [xh(h,2) | xh(h+1,2)]
  // Pixel fragments are read DB steps ahead (a ring of DB + 1), a phase's weight fragments in
  // the first three steps of the phase before it.  Two LDS stages: slab s reads stage s % 2; after the slab's
  // barrier (every wave's DMA of slab s landed, every wave done with slab s - 1) the waves DMA
  // slab s + 1 into the other stage, one piece per step.
  constexpr int DB = IDF_DX3_DB, RB = DB + 1;
  e8 Bq[RB];
  e8 AS[2][3][NF];  // weight sets: P0 / P2 in 0, P1 / F in 1
  e8 AZ[2][NF];     // G: [wl(0,2) ; wl(1,2)] and [0 ; wl(2,2)]
  auto read_B = [&](const char* st, int t) -> e8 {
    if (t < 3 * HR) return rdB(st + oP + ((t % HR) * kDxCW + t / HR) * 32);
    if (t < 4 * HR) return rdB(st + oF + (t - 3 * HR) * kDxCW * 32);
    return rdB(st + oG + (t - 4 * HR) * kDxCW * 32);
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
      if (m < 0 || m >= WR) continue;
#pragma unroll
      for (int n = 0; n < NF; ++n) mma(A[dy][n], Bv, acc[m][n]);
    }
  };

  const int nslab = g.nslab;
  if constexpr (IDF_DX3_XPF) {
    constexpr int X = (IDF_DX3_X < NS - DB && IDF_DX3_X + 1 >= 3 * HR) ? IDF_DX3_X : NS - DB - 3;
    static_assert(X + 1 >= 3 * HR && NS - DB > X && X >= L::PPW, "cross-slab prefetch schedule");
    if (nslab > 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (nslab > 1) {
#pragma unroll
        for (int i = 0; i < L::PPW; ++i) dma(1, 1, i);
      }
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) read_A(lds, 0, dy, AS[0][dy]);
#pragma unroll
      for (int k = 0; k < DB; ++k) Bq[k] = read_B(lds, k);
    }
    for (int s = 0; s < nslab; ++s) {
      const char* cur = lds + (s & 1) * L::STAGE;
      const char* nxt = lds + ((s + 1) & 1) * L::STAGE;
      const bool more = s + 1 < nslab;
      DX3_STAMP(s, 0);
      // every wave is done with slab s - 1: its stage may take slab s + 1
      if (s >= 1) __builtin_amdgcn_s_barrier();
      DX3_STAMP(s, 1);
      auto step = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if (IDF_DX3_SB) __builtin_amdgcn_sched_barrier(0);
        if constexpr (t == 9) DX3_STAMP(s, 2);
        if constexpr (t < L::PPW) {
          if (s >= 1 && more) dma(s + 1, (s + 1) & 1, t);
        }
        if constexpr (t == X) {  // slab s + 1's stage complete (every wave's DMA landed)
          if (more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
          }
        }
        if constexpr (t < 3) read_A(cur, 1, t, AS[1][t]);
        if constexpr (t >= HR && t < HR + 3) read_A(cur, 2, t - HR, AS[0][t - HR]);
        if constexpr (t >= 2 * HR && t < 2 * HR + 3) read_A(cur, 3, t - 2 * HR, AS[1][t - 2 * HR]);
        if constexpr (t == 2 * HR + 3 || t == 2 * HR + 4) {
#pragma unroll
          for (int n = 0; n < NF; ++n) {
            if (t == 2 * HR + 3) AZ[0][n] = rdA(cur + oAG + n * 512);
            else AZ[1][n] = rdA(zlane ? zO + n * 512 : cur + oAO + n * 512);
          }
        }
        // slab s + 1's first weights (AS[0] is free once phase 2 is done)
        if constexpr (t > X && t <= X + 3) {
          if (more) read_A(nxt, 0, t - X - 1, AS[0][t - X - 1]);
        }
        if constexpr (t + DB < NS) Bq[(t + DB) % RB] = read_B(cur, t + DB);
        else if (more) Bq[(t + DB) % RB] = read_B(nxt, t + DB - NS);
        const e8& Bv = Bq[t % RB];
        if constexpr (t < 3 * HR) {
          mma_rows(AS[(t / HR) & 1], Bv, t % HR);
        } else if constexpr (t < 4 * HR) {
          mma_rows(AS[1], Bv, t - 3 * HR);
        } else {
          constexpr int h = t - 4 * HR;
          if constexpr (h < WR) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(AZ[0][n], Bv, acc[h][n]);
          }
          if constexpr (h > 0) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(AZ[1][n], Bv, acc[h - 1][n]);
          }
        }
      };
      dx_unroll(step, std::make_integer_sequence<int, NS>{});
      DX3_STAMP(s, 3);
      // the ring ran NS steps: slab s + 1's fragment k is in Bq[(NS + k) % RB]
      e8 f[DB];
#pragma unroll
      for (int k = 0; k < DB; ++k) f[k] = Bq[(NS + k) % RB];
#pragma unroll
      for (int k = 0; k < DB; ++k) Bq[k] = f[k];
    }
  } else {
    const int nslab = g.nslab;
    for (int s = 0; s < nslab; ++s) {
      const char* cur = lds + (s & 1) * L::STAGE;
      // this wave's DMA of slab s landed; after the barrier every wave's has, and every wave is
      // done reading stage (s + 1) % 2 (slab s - 1)
      DX3_STAMP(s, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!(IDF_DX3_ABLATE & 8)) __builtin_amdgcn_s_barrier();
      DX3_STAMP(s, 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) read_A(cur, 0, dy, AS[0][dy]);
#pragma unroll
      for (int k = 0; k < DB; ++k) Bq[k] = read_B(cur, k);
      const bool more = s + 1 < nslab;
      auto step = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if (IDF_DX3_SB) __builtin_amdgcn_sched_barrier(0);  // keep the schedule: steps do not mix
        if constexpr (t == 9) DX3_STAMP(s, 2);
        // slab s + 1's DMA, one piece every IDF_DX3_DMAS steps from step IDF_DX3_DMA0
        constexpr int ds = IDF_DX3_DMAS > 0 ? IDF_DX3_DMAS : 1;
        auto dma_at = [&](auto dtc) {
          constexpr int dt = decltype(dtc)::value;
          if constexpr (IDF_DX3_DMAS == 0 && dt == 0) {  // the whole slab's pieces at once
            if (more) {
#pragma unroll
              for (int i = 0; i < L::PPW; ++i) dma(s + 1, (s + 1) & 1, i);
            }
          } else if constexpr (IDF_DX3_DMAS > 0 && dt >= 0 && dt % ds == 0 && dt / ds < L::PPW) {
            if (more) dma(s + 1, (s + 1) & 1, dt / ds);
          }
        };
        if (IDF_DX3_STAG == 0 || !(wave & 4)) dma_at(std::integral_constant<int, t - IDF_DX3_DMA0>{});
        else dma_at(std::integral_constant<int, t - IDF_DX3_DMA0 - IDF_DX3_STAG>{});
        // weights of the next phase, one kernel row per step, in the first three steps of the
        // phase before it (its register set was freed by the phase before that)
        if constexpr (t < 3) read_A(cur, 1, t, AS[1][t]);
        if constexpr (t >= HR && t < HR + 3) read_A(cur, 2, t - HR, AS[0][t - HR]);
        if constexpr (t >= 2 * HR && t < 2 * HR + 3) read_A(cur, 3, t - 2 * HR, AS[1][t - 2 * HR]);
        if constexpr (t == 2 * HR + 3 || t == 2 * HR + 4) {
#pragma unroll
          for (int n = 0; n < NF; ++n) {
            if (t == 2 * HR + 3) AZ[0][n] = rdA(cur + oAG + n * 512);
            else AZ[1][n] = rdA(zlane ? zO + n * 512 : cur + oAO + n * 512);
          }
        }
        // pixel fragment DB steps ahead (within the slab)
        if constexpr (t + DB < NS) Bq[(t + DB) % RB] = read_B(cur, t + DB);
        const e8& Bv = Bq[t % RB];
        if constexpr (t < 3 * HR) {
          mma_rows(AS[(t / HR) & 1], Bv, t % HR);
        } else if constexpr (t < 4 * HR) {
          mma_rows(AS[1], Bv, t - 3 * HR);
        } else {
          constexpr int h = t - 4 * HR;
          if constexpr (h < WR) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(AZ[0][n], Bv, acc[h][n]);
          }
          if constexpr (h > 0) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(AZ[1][n], Bv, acc[h - 1][n]);
          }
        }
      };
      dx_unroll(step, std::make_integer_sequence<int, NS>{});
      DX3_STAMP(s, 3);
    }
  }

  // ---- epilogue: lane holds outputs 16n + 4q .. +3 of pixel (row r0 + m, column j) of its
  // tile.  fp32 outputs to out; their split pairs to XS at channel C + 16n + 4q (zeros for the
  // padding outputs n >= N and on to the next 16-channel boundary past C + N, so the next
  // layer's last slab reads finite values; never past the split buffer).
  DX3_PHASE(2, __builtin_amdgcn_s_memtime());
  if (tile >= g.ntiles) return;
  int qt = tile;
  const int tx = qt - udiv_s(qt, g.tiles_x) * g.tiles_x;
  qt = udiv_s(qt, g.tiles_x);
  const int ty = qt - udiv_s(qt, g.tiles_y) * g.tiles_y;
  const int b = udiv_s(qt, g.tiles_y);
  const WAct act(g.act, g.slope);
  const float* btab = (const float*)(lds + L::BOFF);
  bool out_ok = true;
  const int x = 16 * tx + j;
  const int zr = (g.C + g.N + 15) / 16 * 16, zend = zr < 16 * g.nslab_xs ? zr : 16 * g.nslab_xs;
  char* xsb = (char*)g.xs;
#pragma unroll
  for (int m = 0; m < WR; ++m) {
    const int y = 16 * ty + r0 + m;
    if (y >= g.H || x >= g.Wd) continue;
    const int cls = bias_class(y, x, g.H, g.Wd);
    const int64_t pix = ((int64_t)b * g.H + y) * g.Wd + x;
    float* dst = g.out + pix * g.ldo;
#pragma unroll
    for (int n = 0; n <= NF; ++n) {
      const int n0 = 16 * n + 4 * q;
      d4 v = d4{0.f, 0.f, 0.f, 0.f};
      if (n < NF && n0 < g.N) {
        const d4 bv = *(const d4*)(btab + cls * (NF * 16) + n0);
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
          for (int k = g.N - n0; k < 4; ++k) v[k] = 0.0f;
        }
      }
      const int c = g.C + n0;  // split channel of v[0]; c % 4 == 0, so v stays in one slab
      if (!(IDF_DX3_ABLATE & 128) && c < zend) {
        const e4 h = __builtin_convertvector(v, e4);
        const e4 l = __builtin_convertvector(v - __builtin_convertvector(h, d4), e4);
        char* p = xsb + (int64_t)(c >> 4) * 2 * plane_b + pix * 32 + (c & 15) * 2;
        *(e4*)p = h;
        *(e4*)(p + plane_b) = l;
      }
    }
  }
  if (!out_ok && g.flag) atomicOr(g.flag, 1u);
  DX3_PHASE(3, __builtin_amdgcn_s_memtime());
  DX3_PHASE(5, __builtin_amdgcn_s_memrealtime());
}

// Block-input split: XS channels [c0, c1) of every pixel from the fp32 rows x (ld_x floats),
// zeros for [c1, round16(c1)) (the first layer's own output slab: other blocks of that
// layer's launch read it -- as halo -- while its own blocks write it, so the value a reader
// sees depends on timing; it is only ever multiplied by exactly-zero weights (packing
// dx3_weights asserts the weights of channels >= C are +0) and every value written there is
// finite (these zeros, and outputs under the |y| < 8192 guard), so the product is +-0 either
// way and the sum's bits do not depend on which value was read);
// ORs bit 0 of flag for a value that is NaN or |x| >= 32768 (the f16 pairs' range).  One
// thread per (pixel, 4 channels).
__global__ void __launch_bounds__(256) dx3_split_cols_kernel(int64_t P, int32_t c0, int32_t c1,
                                                             const float* __restrict__ x,
                                                             int64_t ld_x, uint16_t* __restrict__ xs,
                                                             uint32_t* __restrict__ flag) {
  const int nq = ((c1 + 15) / 16 * 16 - c0) / 4;  // channel quads per pixel
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= P * nq) return;
  const int64_t pix = g / nq;
  const int c = c0 + 4 * (int)(g - pix * nq);
  d4 v = d4{0.f, 0.f, 0.f, 0.f};
  if (c < c1) v = *(const d4*)(x + pix * ld_x + c);  // c1 % 4 == 0: a quad is all in or all out
  const e4 h = __builtin_convertvector(v, e4);
  const e4 l = __builtin_convertvector(v - __builtin_convertvector(h, d4), e4);
  char* p = (char*)xs + ((int64_t)(c >> 4) * 2 * P + pix) * 32 + (c & 15) * 2;
  *(e4*)p = h;
  *(e4*)(p + P * 32) = l;
  // each value compared on its own: fmaxf would drop a NaN
  const bool ok = fabsf(v[0]) < kDxInGuard && fabsf(v[1]) < kDxInGuard &&
                  fabsf(v[2]) < kDxInGuard && fabsf(v[3]) < kDxInGuard;
  if (!ok && flag) atomicOr(flag, 1u);
}

}  // namespace idf

using namespace idf;

#if IDF_DX3_STAMPS
extern "C" int idf_dx3_stamps(unsigned long long* host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dx3_stamp), sizeof(g_dx3_stamp)) != hipSuccess) return 2;
  return hipMemcpyFromSymbol(host + 8 * 40 * 4, HIP_SYMBOL(g_dx3_phase), sizeof(g_dx3_phase)) == hipSuccess ? 0 : 2;
}
#endif

extern "C" int idf_conv3x3_dx3_supported(int32_t H, int32_t W, int32_t N) {
  return H >= 1 && W >= 16 && W % 16 == 0 && N >= 1 && N <= 48;
}

extern "C" int64_t idf_dx3_split_bytes(int64_t P, int32_t channels) {
  if (P < 0 || channels < 0) return -1;
  return (int64_t)((channels + 15) / 16) * 2 * P * 32;
}

extern "C" int idf_dx3_split_cols(void* stream, int64_t P, int32_t c0, int32_t c1, const float* x,
                                  int64_t ld_x, uint16_t* xs, int32_t nslab_xs, uint32_t* d_flag) {
  if (P <= 0 || c1 <= c0) return (P < 0 || c1 < c0) ? IDF_ERR_ARG : IDF_OK;
  if (!x || !xs || (c0 & 15) || (c1 & 3) || (ld_x & 3) || (uintptr_t)x % 16) return IDF_ERR_ARG;
  if ((c1 + 15) / 16 > nslab_xs) return IDF_ERR_ARG;
  const int64_t n = P * (((c1 + 15) / 16 * 16 - c0) / 4);
  hipLaunchKernelGGL(dx3_split_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P, c0, c1, x, ld_x, xs, d_flag);
  return idf_last_error();
}

extern "C" int idf_conv3x3_dx3(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                               uint16_t* xs, int32_t nslab_xs, const uint16_t* w, int32_t nft,
                               float yscale, const float* b3, const float* vtap, int32_t ldv,
                               const float* bfull, int32_t N, float* out, int64_t ld_out,
                               int32_t act, float slope, uint32_t* d_flag) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || !w || !xs || !out || !b3) return IDF_ERR_ARG;
  if (!idf_conv3x3_dx3_supported(H, W, N)) return IDF_ERR_UNSUPPORTED;
  const int nf = (N + 15) / 16;
  if (nft != nf) return IDF_ERR_ARG;  // the weights hold exactly the kernel's fragments
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  if ((uintptr_t)out % 16 || ld_out % 4) return IDF_ERR_ARG;  // 16-B output stores
  if ((C + 15) / 16 > nslab_xs) return IDF_ERR_ARG;          // the input slabs must exist
  const int64_t P = (int64_t)B * H * W;
  // 32-bit buffer offsets: the split buffer must span < 4 GiB
  if (idf_dx3_split_bytes(P, 16 * nslab_xs) >= (int64_t)kDxInvalid) return IDF_ERR_UNSUPPORTED;
  Dx3Args g = {};
  g.xs = xs; g.P = P; g.nslab_xs = nslab_xs; g.C = C;
  g.Wt = w; g.nslab = (C + 15) / 16; g.nft = nft; g.N = N;
  g.B = B; g.H = H; g.Wd = W;
  g.tiles_y = (H + 15) / 16;
  g.tiles_x = W / 16;
  const int64_t ntiles = (int64_t)B * g.tiles_y * g.tiles_x;
  if (ntiles >= (1 << 20)) return IDF_ERR_UNSUPPORTED;  // udiv_s operands
  g.ntiles = (int32_t)ntiles;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out; g.yscale = yscale; g.flag = d_flag;
  hipStream_t s = (hipStream_t)stream;
  // two tiles per block (4 rows per wave) while that still gives every CU a block; else one
  // tile per block (2 rows per wave)
  const bool two = ntiles >= 2 * 256 && !IDF_DX3_FORCE1;
#define IDF_DX3_LAUNCH(nf_, wr_)                                                                   \
  hipLaunchKernelGGL((conv3_dx3_kernel<nf_, wr_>),                                               \
                     dim3((unsigned)((ntiles + Dx3Lds<nf_, wr_>::T - 1) / Dx3Lds<nf_, wr_>::T)), \
                     dim3(kDxThreads), 0, s, g)
  switch (nf) {
    case 1: if (two) IDF_DX3_LAUNCH(1, 32 / kDxWaves); else IDF_DX3_LAUNCH(1, 16 / kDxWaves); break;
    case 2: if (two) IDF_DX3_LAUNCH(2, 32 / kDxWaves); else IDF_DX3_LAUNCH(2, 16 / kDxWaves); break;
    default: if (two) IDF_DX3_LAUNCH(3, 32 / kDxWaves); else IDF_DX3_LAUNCH(3, 16 / kDxWaves); break;
  }
#undef IDF_DX3_LAUNCH
  return idf_last_error();
}
