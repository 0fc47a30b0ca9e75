// conv3_wq.hip -- "wq": the DenseLayer 3x3 convolution (nnlayer.py:48-51 with the 1x1 folded
// in, nnblock.py:53-56) as Winograd F(2x2, 3x3) with fp32-accurate split-f16 products, each
// wave owning EVERY transform position of its tiles.
//
// Same arithmetic contract as conv3_wino.hip's X3 path ("wx3"): per 2x2 output tile
//   Y = A^T [ sum_c U_c (.) V_c ] A,  V_c = B^T d_c B,  U' = U 2^k (host, float64, rounded once),
// every f32 operand an f16 pair (V = Vh + Vl, U' = Uh + Ul), V.U' ~= Vl.Uh + Vh.Ul + Vh.Uh on
// v_mfma_f32_16x16x16_f16 with f32 accumulation, Y scaled by yscale = 2^-k.  The U layout is
// wx3's (idfcodec/packing.py wino_weights_x3).  What differs is the shape of the work:
//
//  * Block = 4 waves (one per SIMD), 64 Winograd tiles (256 output pixels) x 48 outputs; wave w
//    owns tile fragment w (16 tiles) at all 16 positions.  Its accumulators (16 positions x 3
//    n-fragments x 4 = 192 registers) use the lone wave's 512-register budget.
//  * The input transform is the minimal separable one (16 patch reads, 4 x 4 row combinations,
//    then 4 column combinations per row: 2 adds per V value), with no work repeated across
//    waves.
//  * The output transform never leaves the registers: an MFMA lane holds the same (tile,
//    output) at every position, so A^T M A is per-lane arithmetic -- no LDS staging, no
//    barriers in the epilogue (wx3 spends ~11k cycles per block there, ~14-27% of a launch).
//  * U goes through LDS once per block and slab (48 KiB, double-buffered): each wave reads the
//    fragments of the row it is about to multiply, one row ahead of its MFMAs.
//  * Per 16-channel slab s, four phases (rows a = 0..3 of B^T): phase k issues row k-1's 36
//    MFMAs beside row k's transform + f16 split and row k's U reads; phase 0 (after the slab
//    barrier) issues the previous slab's row-3 MFMAs beside the new slab's patch reads, so the
//    barrier and the LDS read latency sit under queued MFMAs.  Slab s+1's U comes by LDS-DMA
//    (phase 1); its halo (register-staged, coalesced 64-B-per-pixel loads issued four phases
//    earlier: one wave per SIMD hides no load latency) is written in phase 3, and slab s+2's
//    halo loads follow.  One barrier per slab.
//
// Scope: split-f16 mode, one K split, 3 n-fragments, tile widths 32 and 16 (imagenet64's
// 32x32 and 16x16 levels, 60% of the codec's GPU time); everything else stays on wx3.
// Determinism: every output is a fixed-order f32 sum that depends on the geometry and channel
// count only (never the batch size or block placement), so an encoder and a decoder running
// this kernel agree bit for bit.  Its bits differ from wx3's (another output-transform order):
// the engine runs the same kernel on both sides.  Parity: tests/test_gpu_wq.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "idf_codec_internal.h"
#include "wino_common.h"

#pragma clang fp contract(off)

// timing-only ablations (tools/wq_ablate.sh builds; never set in the library build): bit 0 no U
// pieces, bit 1 no halo loads/writes, bit 2 no slab barrier, bit 3 no U stage reads, bit 4 no
// transform / split VALU (hi/lo taken from the patch bits), bit 5 halo loads waited for but not
// written to LDS, bit 6 halo writes of registers never loaded (zeros)
#ifndef IDF_WQ_ABLATE
#define IDF_WQ_ABLATE 0
#endif
// halo staging: 1 = LDS-DMA pieces (64 slots of one channel quad each), 0 = coalesced
// register-staged loads + ds_write (four phases ahead)
#ifndef IDF_WQ_HALO_DMA
#define IDF_WQ_HALO_DMA 0
#endif
// L2 prefetch of the halo three slabs ahead (register-staged halo only): one 4-B LDS-DMA per
// halo pixel into a scratch LDS row, so that the real loads, issued a slab later, hit L2
#ifndef IDF_WQ_PREFETCH
#define IDF_WQ_PREFETCH 0
#endif

namespace idf {
namespace wq {

typedef float w4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kThreads = 256;
constexpr int kSlots = 448;                       // halo slots per channel quad (>= kWMaxHalo)
constexpr int kStage = 4 * kSlots * 4;            // floats: [4 quads][kSlots][4]
constexpr int kNF = 3;                            // n-fragments per block (48 outputs)
constexpr int kUStage = 16 * kNF * 256;           // floats: [16 pos][3 nf][64 lanes][4]
constexpr int kHaloLoads = (kWMaxHalo + 63) / 64;  // per wave and slab: 16 slots x 4 quads each
constexpr int kULoads = 16 * kNF / 4;             // U fragments per wave and slab
constexpr uint32_t kInvalid = 0xFFFFFFF0u;        // buffer offset that always reads 0
constexpr float kGuardIn = 32768.0f;
constexpr float kGuardOut = 8192.0f;
template <int n> using C = std::integral_constant<int, n>;

struct Args {
  const float* X;
  int64_t ldx;
  int32_t C;
  const float* U;  // x3 layout: [16 pos][nslab][nft][64 lanes][hi 4, lo 4 f16]
  int32_t nslab, nft, N;
  int32_t B, H, Wd;
  int32_t IMGS, TH, TW;
  int32_t tiles_y, tiles_x, n_tiles;
  const float* b3;
  const float* vtap;
  const float* bfull;
  int32_t ldv;
  int32_t act;
  float slope;
  float* out;
  int64_t ldo;
  float yscale;
  uint32_t* flag;
};

// s0 * x0 + s1 * x1 per channel, scalar adds (packed f32 adds cost extra issue beside MFMAs)
template <bool NEG0, bool NEG1>
__device__ __forceinline__ w4 comb(const w4& x0, const w4& x1) {
  w4 r;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (!NEG0 && !NEG1) r[k] = x0[k] + x1[k];
    else if (!NEG0 && NEG1) r[k] = x0[k] - x1[k];
    else if (NEG0 && !NEG1) r[k] = x1[k] - x0[k];
    else r[k] = -(x0[k] + x1[k]);
  }
  return r;
}

// f16 pair split: h = f16(v), l = f16(v - h) (both nearest-even; v - h is exact in f32)
__device__ __forceinline__ void split(const w4& v, h4& h, h4& l) {
  h = __builtin_convertvector(v, h4);
  l = __builtin_convertvector(v - __builtin_convertvector(h, w4), h4);
}

template <int TWC, bool CHK>
__global__ void __launch_bounds__(kThreads) conv3_wq_kernel(Args g) {
  constexpr int HWc = halo_pitch(TWC), EHc = HWc / 2;
  __shared__ __attribute__((aligned(16))) float lds[2 * kStage + 2 * kUStage + 16 * 16 * kNF + 4 * 64];
  float* const ust = lds + 2 * kStage;
  float* const btab = ust + 2 * kUStage;  // [16 border classes][48]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x;
  const int nt = bid - udiv_s(bid, g.n_tiles) * g.n_tiles;
  bid = udiv_s(bid, g.n_tiles);
  const int tx_ = bid - udiv_s(bid, g.tiles_x) * g.tiles_x;
  bid = udiv_s(bid, g.tiles_x);
  const int tb = udiv_s(bid, g.tiles_y);
  const int ty_ = bid - tb * g.tiles_y;
  const int b0 = tb * g.IMGS, y0 = ty_ * g.TH, x0 = tx_ * g.TW;
  const int HH = g.TH + 2;
  const int NH = g.IMGS * HH * HWc;
  const int TTW = g.TW >> 1, TPI = (g.TH >> 1) * TTW;
  const int nf0 = nt * kNF;
  const int nslab = g.nslab;

  // ---- staging sources: halo (16 slots x 4 channel quads per load) and U fragments
  const float* xbase = g.X + (int64_t)b0 * g.H * g.Wd * g.ldx;
  const int64_t xbytes = ((int64_t)g.B * g.H * g.Wd * g.ldx - (int64_t)b0 * g.H * g.Wd * g.ldx) * 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xbase, 0, (int)(xbytes < (int64_t)kInvalid ? xbytes : (int64_t)kInvalid), 0x00020000);
  const int64_t ubytes = (int64_t)16 * nslab * g.nft * 1024;
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.U, 0, (int)(ubytes < (int64_t)kInvalid ? ubytes : (int64_t)kInvalid), 0x00020000);
  const int hq4 = 4 * ((lane >> 3) & 3);
  uint32_t hsrc[kHaloLoads];
  int hdst[kHaloLoads];
  {
    const int sl = (lane & 7) + 8 * (lane >> 5), hq = (lane >> 3) & 3;
#pragma unroll
    for (int m = 0; m < kHaloLoads; ++m) {
      const int slot = 16 * (wave + 4 * m) + sl;
      hsrc[m] = kInvalid;
      hdst[m] = (hq * kSlots + (slot < kSlots ? slot : kSlots - 1)) * 4;
      if (slot < NH) {
        const int img = udiv_s(slot, HH * HWc);
        const int rem = slot - img * HH * HWc;
        const int hy = udiv_s(rem, HWc), cs = rem - hy * HWc;
        const int hx = cs < EHc ? 2 * cs : 2 * (cs - EHc) + 1;
        const int y = y0 + hy - 1, x = x0 + hx - 1;
        if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd && hx < g.TW + 2)
          hsrc[m] = (uint32_t)(((((int64_t)img * g.H + y) * g.Wd + x) * g.ldx + hq4) * 4);
      }
    }
  }
  w4 hb[IDF_WQ_HALO_DMA ? 1 : kHaloLoads];
  if (IDF_WQ_ABLATE & 64) {
#pragma unroll
    for (int m = 0; m < (IDF_WQ_HALO_DMA ? 1 : kHaloLoads); ++m) hb[m] = w4{0.f, 0.f, 0.f, 0.f};
  }
  // DMA form: this wave's piece m is f = wave + 4m of the stage's 28: channel quad f / 7, halo
  // slots [64 (f % 7), +64); xsrc = byte offset of the lane's slot pixel at channel 4q of slab 0
  uint32_t xsrc[kHaloLoads];
  if constexpr (IDF_WQ_HALO_DMA) {
    static_assert(kSlots == 7 * 64 && kHaloLoads == 7, "halo DMA pieces");
#pragma unroll
    for (int m = 0; m < kHaloLoads; ++m) {
      const int f = wave + 4 * m, q = f / 7, slot = 64 * (f - 7 * q) + lane;
      xsrc[m] = kInvalid;
      if (slot < NH) {
        const int img = udiv_s(slot, HH * HWc);
        const int rem = slot - img * HH * HWc;
        const int hy = udiv_s(rem, HWc), cs = rem - hy * HWc;
        const int hx = cs < EHc ? 2 * cs : 2 * (cs - EHc) + 1;
        const int y = y0 + hy - 1, x = x0 + hx - 1;
        if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd && hx < g.TW + 2)
          xsrc[m] = (uint32_t)(((((int64_t)img * g.H + y) * g.Wd + x) * g.ldx + 4 * q) * 4);
      }
    }
  }
  // prefetch: this wave's slot blocks wave and wave + 4 (of 7), channel quad 0 of each slot
  constexpr bool PF = IDF_WQ_PREFETCH && !IDF_WQ_HALO_DMA;
  uint32_t pfsrc[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int slot = 64 * (wave + 4 * m) + lane;
    pfsrc[m] = kInvalid;
    if (PF && wave + 4 * m < 7 && slot < NH) {
      const int img = udiv_s(slot, HH * HWc);
      const int rem = slot - img * HH * HWc;
      const int hy = udiv_s(rem, HWc), cs = rem - hy * HWc;
      const int hx = cs < EHc ? 2 * cs : 2 * (cs - EHc) + 1;
      const int y = y0 + hy - 1, x = x0 + hx - 1;
      if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd && hx < g.TW + 2)
        pfsrc[m] = (uint32_t)((((int64_t)img * g.H + y) * g.Wd + x) * g.ldx * 4);
    }
  }
  float* const pf_sink = lds + 2 * kStage + 2 * kUStage + 16 * 16 * kNF + 64 * wave;
  auto prefetch = [&](int slab) {
    if constexpr (PF) {
      const int c0 = slab * 16;
      // every wave issues both pieces (wave 3's second reads nothing): the barrier's vmcnt
      // counts exactly 7 halo loads + 2 prefetches younger than the U pieces
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const uint32_t off = pfsrc[m] != kInvalid && c0 < g.C ? pfsrc[m] + (uint32_t)c0 * 4u : kInvalid;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)pf_sink, 4, off, 0, 0, 0);
      }
    }
  };
  auto issue_halo1 = [&](int slab, int buf, int m) {
    if (IDF_WQ_ABLATE & 2) return;
    const int f = wave + 4 * m, q = f / 7, k = f - 7 * q;
    const int c0 = slab * 16;
    const uint32_t off =
        (xsrc[m] != kInvalid && c0 + 4 * q < g.C) ? xsrc[m] + (uint32_t)c0 * 4u : kInvalid;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(lds + buf * kStage + (q * kSlots + 64 * k) * 4),
                                             16, off, 0, 0, 0);
  };
  // slab `slab`'s halo into the staging registers (4 lanes x 16 B = one pixel's 64 B)
  auto load_halo = [&](int slab) {
    if (IDF_WQ_ABLATE & (2 | 64) || IDF_WQ_HALO_DMA) return;
    const int c0 = slab * 16;
    const bool chan_ok = c0 + hq4 < g.C;
#pragma unroll
    for (int m = 0; m < kHaloLoads; ++m) {
      const uint32_t off = (hsrc[m] != kInvalid && chan_ok) ? hsrc[m] + (uint32_t)c0 * 4u : kInvalid;
      hb[m] = __builtin_bit_cast(w4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto store_halo = [&](int buf) {
    if (IDF_WQ_ABLATE & 2 || IDF_WQ_HALO_DMA) return;
    if (IDF_WQ_ABLATE & 32) {  // the loads and their wait, no LDS writes
#pragma unroll
      for (int m = 0; m < kHaloLoads; ++m) asm volatile("" ::"v"(hb[m]));
      return;
    }
#pragma unroll
    for (int m = 0; m < kHaloLoads; ++m) *(w4*)(lds + buf * kStage + hdst[m]) = hb[m];
  };
  // slab `slab`'s U fragments -> U stage `buf` by LDS-DMA: each piece is one contiguous 1-KiB
  // fragment (the wave's 12 of the block's 48), no staging registers
  auto issue_u1 = [&](int slab, int buf, int k) {
    if (IDF_WQ_ABLATE & 1) return;
    const uint32_t ubase = (uint32_t)slab * (uint32_t)g.nft * 1024u + (uint32_t)lane * 16u;
    const int c = wave * kULoads + k, pos = c / kNF, j = c - pos * kNF;
    const uint32_t off = ubase + (uint32_t)((pos * nslab * g.nft + nf0 + j) * 1024);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_ptr_t)(ust + buf * kUStage + c * 256), 16,
                                             off, 0, 0, 0);
  };
  auto issue_u = [&](int slab, int buf) {
#pragma unroll
    for (int k = 0; k < kULoads; ++k) issue_u1(slab, buf, k);
  };
  // the slab barrier: the U pieces (issued before the 7 halo loads of the slab after next)
  // have landed, every wave's LDS traffic of the slab is done
  static_assert(kHaloLoads == 7, "barrier vmcnt");
  auto barrier = [] {
    if (IDF_WQ_HALO_DMA) {
      if (IDF_WQ_ABLATE & 4) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else if (IDF_WQ_PREFETCH) {  // the halo loads and (younger) prefetches may be in flight
      if (IDF_WQ_ABLATE & 4) asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      if (IDF_WQ_ABLATE & 4) asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };

  // ---- this lane's patch base: tile 16 * wave + (lane & 15), channel quad lane >> 4
  int pbase;
  {
    const int t = 16 * wave + (lane & 15);
    int img = udiv_s(t, TPI);
    const int rem = t - img * TPI;
    const int ty = udiv_s(rem, TTW), tx = rem - ty * TTW;
    if (img >= g.IMGS) img = 0;  // idle rows read valid LDS
    pbase = ((lane >> 4) * kSlots + (img * HH + 2 * ty) * HWc + tx) * 4;
  }
  auto cs = [](int j) { return (j & 1) ? EHc + (j >> 1) : (j >> 1); };

  w4 acc[16][kNF];
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int j = 0; j < kNF; ++j) acc[p][j] = w4{0.f, 0.f, 0.f, 0.f};
  float gmax = 0.0f;

  w4 d[4][4];  // the current slab's 4x4 patch (this lane's tile and channel quad)
  auto fetch = [&](int buf) {
    const float* P = lds + buf * kStage + pbase;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) d[i][j] = *(const w4*)(P + (i * HWc + cs(j)) * 4);
  };
  // row a's four V = (B^T d B)[a][b] as f16 pairs (hl[b][0] = hi, hl[b][1] = lo): the row
  // combinations R[j] = B^T[a] . d[.][j], then the column combinations of R
  auto vsplit = [&](auto ac, h4 (&hl)[4][2]) {
    constexpr int a = decltype(ac)::value;
    using RA = BT<a>;
    if (IDF_WQ_ABLATE & 16) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        hl[b][0] = __builtin_bit_cast(h4, __builtin_shufflevector(d[a][b], d[a][b], 0, 1));
        hl[b][1] = __builtin_bit_cast(h4, __builtin_shufflevector(d[a][b], d[a][b], 2, 3));
      }
      return;
    }
    w4 R[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) R[j] = comb<RA::neg0, RA::neg1>(d[RA::i0][j], d[RA::i1][j]);
    w4 v[4];
    v[0] = comb<BT<0>::neg0, BT<0>::neg1>(R[BT<0>::i0], R[BT<0>::i1]);
    v[1] = comb<BT<1>::neg0, BT<1>::neg1>(R[BT<1>::i0], R[BT<1>::i1]);
    v[2] = comb<BT<2>::neg0, BT<2>::neg1>(R[BT<2>::i0], R[BT<2>::i1]);
    v[3] = comb<BT<3>::neg0, BT<3>::neg1>(R[BT<3>::i0], R[BT<3>::i1]);
#pragma unroll
    for (int b = 0; b < 4; ++b) split(v[b], hl[b][0], hl[b][1]);
    if constexpr (CHK) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        gmax = fmaxf(fmaxf(gmax, fmaxf(fabsf(v[b][0]), fabsf(v[b][1]))),
                     fmaxf(fabsf(v[b][2]), fabsf(v[b][3])));
    }
  };
  // Row a's 36 MFMAs, position-major: per position b the products Vl.Uh, Vh.Ul, Vh.Uh of each
  // n-fragment (an accumulator every third MFMA); after u[b][j]'s last use (MFMA 9b+6+j) it is
  // reloaded with row a_next's fragment from stage nbuf, so one row's U plus one position is live.
  auto row = [&](auto ac, auto anc, const h4 (&hl)[4][2], w4 (&u)[4][kNF], int nbuf, int b0,
                 int b1, auto&& hook) {
    constexpr int a = decltype(ac)::value, an = decltype(anc)::value;
#pragma unroll
    for (int b = b0; b < b1; ++b) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < kNF; ++j) {
          const h8 uu = __builtin_bit_cast(h8, u[b][j]);
          const h4 uh = __builtin_shufflevector(uu, uu, 0, 1, 2, 3);
          const h4 ul = __builtin_shufflevector(uu, uu, 4, 5, 6, 7);
          const h4 av = p == 0 ? hl[b][1] : hl[b][0];
          const h4 bv = p == 1 ? ul : uh;
          acc[4 * a + b][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(av, bv, acc[4 * a + b][j], 0, 0, 0);
          hook(9 * b + 3 * p + j);
        }
#pragma unroll
      for (int j = 0; j < kNF; ++j)
        if (!(IDF_WQ_ABLATE & 8))
          u[b][j] = *(const w4*)(ust + nbuf * kUStage + ((4 * an + b) * kNF + j) * 256 + lane * 4);
    }
  };
  // The interleave of one phase (a scheduling region of nk MFMAs): the phase's nw halo writes
  // lead its first MFMAs (one each), MFMA k is followed by the U reload whose operand it
  // retires (k = 9b+6+j), its nm VMEM instructions one per MFMA from MFMA m0, and nv VALU.
  auto sched = [](auto c_nk, auto c_nv, auto c_nw, auto c_nm, auto c_m0) {
    constexpr int nk = decltype(c_nk)::value, nv = decltype(c_nv)::value;
    constexpr int nw = decltype(c_nw)::value, nm = decltype(c_nm)::value;
    constexpr int m0 = decltype(c_m0)::value;
#pragma unroll
    for (int k = 0; k < nk; ++k) {
      if (k < nw) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (k % 9 >= 6) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (k >= m0 && k < m0 + nm) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, nv, 0);
    }
  };
  auto nohook = [](int) {};
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // ---- prologue: slab 0 staged, slab 1's halo loading, slab 0's patch, row-0 operands
  const int S = nslab;
  load_halo(0);
  if constexpr (IDF_WQ_HALO_DMA) {
#pragma unroll
    for (int m = 0; m < kHaloLoads; ++m) issue_halo1(0, 0, m);
  }
  issue_u(0, 0);
  stage_bias(btab, 16 * kNF, nf0 * 16, g.N, g.b3, g.vtap, g.bfull, g.ldv, tid, kThreads);
  store_halo(0);
  __builtin_amdgcn_sched_barrier(0);
  load_halo(1 < S ? 1 : S - 1);
  barrier();
  h4 hA[4][2], hB[4][2];
  w4 u[4][kNF];  // the U fragments of the row being multiplied (reloaded position by position)
  fetch(0);
  vsplit(I0{}, hA);
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int j = 0; j < kNF; ++j) u[b][j] = *(const w4*)(ust + (b * kNF + j) * 256 + lane * 4);
  for (int s = 0; s < S; ++s) {
    const int buf = s & 1;
    // phase 1: row 0's MFMAs; row 1's operands; slab s+1's U pieces -> the other stage
    __builtin_amdgcn_sched_barrier(0);
    vsplit(I1{}, hB);
    {
      const int us = s + 1 < S ? s + 1 : S - 1;
      if constexpr (IDF_WQ_HALO_DMA) {
        // 19 pieces (7 halo, 12 U) spread over the 36 MFMAs
        row(I0{}, I1{}, hA, u, buf, 0, 4, [&](int k) {
          if ((k & 1) == 0 && k / 2 < kHaloLoads) issue_halo1(us, buf ^ 1, k / 2);
          else if ((k & 1) == 0 && k / 2 < kHaloLoads + kULoads) issue_u1(us, buf ^ 1, k / 2 - kHaloLoads);
          if (k == 35) issue_u1(us, buf ^ 1, kULoads - 1);
        });
      } else {
        row(I0{}, I1{}, hA, u, buf, 0, 4, [&](int k) {
          if (k >= 8 && k < 8 + 2 * kULoads && (k & 1) == 0) issue_u1(us, buf ^ 1, (k - 8) >> 1);
        });
      }
    }
    sched(C<36>{}, C<2>{}, C<0>{}, C<0>{}, C<0>{});
    // phase 2: row 1's MFMAs; row 2's operands
    __builtin_amdgcn_sched_barrier(0);
    vsplit(I2{}, hA);
    row(I1{}, I2{}, hB, u, buf, 0, 4, nohook);
    sched(C<36>{}, C<2>{}, C<0>{}, C<0>{}, C<0>{});
    __builtin_amdgcn_sched_barrier(0);
    // phase 3: row 2's MFMAs; row 3's operands; slab s+1's halo (loaded four phases ago) -> the
    // other stage, then slab s+2's halo loads
    vsplit(I3{}, hB);
    store_halo(buf ^ 1);
    row(I2{}, I3{}, hA, u, buf, 0, 4, nohook);
    load_halo(s + 2 < S ? s + 2 : S - 1);
    sched(C<36>{}, C<2>{}, C<kHaloLoads>{}, C<kHaloLoads>{}, C<20>{});
    __builtin_amdgcn_sched_barrier(0);
    prefetch(s + 3 < S ? s + 3 : S - 1);  // after the halo loads: the barrier lets both fly
    barrier();
    // phase 0: row 3's MFMAs beside slab s+1's patch reads and row-0 operands (past the last
    // slab: the last slab again, unused); its U reloads read slab s+1's stage
    // (0a: the 16 patch reads beside position 12's MFMAs; 0b: the rest with the transform)
    fetch(buf ^ 1);
    row(I3{}, I0{}, hB, u, buf ^ 1, 0, 1, nohook);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    vsplit(I0{}, hA);
    row(I3{}, I0{}, hB, u, buf ^ 1, 1, 4, nohook);
    sched(C<27>{}, C<3>{}, C<0>{}, C<0>{}, C<0>{});
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- range guard on the inputs (block inputs only): |V| and NaN (via the accumulators)
  if constexpr (CHK) {
    float asum = 0.0f;
#pragma unroll
    for (int p = 0; p < 16; ++p)
#pragma unroll
      for (int j = 0; j < kNF; ++j) asum += (acc[p][j][0] + acc[p][j][1]) + (acc[p][j][2] + acc[p][j][3]);
    if ((!(gmax < kGuardIn) || !(asum - asum == 0.0f)) && g.flag) atomicOr(g.flag, 1u);
  }

  // ---- epilogue: A^T M A per lane (tile 16 * wave + 4 * (lane >> 4) + r, output lane & 15).
  // Stores go through a buffer resource over the block's images: an out-of-image pixel or an
  // output column past N gets an out-of-range offset and the store is dropped (no branches).
  const int nn = lane & 15;
  const int64_t obytes = ((int64_t)g.B * g.H * g.Wd - (int64_t)b0 * g.H * g.Wd) * g.ldo * 4;
  const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.out + (int64_t)b0 * g.H * g.Wd * g.ldo), 0,
      (int)(obytes < (int64_t)kInvalid ? obytes : (int64_t)kInvalid), 0x00020000);
  uint32_t po[4][4];  // [tile r][pixel 2 rr + cc]: byte offset of the pixel's row, or kInvalid
  int pcls[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int t = 16 * wave + 4 * (lane >> 4) + r;
    const int img = udiv_s(t, TPI);
    const int rem = t - img * TPI;
    const int ty = udiv_s(rem, TTW), tx = rem - ty * TTW;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int y = y0 + 2 * ty + (e >> 1), x = x0 + 2 * tx + (e & 1);
      const bool ok = img < g.IMGS && b0 + img < g.B && y < g.H && x < g.Wd;
      po[r][e] = ok ? (uint32_t)((img * g.H + y) * g.Wd + x) * (uint32_t)(g.ldo * 4) : kInvalid;
      pcls[r][e] = bias_class(y, x, g.H, g.Wd) * (16 * kNF) + nn;
    }
  }
  bool out_ok = true;
  auto epilogue = [&](auto tanh_c) {
    constexpr bool TANH = decltype(tanh_c)::value;
    const WAct act(g.act, g.slope);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < kNF; ++j) {
        const int n = (nf0 + j) * 16 + nn;
        float u0[4], u1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          u0[b] = (acc[b][j][r] + acc[4 + b][j][r]) + acc[8 + b][j][r];
          u1[b] = (acc[4 + b][j][r] - acc[8 + b][j][r]) - acc[12 + b][j][r];
        }
        float Y[4];
        Y[0] = (u0[0] + u0[1]) + u0[2];
        Y[1] = (u0[1] - u0[2]) - u0[3];
        Y[2] = (u1[0] + u1[1]) + u1[2];
        Y[3] = (u1[1] - u1[2]) - u1[3];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = Y[e] * g.yscale + btab[pcls[r][e] + j * 16];
          v = TANH ? wact(v, g.act, g.slope) : act(v);
          const bool st = po[r][e] != kInvalid && n < g.N;
          out_ok = out_ok && (!st || fabsf(v) < kGuardOut);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), orr,
                                                st ? po[r][e] + (uint32_t)n * 4u : kInvalid, 0, 0);
        }
      }
  };
  if (g.act == IDF_ACT_TANH) epilogue(std::true_type{});
  else epilogue(std::false_type{});
  if (!out_ok && g.flag) atomicOr(g.flag, 1u);
}


// ------------------------------------------------------------------------------------------
// "wp": the same arithmetic at TWO waves per SIMD.  Block = 8 waves, 64 tiles x 48 outputs;
// wave w owns tile fragment w & 3 at the eight positions of B^T rows 2 rp, 2 rp + 1 (rp =
// w >> 2): 96 accumulators, so that the SIMD's other wave hides this one's load and LDS
// latency (wq's single wave cannot).  Per slab: phase A = row r0's MFMAs beside row r1's
// transform and U reads (into registers: the stage is rewritten after the barrier), the halo
// writes of slab s+1, its U pieces and slab s+2's halo loads; the barrier; phase B = row r1's
// MFMAs beside slab s+1's patch reads and row r0's transform.  Epilogue: the wave pair of a
// tile fragment exchanges its half-row sums of A^T M through LDS (one barrier) and each
// finishes two of its lanes' four tiles.
constexpr int kPThreads = 512;
constexpr int kPHalo = 4;               // halo loads per wave and slab (28 per stage, 8 waves)
constexpr int kPU = 16 * kNF / 8;       // U pieces per wave and slab

template <int TWC, bool CHK>
__global__ void __launch_bounds__(kPThreads) conv3_wp_kernel(Args g) {
  constexpr int HWc = halo_pitch(TWC), EHc = HWc / 2;
  __shared__ __attribute__((aligned(16))) float lds[2 * kStage + 2 * kUStage + 16 * 16 * kNF];
  float* const ust = lds + 2 * kStage;
  float* const btab = ust + 2 * kUStage;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tf = wave & 3, rp = wave >> 2;
  int bid = blockIdx.x;
  const int nt = bid - udiv_s(bid, g.n_tiles) * g.n_tiles;
  bid = udiv_s(bid, g.n_tiles);
  const int tx_ = bid - udiv_s(bid, g.tiles_x) * g.tiles_x;
  bid = udiv_s(bid, g.tiles_x);
  const int tb = udiv_s(bid, g.tiles_y);
  const int ty_ = bid - tb * g.tiles_y;
  const int b0 = tb * g.IMGS, y0 = ty_ * g.TH, x0 = tx_ * g.TW;
  const int HH = g.TH + 2;
  const int NH = g.IMGS * HH * HWc;
  const int TTW = g.TW >> 1, TPI = (g.TH >> 1) * TTW;
  const int nf0 = nt * kNF;
  const int S = g.nslab;

  const float* xbase = g.X + (int64_t)b0 * g.H * g.Wd * g.ldx;
  const int64_t xbytes = ((int64_t)g.B * g.H * g.Wd * g.ldx - (int64_t)b0 * g.H * g.Wd * g.ldx) * 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xbase, 0, (int)(xbytes < (int64_t)kInvalid ? xbytes : (int64_t)kInvalid), 0x00020000);
  const int64_t ubytes = (int64_t)16 * S * g.nft * 1024;
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.U, 0, (int)(ubytes < (int64_t)kInvalid ? ubytes : (int64_t)kInvalid), 0x00020000);
  // halo staging: load m of this wave covers slot block f = wave + 8 m (16 slots x 4 quads)
  const int hq4 = 4 * ((lane >> 3) & 3);
  uint32_t hsrc[kPHalo];
  int hdst[kPHalo];
  {
    const int sl = (lane & 7) + 8 * (lane >> 5), hq = (lane >> 3) & 3;
#pragma unroll
    for (int m = 0; m < kPHalo; ++m) {
      const int slot = 16 * (wave + 8 * m) + sl;
      hsrc[m] = kInvalid;
      hdst[m] = (hq * kSlots + (slot < kSlots ? slot : kSlots - 1)) * 4;
      if (slot < NH) {
        const int img = udiv_s(slot, HH * HWc);
        const int rem = slot - img * HH * HWc;
        const int hy = udiv_s(rem, HWc), cs = rem - hy * HWc;
        const int hx = cs < EHc ? 2 * cs : 2 * (cs - EHc) + 1;
        const int y = y0 + hy - 1, x = x0 + hx - 1;
        if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd && hx < g.TW + 2)
          hsrc[m] = (uint32_t)(((((int64_t)img * g.H + y) * g.Wd + x) * g.ldx + hq4) * 4);
      }
    }
  }
  w4 hb[kPHalo];
  auto load_halo = [&](int slab) {
    const int c0 = slab * 16;
    const bool chan_ok = c0 + hq4 < g.C;
#pragma unroll
    for (int m = 0; m < kPHalo; ++m) {
      const uint32_t off = (hsrc[m] != kInvalid && chan_ok) ? hsrc[m] + (uint32_t)c0 * 4u : kInvalid;
      hb[m] = __builtin_bit_cast(w4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto store_halo = [&](int buf) {
#pragma unroll
    for (int m = 0; m < kPHalo; ++m)
      if (wave + 8 * m < 28) *(w4*)(lds + buf * kStage + hdst[m]) = hb[m];  // wave-uniform
  };
  auto issue_u1 = [&](int slab, int buf, int k) {
    const uint32_t ubase = (uint32_t)slab * (uint32_t)g.nft * 1024u + (uint32_t)lane * 16u;
    const int c = wave * kPU + k, pos = c / kNF, j = c - pos * kNF;
    const uint32_t off = ubase + (uint32_t)((pos * S * g.nft + nf0 + j) * 1024);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (lds_ptr_t)(ust + buf * kUStage + c * 256), 16,
                                             off, 0, 0, 0);
  };
  // the slab barrier: every U piece landed (the 4 younger halo loads may fly)
  auto barrier = [] { asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  int pbase;
  {
    const int t = 16 * tf + (lane & 15);
    int img = udiv_s(t, TPI);
    const int rem = t - img * TPI;
    const int ty = udiv_s(rem, TTW), tx = rem - ty * TTW;
    if (img >= g.IMGS) img = 0;
    pbase = ((lane >> 4) * kSlots + (img * HH + 2 * ty) * HWc + tx) * 4;
  }
  auto cs = [](int j) { return (j & 1) ? EHc + (j >> 1) : (j >> 1); };

  w4 acc[8][kNF];
#pragma unroll
  for (int p = 0; p < 8; ++p)
#pragma unroll
    for (int j = 0; j < kNF; ++j) acc[p][j] = w4{0.f, 0.f, 0.f, 0.f};
  float gmax = 0.0f;

  auto run = [&](auto rpc) {
    constexpr int RP = decltype(rpc)::value;
    constexpr int R0 = 2 * RP, R1 = 2 * RP + 1;
    using T0 = BT<R0>;
    using T1 = BT<R1>;
    // patch rows: row r0 needs T0::i0, T0::i1; row r1 needs T1::i0, T1::i1 (one of them shared)
    constexpr int XR = (T1::i0 != T0::i0 && T1::i0 != T0::i1) ? T1::i0 : T1::i1;  // the extra row
    w4 da[4], db[4], dx[4];  // rows T0::i0, T0::i1, XR of the current slab
    auto fetch_row = [&](int buf, int i, w4 (&d)[4]) {
      const float* P = lds + buf * kStage + pbase;
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = *(const w4*)(P + (i * HWc + cs(j)) * 4);
    };
    auto rowsel = [&](int i) -> const w4* { return i == T0::i0 ? da : (i == T0::i1 ? db : dx); };
    // row a's four V as f16 pairs
    auto vsplit = [&](auto tc, h4 (&hl)[4][2]) {
      using TA = decltype(tc);
      const w4* p0 = rowsel(TA::i0);
      const w4* p1 = rowsel(TA::i1);
      w4 R[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) R[j] = comb<TA::neg0, TA::neg1>(p0[j], p1[j]);
      w4 v[4];
      v[0] = comb<BT<0>::neg0, BT<0>::neg1>(R[BT<0>::i0], R[BT<0>::i1]);
      v[1] = comb<BT<1>::neg0, BT<1>::neg1>(R[BT<1>::i0], R[BT<1>::i1]);
      v[2] = comb<BT<2>::neg0, BT<2>::neg1>(R[BT<2>::i0], R[BT<2>::i1]);
      v[3] = comb<BT<3>::neg0, BT<3>::neg1>(R[BT<3>::i0], R[BT<3>::i1]);
#pragma unroll
      for (int b = 0; b < 4; ++b) split(v[b], hl[b][0], hl[b][1]);
      if constexpr (CHK) {
#pragma unroll
        for (int b = 0; b < 4; ++b)
          gmax = fmaxf(fmaxf(gmax, fmaxf(fabsf(v[b][0]), fabsf(v[b][1]))),
                       fmaxf(fabsf(v[b][2]), fabsf(v[b][3])));
      }
    };
    auto mfma_pos = [&](int pl, const h4 (&hl)[2], const w4 (&u)[kNF]) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < kNF; ++j) {
          const h8 uu = __builtin_bit_cast(h8, u[j]);
          const h4 uh = __builtin_shufflevector(uu, uu, 0, 1, 2, 3);
          const h4 ul = __builtin_shufflevector(uu, uu, 4, 5, 6, 7);
          const h4 av = p == 0 ? hl[1] : hl[0];
          const h4 bv = p == 1 ? ul : uh;
          acc[pl][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(av, bv, acc[pl][j], 0, 0, 0);
        }
    };
    auto read_u1 = [&](int buf, int pos, w4 (&u)[kNF]) {
#pragma unroll
      for (int j = 0; j < kNF; ++j)
        u[j] = *(const w4*)(ust + buf * kUStage + (pos * kNF + j) * 256 + lane * 4);
    };
    h4 hA[4][2], hB[4][2];
    w4 u1[4][kNF];  // row r1's U, read before the slab barrier
    // prologue
    load_halo(0);
#pragma unroll
    for (int k = 0; k < kPU; ++k) issue_u1(0, 0, k);
    stage_bias(btab, 16 * kNF, nf0 * 16, g.N, g.b3, g.vtap, g.bfull, g.ldv, tid, kPThreads);
    store_halo(0);
    __builtin_amdgcn_sched_barrier(0);
    load_halo(1 < S ? 1 : S - 1);
    barrier();
    fetch_row(0, T0::i0, da);
    fetch_row(0, T0::i1, db);
    vsplit(T0{}, hA);
    for (int s = 0; s < S; ++s) {
      const int buf = s & 1;
      // phase A: row r0's MFMAs (U read position by position); row r1's operands; slab s+1's
      // halo writes and U pieces, slab s+2's halo loads
      __builtin_amdgcn_sched_barrier(0);
      fetch_row(buf, XR, dx);
      vsplit(T1{}, hB);
      store_halo(buf ^ 1);
      {
        const int us = s + 1 < S ? s + 1 : S - 1;
        w4 u0[4][kNF];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          read_u1(buf, 4 * R0 + b, u0[b]);
          mfma_pos(b, hA[b], u0[b]);
          issue_u1(us, buf ^ 1, b);
          if (b < 2) issue_u1(us, buf ^ 1, 4 + b);
        }
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) read_u1(buf, 4 * R1 + b, u1[b]);
#pragma unroll
      for (int k = 0; k < 36; ++k) {
        if (k < kPHalo) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (k < 28) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
      // slab s+2's halo loads strictly after the U pieces: the barrier's vmcnt(4) then waits
      // for exactly the pieces
      __builtin_amdgcn_sched_barrier(0);
      load_halo(s + 2 < S ? s + 2 : S - 1);
      __builtin_amdgcn_sched_barrier(0);
      barrier();
      // phase B: row r1's MFMAs beside slab s+1's patch reads and row r0's operands (past the
      // last slab: the last slab again, unused)
      fetch_row(buf ^ 1, T0::i0, da);
      fetch_row(buf ^ 1, T0::i1, db);
      vsplit(T0{}, hA);
#pragma unroll
      for (int b = 0; b < 4; ++b) mfma_pos(4 + b, hB[b], u1[b]);
#pragma unroll
      for (int k = 0; k < 36; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (k < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (k >= 6) __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if (rp == 0) run(C<0>{});
  else run(C<1>{});

  if constexpr (CHK) {
    float asum = 0.0f;
#pragma unroll
    for (int p = 0; p < 8; ++p)
#pragma unroll
      for (int j = 0; j < kNF; ++j) asum += (acc[p][j][0] + acc[p][j][1]) + (acc[p][j][2] + acc[p][j][3]);
    if ((!(gmax < kGuardIn) || !(asum - asum == 0.0f)) && g.flag) atomicOr(g.flag, 1u);
  }

  // ---- epilogue.  Half-row sums of A^T M for this wave's rows, per (tile r, n-fragment j,
  // column b): rp = 0 holds m0, m1 -> P = m0 + m1 (row 0 of A^T M), Q = m1 (row 1); rp = 1
  // holds m2, m3 -> P = m2, Q = -(m2 + m3).  Row 0 = P0 + P1, row 1 = Q0 + Q1 (a fixed order).
  // rp = 0 finishes tiles r = 0, 1 of its lanes, rp = 1 tiles r = 2, 3: each writes the other
  // two tiles' (P, Q) to LDS, reads its partner's for its own two.
  float* xch = lds;  // [8 waves][2 tiles][3 nf][4 b][2][64 lanes] (98 KB, the stages are free)
  __syncthreads();   // every wave is past its last stage read
  auto pq = [&](int r, int j, int b, float& P, float& Q) {
    const float m0 = acc[b][j][r], m1 = acc[4 + b][j][r];  // this wave's rows 2rp, 2rp+1
    if (rp == 0) { P = m0 + m1; Q = m1; }
    else { P = m0; Q = -(m0 + m1); }
  };
  const int give0 = rp == 0 ? 2 : 0;  // the tiles this wave hands to its partner
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int j = 0; j < kNF; ++j)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float P, Q;
        pq(give0 + rr, j, b, P, Q);
        float* dst = xch + ((((wave * 2 + rr) * kNF + j) * 4 + b) * 2) * 64 + lane;
        dst[0] = P;
        dst[64] = Q;
      }
  __syncthreads();
  const int partner = wave ^ 4, own0 = rp == 0 ? 0 : 2;
  const int nn = lane & 15;
  const int64_t obytes = ((int64_t)g.B * g.H * g.Wd - (int64_t)b0 * g.H * g.Wd) * g.ldo * 4;
  const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.out + (int64_t)b0 * g.H * g.Wd * g.ldo), 0,
      (int)(obytes < (int64_t)kInvalid ? obytes : (int64_t)kInvalid), 0x00020000);
  bool out_ok = true;
  auto epilogue = [&](auto tanh_c) {
    constexpr bool TANH = decltype(tanh_c)::value;
    const WAct act(g.act, g.slope);
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int r = own0 + rr;
      const int t = 16 * tf + 4 * (lane >> 4) + r;
      const int img = udiv_s(t, TPI);
      const int rem = t - img * TPI;
      const int ty = udiv_s(rem, TTW), tx = rem - ty * TTW;
      uint32_t po[4];
      int pcl[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int y = y0 + 2 * ty + (e >> 1), x = x0 + 2 * tx + (e & 1);
        const bool ok = img < g.IMGS && b0 + img < g.B && y < g.H && x < g.Wd;
        po[e] = ok ? (uint32_t)((img * g.H + y) * g.Wd + x) * (uint32_t)(g.ldo * 4) : kInvalid;
        pcl[e] = bias_class(y, x, g.H, g.Wd) * (16 * kNF) + nn;
      }
#pragma unroll
      for (int j = 0; j < kNF; ++j) {
        const int n = (nf0 + j) * 16 + nn;
        float u0[4], u1v[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          float P, Q;
          pq(r, j, b, P, Q);
          const float* src = xch + ((((partner * 2 + rr) * kNF + j) * 4 + b) * 2) * 64 + lane;
          const float Po = src[0], Qo = src[64];
          // row sums in a fixed order: the rp = 0 half first
          u0[b] = rp == 0 ? P + Po : Po + P;
          u1v[b] = rp == 0 ? Q + Qo : Qo + Q;
        }
        float Y[4];
        Y[0] = (u0[0] + u0[1]) + u0[2];
        Y[1] = (u0[1] - u0[2]) - u0[3];
        Y[2] = (u1v[0] + u1v[1]) + u1v[2];
        Y[3] = (u1v[1] - u1v[2]) - u1v[3];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = Y[e] * g.yscale + btab[pcl[e] + j * 16];
          v = TANH ? wact(v, g.act, g.slope) : act(v);
          const bool st = po[e] != kInvalid && n < g.N;
          out_ok = out_ok && (!st || fabsf(v) < kGuardOut);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), orr,
                                                st ? po[e] + (uint32_t)n * 4u : kInvalid, 0, 0);
        }
      }
    }
  };
  if (g.act == IDF_ACT_TANH) epilogue(std::true_type{});
  else epilogue(std::false_type{});
  if (!out_ok && g.flag) atomicOr(g.flag, 1u);
}

}  // namespace wq

// Launch the wq kernel when the geometry and mode are its scope; IDF_ERR_UNSUPPORTED otherwise
// (the caller then runs wx3).  Arguments as idf_conv3x3_wx3.
int wq_launch(void* stream, int32_t B, int32_t H, int32_t W, int32_t C, const float* x,
              int64_t ld_x, const uint16_t* u, int32_t nft, float yscale, const float* b3,
              const float* vtap, int32_t ldv, const float* bfull, int32_t N, float* out,
              int64_t ld_out, int32_t act, float slope, uint32_t* flag, int32_t check_input) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || (ld_x & 3) || !u || !out) return IDF_ERR_ARG;
  const int nf_total = (N + 15) / 16;
  if (nf_total % wq::kNF != 0 || nft < nf_total) return IDF_ERR_UNSUPPORTED;
  const int nslab = (C + 15) / 16;
  WinoPlan pl = wino_plan(H, W, nslab, N);
  if (!pl.ok || pl.big || pl.ksplit != 1 || !(pl.TW == 32 || pl.TW == 16)) return IDF_ERR_UNSUPPORTED;
  // per-block buffer offsets (input halo, output stores) are 32-bit
  if ((int64_t)pl.IMGS * H * W * ld_x * 4 >= (int64_t)wq::kInvalid) return IDF_ERR_UNSUPPORTED;
  if ((int64_t)pl.IMGS * H * W * ld_out * 4 >= (int64_t)wq::kInvalid) return IDF_ERR_UNSUPPORTED;
  if ((int64_t)16 * nslab * nft * 1024 >= (int64_t)wq::kInvalid) return IDF_ERR_UNSUPPORTED;
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  wq::Args g = {};
  g.X = x; g.ldx = ld_x; g.C = C; g.U = (const float*)u; g.nslab = nslab; g.nft = nft; g.N = N;
  g.B = B; g.H = H; g.Wd = W;
  g.IMGS = pl.IMGS; g.TH = pl.TH; g.TW = pl.TW;
  const int tiles_b = (B + pl.IMGS - 1) / pl.IMGS;
  g.tiles_y = (H + pl.TH - 1) / pl.TH;
  g.tiles_x = (W + pl.TW - 1) / pl.TW;
  g.n_tiles = nf_total / wq::kNF;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out; g.yscale = yscale; g.flag = flag;
  const int64_t blocks = (int64_t)tiles_b * g.tiles_y * g.tiles_x * g.n_tiles;
  if (blocks >= (1 << 20) || nslab >= (1 << 20)) return IDF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  // IDF_WQ_VARIANT=p: the two-waves-per-SIMD form (conv3_wp_kernel)
  static const bool wp = [] {
    const char* e = getenv("IDF_WQ_VARIANT");
    return e && e[0] == 'p';
  }();
#define IDF_WQ_LAUNCH(twc, chk)                                                                 \
  do {                                                                                          \
    if (wp)                                                                                     \
      hipLaunchKernelGGL((wq::conv3_wp_kernel<twc, chk>), dim3((unsigned)blocks),               \
                         dim3(wq::kPThreads), 0, s, g);                                         \
    else                                                                                        \
      hipLaunchKernelGGL((wq::conv3_wq_kernel<twc, chk>), dim3((unsigned)blocks),               \
                         dim3(wq::kThreads), 0, s, g);                                          \
  } while (0)
  if (pl.TW == 32) { if (check_input) IDF_WQ_LAUNCH(32, true); else IDF_WQ_LAUNCH(32, false); }
  else { if (check_input) IDF_WQ_LAUNCH(16, true); else IDF_WQ_LAUNCH(16, false); }
#undef IDF_WQ_LAUNCH
  return idf_last_error();
}

bool wq_enabled() {
  static const bool on = [] {
    const char* e = getenv("IDF_WQ");
    return e && e[0] == '1';
  }();
  return on;
}

}  // namespace idf

extern "C" int idf_conv3x3_wq(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                              const float* x, int64_t ld_x, const uint16_t* u, int32_t nft,
                              float yscale, const float* b3, const float* vtap, int32_t ldv,
                              const float* bfull, int32_t N, float* out, int64_t ld_out,
                              int32_t act, float slope, uint32_t* d_flag, int32_t check_input) {
  return idf::wq_launch(stream, B, H, W, C, x, ld_x, u, nft, yscale, b3, vtap, ldv, bfull, N, out,
                        ld_out, act, slope, d_flag, check_input);
}
