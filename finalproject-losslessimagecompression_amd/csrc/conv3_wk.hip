// conv3_wk.hip -- "wk": the DenseLayer 3x3 convolution (nnlayer.py:48-51 with the 1x1 folded
// in, nnblock.py:53-56) as Winograd F(2x2, 3x3) with fp32-accurate split-f16 products, all
// three of them on K=32 MFMAs (v_mfma_f32_16x16x32_f16), one wave per SIMD.
//
// What it computes is what conv3_wino.hip's X3 path ("wx3") computes: per 2x2 output tile
//   Y = A^T [ sum_c U_c (.) V_c ] A,  V_c = B^T d_c B,  U_c = G g_c G^T (host, float64),
// with every f32 operand carried as an f16 pair (V = Vh + Vl, U' = U 2^k = Uh + Ul) and
// V.U' ~= Vh.Uh + Vl.Uh + Vh.Ul accumulated in f32 (each f16 x f16 product is exact in f32;
// the dropped Vl.Ul is ~2^-22 of V.U').  What differs is the shape of the work:
//
//  * K=32 products.  A lane holds EIGHT channels of a 32-channel slab (its two channel quads
//    2lq, 2lq+1), so one v_mfma_f32_16x16x32_f16 takes Vh[8] x Uh[8] (or Vl x Uh, Vh x Ul)
//    for 16 tiles x 16 outputs: three K=32 MFMAs per (position, n-fragment) and 32 channels
//    where wx3 issues six K=16 MFMAs -- the K=16 form runs at half the f16 rate on gfx950
//    (16 cycles for half the work), so this halves the matrix-pipe time.
//  * One wave per SIMD, a full B^T row per wave.  Block = 4 waves = 64 Winograd tiles (256
//    output pixels) x 16*NF outputs; wave a owns the four positions (a, 0..3), so its input
//    transform is the minimal separable one (four row combinations T_j = +-d[i0][j] +-
//    d[i1][j], then four column combinations, no work shared or repeated across waves) and
//    its accumulators (4 positions x 4 tile fragments x NF n-fragments = 192 VGPRs at NF = 3)
//    plus the slab's U fragments (96) fit the 512-register budget of a lone wave.
//  * Output transform half in registers.  A wave holds every column position of its row, so
//    (M A)[a][c] (c = 0, 1) is formed from its own accumulators; only those two values per
//    (tile, output) go through LDS for the row half -- half the staging of wx3, and all
//    n-fragments in one pass (2 barriers per tile instead of 2 per n-fragment).
//  * XCD-aware block order: consecutive tiles of the image grid run on one XCD (blocks b and
//    b + 8 share an XCD under round-robin dispatch), so the halo rows neighbouring tiles both
//    read come from that XCD's L2.
//
// Per 32-channel slab the tile's (rows+2) x (cols+2) halo is staged in LDS (channel-quad-major
// [8 quads][kSlots][4 floats], columns de-interleaved even/odd so the stride-2 patch reads of
// 16 neighbouring tiles are conflict-free ds_read_b128s) through registers with coalesced
// 128-B-per-pixel loads, double-buffered: slab s+1's loads are issued in step 0 of slab s and
// written in steps 1-2, one barrier per slab (before step 3, which prepares slab s+1's first
// fragment).  U fragments (Uh[8], Ul[8] per lane; idfcodec/packing.py wk_weights) are loaded
// straight into registers; slab s+1's replace slab s's right after their last MFMA (step 3).
//
// Determinism: every output is a fixed-order f32 sum whose order depends on the geometry and
// channel count only (never the batch size or block placement), so an encoder and a decoder
// running this kernel agree bit for bit.  Parity: tests/test_gpu_wk.py (<= 1e-5 against fp64
// conv2d, within a small factor of the exact-f32 kernel's own error).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "idf_codec_internal.h"
#include "wino_common.h"

#pragma clang fp contract(off)

// timing-only ablations (tools/native, never set in the library build): bit 0 no halo
// loads/stores, bit 1 no LDS reads (fixed operands), bit 2 no MFMAs, bit 3 no transform /
// split VALU, bit 4 no in-loop barrier, bit 5 no U reloads, bit 6 no epilogue stores
#ifndef IDF_WK_ABLATE
#define IDF_WK_ABLATE 0
#endif
// timing-only s_memtime stamps per (block, wave) into g.part (tools/native wk_stamps)
#ifndef IDF_WK_STAMPS
#define IDF_WK_STAMPS 0
#endif

namespace idf {
namespace wk {

typedef float w4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 512;
constexpr int kSlots = 448;                     // halo slots per channel quad of a stage (>= 400)
constexpr int kStage = 8 * kSlots * 4;          // floats: [8 quads][kSlots][4]
constexpr int kRounds = (kWMaxHalo + 63) / 64;  // halo loads per thread per slab (7)
constexpr uint32_t kInvalid = 0xFFFFFFF0u;      // buffer offset that always reads 0
constexpr uint32_t kHaloOut = 0x80000000u;      // halo slot outside the image (see load_halo)
constexpr uint32_t kChanOut = 0x40000000u;      // channel quad past C
constexpr float kGuardIn = 32768.0f;            // |V| bound of the f16 pairs (f16 max 65504)
constexpr float kGuardOut = 8192.0f;            // layer outputs (|V| <= 4 max|input| next layer)

struct Args {
  const float* X;
  int64_t ldx;
  int64_t slab_stride;  // 0: X is pixel-major [P][ldx]; else slab-major [C/32][slab_stride / 32][32]
  int32_t C;
  const uint16_t* U;  // [16 pos][nslab][nft][2: hi, lo][64 lanes][8 f16]
  int32_t nslab, nft, N;
  int32_t B, H, Wd;
  int32_t IMGS, TH, TW;
  int32_t tiles_b, tiles_y, tiles_x, n_tiles, ksplit, nblocks;
  const float* b3;
  const float* vtap;
  const float* bfull;
  int32_t ldv;
  int32_t act;
  float slope;
  float* out;
  int64_t ldo;
  float* part;  // split-K partial sums [ksplit][P][ldp]
  int32_t ldp;
  const float* res;  // optional residual added before the activation (VQ-VAE ResBlock)
  int64_t ldr;
  float yscale;     // 2^-k: undoes the U' = U 2^k scaling of the f16 pairs
  uint32_t* flag;   // bit 0 set when a range guard trips
  int32_t vec4;     // out and ldo allow 16-B stores of 4 outputs
};

// s0*x0 + s1*x1 per channel, four scalar adds (packed f32 adds cost more issue beside MFMAs)
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

// f16 pair of four f32 values: h = f16(v), l = f16(v - h), both nearest-even (v - h is exact).
// IDF_WK_MIX: l by v_fma_mix{lo,hi}_f16 (reads h as f16 and v as f32, rounds fma(-h, 1, v) to
// f16 once: the same bits, one instruction per value instead of a convert back and a subtract)
#ifndef IDF_WK_MIX
#define IDF_WK_MIX 1
#endif
__device__ __forceinline__ void split(const w4& v, h4& h, h4& l) {
  h = __builtin_convertvector(v, h4);
  if (!IDF_WK_MIX) {
    l = __builtin_convertvector(v - __builtin_convertvector(h, w4), h4);
    return;
  }
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const h2 ha = __builtin_shufflevector(h, h, 0, 1), hb = __builtin_shufflevector(h, h, 2, 3);
  uint32_t la, lb;
  asm("v_fma_mixlo_f16 %0, -%2, 1.0, %4 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %1, -%3, 1.0, %6 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, -%2, 1.0, %5 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, -%3, 1.0, %7 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(la), "=&v"(lb)
      : "v"(ha), "v"(hb), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  l = __builtin_bit_cast(h4, u2{la, lb});
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int NF, int TWC, bool CHK>
__global__ void __launch_bounds__(kThreads, 1) conv3_wk_kernel(Args g) {
  constexpr int NN = NF * 16;  // outputs per block
  __shared__ __attribute__((aligned(16))) float lds[2 * kStage + 16 * NN];
  float* const btab = lds + 2 * kStage;  // epilogue bias table [16 border classes][NN]
  static_assert(8 * 64 * NN <= 2 * kStage, "epilogue staging must fit in the stages");

  uint64_t stamp[6] = {0, 0, 0, 0, 0, 0};
  if (IDF_WK_STAMPS) stamp[0] = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: blocks b and b + 8 run on one XCD; give each XCD a contiguous run
  int bid = blockIdx.x;
  if ((g.nblocks & 7) == 0) bid = (bid & 7) * (g.nblocks >> 3) + (bid >> 3);
  const int ks = bid - udiv_s(bid, g.ksplit) * g.ksplit;
  bid = udiv_s(bid, g.ksplit);
  const int nt = bid - udiv_s(bid, g.n_tiles) * g.n_tiles;
  bid = udiv_s(bid, g.n_tiles);
  const int tx_ = bid - udiv_s(bid, g.tiles_x) * g.tiles_x;
  bid = udiv_s(bid, g.tiles_x);
  const int tb = udiv_s(bid, g.tiles_y);
  const int ty_ = bid - tb * g.tiles_y;
  const int b0 = tb * g.IMGS, y0 = ty_ * g.TH, x0 = tx_ * g.TW;
  const int HWp = TWC > 0 ? halo_pitch(TWC) : halo_pitch(g.TW), HH = g.TH + 2, EH = HWp >> 1;
  const int NH = g.IMGS * HH * HWp;
  const int TTW = g.TW >> 1, TPI = (g.TH >> 1) * TTW;
  const int s_lo = udiv_s(ks * g.nslab, g.ksplit);
  const int s_hi = udiv_s((ks + 1) * g.nslab, g.ksplit);
  const int nf0 = nt * NF;

  // ---- halo loader: round m of thread (wave, lane) stages slot 64m + 8 wave + (lane & 7),
  // channel quad hq = lane >> 3 (8 lanes of one quad = 8 slots: conflict-free b128 writes;
  // one load instruction = 8 pixels x 128 B).  Out-of-range loads read 0 (buffer range check):
  // the record covers the block's own images (< 1 GiB, checked on the host); a halo slot
  // outside the image has source kHaloOut and a channel quad past C adds kChanOut, so every
  // such sum is >= 1 GiB and no select sits on the per-load path.
  const int64_t pstride = g.slab_stride ? 32 : g.ldx;  // floats between pixels
  const float* xbase = g.X + (int64_t)b0 * g.H * g.Wd * pstride;
  const int nimg = g.B - b0 < g.IMGS ? g.B - b0 : g.IMGS;
  const int64_t xrec = g.slab_stride ? ((int64_t)g.nslab * g.slab_stride - (int64_t)b0 * g.H * g.Wd * 32) * 4
                                     : (int64_t)nimg * g.H * g.Wd * g.ldx * 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)xbase, 0, (int)xrec, 0x00020000);
  const int hq = lane >> 3;
  uint32_t hsrc[kRounds];
#pragma unroll
  for (int m = 0; m < kRounds; ++m) {
    const int slot = 64 * m + 8 * wave + (lane & 7);
    hsrc[m] = kHaloOut;
    if (slot < NH) {
      const int img = udiv_s(slot, HH * HWp);
      const int rem = slot - img * HH * HWp;
      const int hy = udiv_s(rem, HWp), cs = rem - hy * HWp;
      const int hx = cs < EH ? 2 * cs : 2 * (cs - EH) + 1;
      const int y = y0 + hy - 1, x = x0 + hx - 1;
      // hx >= TW + 2: a pitch pad slot (never read)
      if (b0 + img < g.B && y >= 0 && y < g.H && x >= 0 && x < g.Wd && hx < g.TW + 2)
        hsrc[m] = (uint32_t)(((((int64_t)img * g.H + y) * g.Wd + x) * pstride + 4 * hq) * 4);
    }
  }
  const int hdst = (hq * kSlots + 8 * wave + (lane & 7)) * 4;  // round m: + 256 m floats
  auto load_halo = [&](int slab, w4* hb, int m0, int m1) {
    const int c0 = slab * 32;
    const uint32_t cb = c0 + 4 * hq < g.C ? (g.slab_stride ? (uint32_t)(slab * g.slab_stride * 4) : (uint32_t)c0 * 4u)
                                          : kChanOut;
#pragma unroll
    for (int m = m0; m < m1; ++m)
      hb[m - m0] = (IDF_WK_ABLATE & 1) ? w4{0.f, 0.f, 0.f, 0.f}
                   : __builtin_bit_cast(w4, __builtin_amdgcn_raw_buffer_load_b128(xr, hsrc[m] + cb, 0, 0));
  };
  auto store_halo = [&](int buf, const w4* hb, int m0, int m1) {
    if (IDF_WK_ABLATE & 1) return;
#pragma unroll
    for (int m = m0; m < m1; ++m) *(w4*)(lds + buf * kStage + hdst + 256 * m) = hb[m - m0];
  };

  // ---- U: fragment (position, n-fragment nf) of slab s: this lane's Uh[8] and Ul[8]; the
  // fragment's wave-uniform offset goes in soffset, the lane's 16 B in voffset
  const int64_t ubytes = (int64_t)16 * g.nslab * g.nft * 2048;
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.U, 0, (int)(ubytes < (int64_t)kInvalid ? ubytes : (int64_t)kInvalid), 0x00020000);
  const int u_voff = lane * 16;

  // ---- per-lane tile bases: tile t = 16 f + (lane & 15) -> slot of its patch's top-left,
  // channel quad 2 lq (the lane's k-group lq holds channels 8 lq .. 8 lq + 7 of the slab)
  const int lr = lane & 15, lq = lane >> 4;
  const float* pb[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int t = 16 * f + lr;
    int img = udiv_s(t, TPI);
    const int rem = t - img * TPI;
    const int ty = udiv_s(rem, TTW), tx = rem - ty * TTW;
    if (img >= g.IMGS) img = 0;  // idle rows read valid LDS
    pb[f] = lds + ((2 * lq) * kSlots + (img * HH + 2 * ty) * HWp + tx) * 4;
  }

  w4 acc[4][2][NF];  // [tile fragment][position q][n-fragment]
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[f][q][j] = w4{0.f, 0.f, 0.f, 0.f};
  float gmax = 0.0f;  // CHK: max |V| of the layer's inputs

  // Epilogue bias table (stage_bias's values, bit for bit): its loads are issued with the
  // prologue's halo and U loads (one global round trip for all), the table written after them.
  constexpr int NE = (16 * NN + kThreads - 1) / kThreads;
  float bq[NE][11];
  auto bias_load = [&]() {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + kThreads * i;
      const int cls = e / NN, k = e - cls * NN, n = nf0 * 16 + k;
      const int ns = (e < 16 * NN && n < g.N) ? n : 0;
      bq[i][0] = g.b3[ns];
      if (g.vtap) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) bq[i][1 + tap] = g.vtap[tap * g.ldv + ns];
        bq[i][10] = g.bfull[ns];
      }
    }
  };
  auto bias_store = [&]() {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + kThreads * i;
      const int cls = e / NN, k = e - cls * NN, n = nf0 * 16 + k;
      float v = 0.0f;
      if (n < g.N) {
        v = bq[i][0];
        if (g.vtap) {
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) {
            const int dy = tap / 3 - 1, dx = tap % 3 - 1;
            const bool ok = !((dy < 0 && (cls & 1)) || (dy > 0 && (cls & 2)) ||
                              (dx < 0 && (cls & 4)) || (dx > 0 && (cls & 8)));
            v = ok ? v + bq[i][1 + tap] : v;
          }
          v = cls == 0 ? bq[i][10] : v;
        }
      }
      if (e < 16 * NN) btab[e] = v;
    }
  };

  // Wave (A, BP) owns positions (A, 2 BP) and (A, 2 BP + 1): they share B^T row A, so the wave
  // reads halo rows i0(A), i1(A) at the three patch columns BP .. BP + 2, forms the three row
  // combinations once and both positions' column combinations from them.
  auto run = [&](auto a_tag, auto bp_tag) {
    constexpr int A = decltype(a_tag)::value, BP = decltype(bp_tag)::value;
    using RA = BT<A>;
    using C0 = BT<2 * BP>;
    using C1 = BT<2 * BP + 1>;
    // six reads of channel-quad half h (rows i0, i1 x columns BP .. BP + 2)
    auto read_half = [&](const float* base, int h, w4 (&d)[2][3]) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
          const int row = r == 0 ? RA::i0 : RA::i1, j = BP + jj;
          if (IDF_WK_ABLATE & 2) {  // fake, lane- and step-varying operands (not constant-folded)
            const float fv = __builtin_bit_cast(float, (uint32_t)(size_t)base) * 1e-30f;
            d[r][jj] = w4{fv + (float)jj, fv * 2.f, fv + (float)r, fv + (float)h};
          } else if constexpr (TWC > 0) {
            constexpr int HWc = halo_pitch(TWC), EHc = HWc / 2;
            const int cs = (j & 1) ? EHc + (j >> 1) : (j >> 1);
            d[r][jj] = *(const w4*)(base + (h * kSlots + row * HWc + cs) * 4);
          } else {
            const int cs = (j & 1) ? EH + (j >> 1) : (j >> 1);
            d[r][jj] = *(const w4*)(base + (h * kSlots + row * HWp + cs) * 4);
          }
        }
    };
    // transform + f16 split of one half: vh[q] / vl[q] = the f16 pair of V at position
    // (A, 2 BP + q) for the half's four channels
    auto xform_half = [&](const w4 (&d)[2][3], h4 (&vh)[2], h4 (&vl)[2], bool valid) {
      w4 T[3];
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) T[jj] = comb<RA::neg0, RA::neg1>(d[0][jj], d[1][jj]);
      w4 V[2];
      V[0] = comb<C0::neg0, C0::neg1>(T[C0::i0 - BP], T[C0::i1 - BP]);
      V[1] = comb<C1::neg0, C1::neg1>(T[C1::i0 - BP], T[C1::i1 - BP]);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (IDF_WK_ABLATE & 8) {
          vh[q] = __builtin_bit_cast(h4, __builtin_shufflevector(d[0][q], d[0][q], 0, 1));
          vl[q] = __builtin_bit_cast(h4, __builtin_shufflevector(d[1][q], d[1][q], 0, 1));
          continue;
        }
        split(V[q], vh[q], vl[q]);
        if constexpr (CHK) {
          const float m = fmaxf(fmaxf(fabsf(V[q][0]), fabsf(V[q][1])), fmaxf(fabsf(V[q][2]), fabsf(V[q][3])));
          gmax = valid ? fmaxf(gmax, m) : gmax;
        }
      }
    };

    h8 uh[2][NF], ul[2][NF];
    auto load_u = [&](int q, int nf, int slab) {
      const int so = __builtin_amdgcn_readfirstlane(
          (((4 * A + 2 * BP + q) * g.nslab + slab) * g.nft + nf0 + nf) * 2048);
      uh[q][nf] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(ur, u_voff, so, 0));
      ul[q][nf] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(ur, u_voff + 1024, so, 0));
    };
    if (s_lo >= s_hi) {
      if (g.ksplit == 1) { bias_load(); bias_store(); }
      return;
    }
    // prologue: U(s_lo), the bias table's loads and slab s_lo's halo in one round trip
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) load_u(q, nf, s_lo);
    if (g.ksplit == 1) bias_load();
    // the halo of slab s + 2 goes in four batches (loads kB[k] .. kB[k+1]), each written two
    // steps after it is issued (see the slab loop); the prologue plays steps (s_lo - 1, 1..3)
    constexpr int kB[5] = {0, 2, 4, 6, kRounds};
    w4 hb0[2], hb1[2], hb2[2], hb3[kRounds - 6];
    {
      w4 hb[kRounds];
      load_halo(s_lo, hb, 0, kRounds);
      load_halo(s_lo + 1, hb0, kB[0], kB[1]);
      load_halo(s_lo + 1, hb1, kB[1], kB[2]);
      load_halo(s_lo + 1, hb2, kB[2], kB[3]);
      store_halo(0, hb, 0, kRounds);
      store_halo(1, hb0, kB[0], kB[1]);
    }
    if (g.ksplit == 1) bias_store();
    lds_barrier();
    if (IDF_WK_STAMPS) stamp[1] = __builtin_amdgcn_s_memtime();
    h8 ahh[2], all[2];
    {
      w4 d[2][2][3];
      h4 vh[2][2], vl[2][2];
      read_half(pb[0], 0, d[0]);
      read_half(pb[0], 1, d[1]);
      xform_half(d[0], vh[0], vl[0], true);
      xform_half(d[1], vh[1], vl[1], true);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        ahh[q] = __builtin_shufflevector(vh[0][q], vh[1][q], 0, 1, 2, 3, 4, 5, 6, 7);
        all[q] = __builtin_shufflevector(vl[0][q], vl[1][q], 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }

    // Per slab s (stage buf), step tf: the 6 NF MFMAs of fragment tf, interleaved with the 12
    // reads of fragment tf + 1 (step 3: fragment 0 of slab s + 1 from stage buf ^ 1) and their
    // transform and split.  The halo streams two steps ahead of its LDS writes (HBM latency
    // under this load exceeds a step): batch k of slab X is issued in step (X-2, 1+k) (batch 3:
    // (X-1, 0)) and written in step (X-2, 3+k) -- (X-2, 3), (X-1, 0), (X-1, 1), (X-1, 2); the
    // stage of X is free from the barrier of step (X-2, 3) on (every wave's last read of slab
    // X - 2 was consumed before it) and the barrier of step (X-1, 3) publishes it.  U(s + 1)
    // replaces U(s) right after each fragment's last MFMA (step 3).
    for (int s = s_lo; s < s_hi; ++s) {
      const int buf = (s - s_lo) & 1;
      const bool more = s + 1 < s_hi;
      const int sn = more ? s + 1 : s;  // U of the next slab (past the end: unused, in range)
      auto step = [&](auto tfc) {
        constexpr int TF = decltype(tfc)::value;
        if constexpr (TF == 3) {
          if (!(IDF_WK_ABLATE & 16)) lds_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
        // halo batches, each written two steps after its loads were issued: slab s + 1's into
        // stage buf ^ 1 (free since the barrier of step (s-1, 3)), slab s + 2's batch 0 into
        // stage buf in step 3 (free since this slab's barrier); past the last slab they read
        // zeros into stages nothing reads
        if constexpr (TF == 0) { store_halo(buf ^ 1, hb1, kB[1], kB[2]); load_halo(s + 1, hb3, kB[3], kB[4]); }
        if constexpr (TF == 1) { store_halo(buf ^ 1, hb2, kB[2], kB[3]); load_halo(s + 2, hb0, kB[0], kB[1]); }
        if constexpr (TF == 2) { store_halo(buf ^ 1, hb3, kB[3], kB[4]); load_halo(s + 2, hb1, kB[1], kB[2]); }
        if constexpr (TF == 3) { store_halo(buf, hb0, kB[0], kB[1]); load_halo(s + 2, hb2, kB[2], kB[3]); }
        const float* nb = (TF < 3 ? pb[TF + 1] : pb[0]) + (TF < 3 ? buf : buf ^ 1) * kStage;
        w4 d[2][2][3];
        h4 vh[2][2], vl[2][2];
        read_half(nb, 0, d[0]);
        read_half(nb, 1, d[1]);
        xform_half(d[0], vh[0], vl[0], TF < 3 || more);
        xform_half(d[1], vh[1], vl[1], TF < 3 || more);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) {
            if (!(IDF_WK_ABLATE & 4)) {
              acc[TF][q][nf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahh[q], uh[q][nf], acc[TF][q][nf], 0, 0, 0);
              acc[TF][q][nf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(all[q], uh[q][nf], acc[TF][q][nf], 0, 0, 0);
              acc[TF][q][nf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahh[q], ul[q][nf], acc[TF][q][nf], 0, 0, 0);
            } else {
              acc[TF][q][nf][0] += (float)ahh[q][0] * (float)uh[q][nf][0] + (float)all[q][1];
            }
            if constexpr (TF == 3) {
              if (!(IDF_WK_ABLATE & 32)) load_u(q, nf, sn);
            }
          }
        // interleave per MFMA: the 12 reads over the first MFMAs, the transform / split VALU
        // after them, the step's halo loads and writes early, the U reloads after their last
        // MFMA (step 3)
        {
          constexpr int NM = 6 * NF;
          constexpr int nvm = TF == 0 ? kB[4] - kB[3] : 2;
          constexpr int nds = TF == 3 ? 2 : (TF == 2 ? kB[4] - kB[3] : 2);
#pragma unroll
          for (int k = 0; k < NM; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            if (k < 6) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
            if (k < nds) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
            if (k < nvm) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // halo load
            if (TF == 3 && k % 3 == 2) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);  // U
            if (k >= 2) __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          ahh[q] = __builtin_shufflevector(vh[0][q], vh[1][q], 0, 1, 2, 3, 4, 5, 6, 7);
          all[q] = __builtin_shufflevector(vl[0][q], vl[1][q], 0, 1, 2, 3, 4, 5, 6, 7);
        }
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  switch (wave) {
    case 0: run(I0{}, I0{}); break;
    case 1: run(I0{}, I1{}); break;
    case 2: run(I1{}, I0{}); break;
    case 3: run(I1{}, I1{}); break;
    case 4: run(I2{}, I0{}); break;
    case 5: run(I2{}, I1{}); break;
    case 6: run(I3{}, I0{}); break;
    default: run(I3{}, I1{}); break;
  }
  if (IDF_WK_STAMPS) stamp[2] = __builtin_amdgcn_s_memtime();

  if constexpr (CHK) {
    // gmax (v_max ignores NaN operands) catches out-of-range V; a NaN anywhere in V reaches
    // the accumulators, so their sum catches it
    float asum = 0.0f;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < NF; ++j)
          asum += (acc[f][q][j][0] + acc[f][q][j][1]) + (acc[f][q][j][2] + acc[f][q][j][3]);
    if ((!(gmax < kGuardIn) || !(asum - asum == 0.0f)) && g.flag) atomicOr(g.flag, 1u);
  }

  // ---- output transform Y = A^T M A.  Columns: (M A)[a][c] = sum over b of M[a][b] A[b][c]
  // (c = 0: m0 + m1 + m2, c = 1: m1 - m2 - m3); wave (a, bp) holds b = 2bp, 2bp + 1 and forms
  // its part P[a][bp][c] in registers (bp 0: m0 + m1 | m1, bp 1: m2 | -m2 - m3).  Rows through
  // LDS, one column c per pass (S[a][bp][tile][n] aliases the halo stages):
  //   Y[0][c] = (Q0 + Q1) + Q2, Y[1][c] = (Q1 - Q2) - Q3, Qa = P[a][0][c] + P[a][1][c].
  const int A_ = wave >> 1, BP_ = wave & 1;
  const WAct act(g.act, g.slope);
  const int64_t pix0 = (int64_t)b0 * g.H * g.Wd;
  float* obase = g.out ? g.out + pix0 * g.ldo : nullptr;
  float* pbase = g.part ? g.part + ((int64_t)ks * ((int64_t)g.B * g.H * g.Wd) + pix0) * g.ldp : nullptr;
  const float* rbase = g.res ? g.res + pix0 * g.ldr : nullptr;
  bool out_ok = true;
  // plain epilogue (every DenseLayer conv of the flow): no split-K, residual or Tanh, 16-B
  // rows, N a multiple of 4, all 64 tiles inside the batch and the image -- no per-pixel or
  // per-channel branches, one 16-B store per pixel
  const bool full = b0 + g.IMGS <= g.B && y0 + g.TH <= g.H && x0 + g.TW <= g.Wd && g.IMGS * TPI == 64;
  const bool plain = full && g.ksplit == 1 && !g.res && g.vec4 && (g.N & 3) == 0 && !act.tanh_;
  float* S = lds;
  constexpr int NITEM = 64 * 4 * NF;  // (tile, 4 outputs) items per pass
  // the passes and items run as rolled loops: the epilogue executes once per block, so its code
  // comes cold from L2 -- compact code costs fewer instruction-fetch round trips
#pragma unroll 1
  for (int c = 0; c < 2; ++c) {
    lds_barrier();  // c = 0: every wave is done with the stages; c = 1: with pass 0's S
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x0v = acc[f][0][j][r], x1v = acc[f][1][j][r];
          const float p = BP_ == 0 ? (c == 0 ? x0v + x1v : x1v) : (c == 0 ? x0v : (-x0v) - x1v);
          const int tile = 16 * f + 4 * lq + r, n = 16 * j + lr;
          S[(wave * 64 + tile) * NN + n] = p;
        }
    lds_barrier();
    if (IDF_WK_STAMPS && c == 0) stamp[3] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < (NITEM + kThreads - 1) / kThreads; ++it) {
      const int e = tid + kThreads * it;
      if (IDF_WK_ABLATE & 128) break;  // timing-only: no finisher
      if (NITEM % kThreads != 0 && e >= NITEM) break;
      const int tile = e / (4 * NF), k4 = e - tile * (4 * NF);
      const int img = udiv_s(tile, TPI);
      const int rem = tile - img * TPI;
      const int ty = udiv_s(rem, TTW), tx = rem - ty * TTW;
      const int nl = 4 * k4, n0 = nf0 * 16 + nl;
      if (!(img < g.IMGS && b0 + img < g.B && n0 < g.N)) continue;
      w4 Q[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const w4 p0 = *(const w4*)(S + ((2 * a) * 64 + tile) * NN + nl);
        const w4 p1 = *(const w4*)(S + ((2 * a + 1) * 64 + tile) * NN + nl);
        Q[a] = p0 + p1;
      }
      const int x = x0 + 2 * tx + c;
#pragma unroll 1
      for (int r = 0; r < 2; ++r) {
        const int y = y0 + 2 * ty + r;
        w4 yv;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          yv[kk] = (r == 0 ? (Q[0][kk] + Q[1][kk]) + Q[2][kk] : (Q[1][kk] - Q[2][kk]) - Q[3][kk]) * g.yscale;
        const int64_t qp = ((int64_t)img * g.H + y) * g.Wd + x;  // relative to the block's image 0
        if (plain) {
          const w4 bv = *(const w4*)(btab + bias_class(y, x, g.H, g.Wd) * NN + nl);
          w4 v;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            v[kk] = act(yv[kk] + bv[kk]);
            out_ok = out_ok && fabsf(v[kk]) < kGuardOut;
          }
          if (IDF_WK_ABLATE & 64) {
            if (v[0] == 12345.f) obase[0] = v[1];
          } else {
            *(w4*)(obase + qp * g.ldo + n0) = v;
          }
          continue;
        }
        if (!(y < g.H && x < g.Wd)) continue;
        if (g.ksplit > 1) {
          float* dst = pbase + qp * g.ldp + n0;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            if (n0 + kk < g.N) dst[kk] = yv[kk];
          continue;
        }
        const w4 bv = *(const w4*)(btab + bias_class(y, x, g.H, g.Wd) * NN + nl);
        w4 v;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) v[kk] = yv[kk] + bv[kk];
        if (rbase) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            if (n0 + kk < g.N) v[kk] = rbase[qp * g.ldr + n0 + kk] + v[kk];
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) v[kk] = act.tanh_ ? wact(v[kk], g.act, g.slope) : act(v[kk]);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) out_ok = out_ok && (n0 + kk >= g.N || fabsf(v[kk]) < kGuardOut);
        float* dst = obase + qp * g.ldo + n0;
        if (g.vec4 && n0 + 4 <= g.N) {
          *(w4*)dst = v;
        } else {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            if (n0 + kk < g.N) dst[kk] = v[kk];
        }
      }
    }
  }
  (void)A_;
  if (!out_ok && g.flag) atomicOr(g.flag, 1u);
  if (IDF_WK_STAMPS) stamp[5] = __builtin_amdgcn_s_memtime();
  if (IDF_WK_STAMPS) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp[4] = __builtin_amdgcn_s_memtime();
    if (lane == 0 && g.part) {
      float* o = g.part + ((int64_t)blockIdx.x * 8 + wave) * 8;
      for (int k = 0; k < 4; ++k) o[k] = (float)(stamp[k + 1] - stamp[k]);
      o[4] = (float)(stamp[4] - stamp[5]);  // the final store drain
    }
  }
}

// split-K: fixed-order sum of the partial slabs, then bias / residual / activation / guard
__global__ void __launch_bounds__(256) conv3_wk_reduce_kernel(Args g) {
  const int64_t P = (int64_t)g.B * g.H * g.Wd;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * g.N) return;
  const int64_t p = i / g.N;
  const int n = (int)(i - p * g.N);
  float s = g.part[p * g.ldp + n];
  for (int k = 1; k < g.ksplit; ++k) s = s + g.part[((int64_t)k * P + p) * g.ldp + n];
  const int64_t rem = p % ((int64_t)g.H * g.Wd);
  const int y = (int)(rem / g.Wd), x = (int)(rem % g.Wd);
  float bsum;
  if (!g.vtap) {
    bsum = g.b3[n];
  } else if (y >= 1 && y <= g.H - 2 && x >= 1 && x <= g.Wd - 2) {
    bsum = g.bfull[n];
  } else {
    bsum = g.b3[n];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ny = y + tap / 3 - 1, nx = x + tap % 3 - 1;
      if (ny >= 0 && ny < g.H && nx >= 0 && nx < g.Wd) bsum = bsum + g.vtap[tap * g.ldv + n];
    }
  }
  float v = s + bsum;
  if (g.res) v = g.res[p * g.ldr + n] + v;
  v = wact(v, g.act, g.slope);
  if (g.flag && !(fabsf(v) < kGuardOut)) atomicOr(g.flag, 1u);
  g.out[p * g.ldo + n] = v;
}

}  // namespace wk
}  // namespace idf

using namespace idf;

// Geometries the wk kernel takes: every Winograd geometry except the packed-small-image stage
// (config 4's 4x4 / 2x2 levels), which stays on conv3_wino.hip's wx3 kernel.
extern "C" int idf_conv3x3_wk_supported(int32_t H, int32_t W) {
  const WinoPlan pl = wino_plan(H, W, 1, 1);
  return pl.ok && !pl.big;
}

extern "C" int64_t idf_conv3x3_wk_workspace(int32_t B, int32_t H, int32_t W, int32_t C, int32_t N) {
  const WinoPlan pl = wino_plan(H, W, (C + 31) / 32, N);
  if (!pl.ok || pl.big || pl.ksplit <= 1) return 0;
  return (int64_t)pl.ksplit * B * H * W * ((N + 3) / 4 * 4);
}

static int wk_launch(void* stream, int32_t B, int32_t H, int32_t W, int32_t C, const float* x,
                     int64_t ld_x, int64_t slab_stride, const uint16_t* u, int32_t nft, float yscale, const float* b3,
                     const float* vtap, int32_t ldv, const float* bfull, int32_t N, float* out,
                     int64_t ld_out, const float* res, int64_t ld_res, int32_t act, float slope,
                     uint32_t* flag, int32_t check_in, float* workspace, int64_t workspace_floats) {
  using namespace idf::wk;
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  if (C <= 0 || (C & 3) || (ld_x & 3) || !u || !out || !b3) return IDF_ERR_ARG;
  const int nf_total = (N + 15) / 16;
  if (nft < nf_total) return IDF_ERR_ARG;
  const int NF = nf_total <= 3 ? nf_total : (nf_total % 3 == 0 ? 3 : (nf_total % 2 == 0 ? 2 : 1));
  Args g = {};
  g.X = x; g.ldx = ld_x; g.slab_stride = slab_stride; g.C = C; g.U = u; g.nslab = (C + 31) / 32; g.nft = nft; g.N = N;
  g.B = B; g.H = H; g.Wd = W;
  const WinoPlan pl = wino_plan(H, W, g.nslab, N);
  if (!pl.ok || pl.big) return IDF_ERR_UNSUPPORTED;
  // halo offsets are 32-bit with out-of-range markers at 1 and 2 GiB: the block's images must
  // span < 1 GiB, the channels < 1 GiB of bytes
  if ((int64_t)pl.IMGS * H * W * ld_x * 4 >= (int64_t)kChanOut || (int64_t)C * 4 >= (int64_t)kChanOut)
    return IDF_ERR_UNSUPPORTED;
  if ((int64_t)16 * g.nslab * nft * 2048 >= (int64_t)kInvalid) return IDF_ERR_UNSUPPORTED;
  g.IMGS = pl.IMGS; g.TH = pl.TH; g.TW = pl.TW; g.ksplit = pl.ksplit;
  g.tiles_b = (B + pl.IMGS - 1) / pl.IMGS;
  g.tiles_y = (H + pl.TH - 1) / pl.TH;
  g.tiles_x = (W + pl.TW - 1) / pl.TW;
  g.n_tiles = (nf_total + NF - 1) / NF;
  if (g.n_tiles * NF > nft) return IDF_ERR_ARG;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out; g.res = res; g.ldr = ld_res;
  g.yscale = yscale; g.flag = flag;
  g.vec4 = ((uintptr_t)out % 16 == 0) && (ld_out % 4 == 0);
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  if (res && ld_res < N) return IDF_ERR_ARG;
  if (IDF_WK_STAMPS) g.part = workspace;
  if (pl.ksplit > 1) {
    g.ldp = (N + 3) / 4 * 4;
    if (!workspace || workspace_floats < (int64_t)pl.ksplit * B * H * W * g.ldp) return IDF_ERR_WORKSPACE;
    g.part = workspace;
  }
  const int64_t blocks = (int64_t)g.tiles_b * g.tiles_y * g.tiles_x * g.n_tiles * pl.ksplit;
  // the kernel's index maps use udiv_s (operands < 2^20)
  if (blocks >= (1 << 20) || (int64_t)(pl.ksplit + 1) * g.nslab >= (1 << 20)) return IDF_ERR_UNSUPPORTED;
  g.nblocks = (int)blocks;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)blocks), blk(kThreads);
  const int twc = NF == 3 && (pl.TW == 32 || pl.TW == 16 || pl.TW == 8) ? pl.TW : 0;
#define IDF_WK(nf, tw, chk) hipLaunchKernelGGL((conv3_wk_kernel<nf, tw, chk>), grid, blk, 0, s, g)
  if (NF == 3) {
    if (twc == 32) { if (check_in) IDF_WK(3, 32, true); else IDF_WK(3, 32, false); }
    else if (twc == 16) { if (check_in) IDF_WK(3, 16, true); else IDF_WK(3, 16, false); }
    else if (twc == 8) { if (check_in) IDF_WK(3, 8, true); else IDF_WK(3, 8, false); }
    else if (check_in) IDF_WK(3, 0, true);
    else IDF_WK(3, 0, false);
  } else if (NF == 2) {
    if (check_in) IDF_WK(2, 0, true); else IDF_WK(2, 0, false);
  } else {
    if (check_in) IDF_WK(1, 0, true); else IDF_WK(1, 0, false);
  }
#undef IDF_WK
  if (pl.ksplit > 1) {
    const int64_t n = (int64_t)B * H * W * N;
    hipLaunchKernelGGL(conv3_wk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
  }
  return idf_last_error();
}

extern "C" int idf_conv3x3_wk(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                              const float* x, int64_t ld_x, const uint16_t* u, int32_t nft,
                              float yscale, const float* b3, const float* vtap, int32_t ldv,
                              const float* bfull, int32_t N, float* out, int64_t ld_out,
                              int32_t act, float slope, uint32_t* d_flag, int32_t check_input,
                              float* workspace, int64_t workspace_floats) {
  return wk_launch(stream, B, H, W, C, x, ld_x, 0, u, nft, yscale, b3, vtap, ldv, bfull, N, out,
                   ld_out, nullptr, 0, act, slope, d_flag, check_input, workspace, workspace_floats);
}

extern "C" int idf_conv3x3_wk_res(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                                  const float* x, int64_t ld_x, const uint16_t* u, int32_t nft,
                                  float yscale, const float* bias, int32_t N, float* out,
                                  int64_t ld_out, const float* res, int64_t ld_res, int32_t act,
                                  float slope, uint32_t* d_flag, int32_t check_input,
                                  float* workspace, int64_t workspace_floats) {
  return wk_launch(stream, B, H, W, C, x, ld_x, 0, u, nft, yscale, bias, nullptr, 0, nullptr, N, out,
                   ld_out, res, ld_res, act, slope, d_flag, check_input, workspace, workspace_floats);
}

// experiment (tools/native wk_bench): the same conv over a slab-major input [C/32][P][32]
extern "C" int idf_conv3x3_wk_slabmajor(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                                        const float* x, int64_t slab_stride, const uint16_t* u,
                                        int32_t nft, float yscale, const float* b3,
                                        const float* vtap, int32_t ldv, const float* bfull,
                                        int32_t N, float* out, int64_t ld_out, int32_t act,
                                        float slope, uint32_t* d_flag, int32_t check_input,
                                        float* workspace, int64_t workspace_floats) {
  return wk_launch(stream, B, H, W, C, x, 32, slab_stride, u, nft, yscale, b3, vtap, ldv, bfull, N,
                   out, ld_out, nullptr, 0, act, slope, d_flag, check_input, workspace,
                   workspace_floats);
}
