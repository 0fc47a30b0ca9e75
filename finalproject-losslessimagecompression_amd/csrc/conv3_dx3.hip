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
// Output tiles are 16 x 16 "packed" pixels (dx3_plan): images a multiple of 16 wide tile one
// image; smaller images pack nbx x nby to a tile (imagenet64's 8 x 8 level: 2 x 2 images,
// config 4's 4 x 4 patches: 4 x 4), and widths that are neither (config 5's 23-wide patches)
// pack side by side in bands of nbx images, a tile crossing at most one image edge.  The LDS
// canvas of a tile holds each image's halo in its own SEGMENT with zero gutters, so a lane's
// 3 x 3 taps never see a neighbouring image: lane j reads canvas slot rowbase * PITCH +
// colbase(j) + tap, and the segment bases are chosen so colbase(j) = j (mod 8) -- every
// ds_read_b128 lane group of the fragment reads then still covers 16 distinct bank quads.
//
// Block = 8 waves (two per SIMD) = WR/2 tiles x NF*16 outputs (one of ngroup output groups);
// a wave owns WR output rows (WR 16-pixel B fragments) of one tile x NF fragments.  Per
// 16-channel slab the block stages into one of two LDS stages, by LDS-DMA issued a slab ahead:
//   * each tile's canvas as two planes, xh [slots][16] and xl [slots][16] (32 B per slot);
//   * the slab's weights in A-fragment order, wh [9 taps][NF][16 out][16 ch] then wl.
// One barrier per slab.  A pixel fragment (16 pixels of one canvas row, one tap column) is read
// once and feeds the 3 output rows x NF fragments that use it.
//
// Split K (nchunk > 1; dx3_plan: the 8 x 8 level, whose 64 tiles per 256 images cannot fill
// the chip): the slabs are cut into nchunk fixed chunks, one block each; a block writes its
// raw accumulators to a partial buffer, and the block that finishes a tile's last chunk (an
// agent-scope counter per tile, self-resetting) sums the chunks in chunk order and runs the
// epilogue -- no reduce launch.  Each output is one fixed-order sum (slabs within a chunk, the
// chunks left to right, the tap/product order below) whose order depends on (H, W, C) only:
// batch- and tile-invariant, so encoder and decoder agree bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "idf_cdf.h"
#include "idf_codec_internal.h"
#include "wino_common.h"

#pragma clang fp contract(off)

namespace idf {

typedef float d4 __attribute__((ext_vector_type(4)));
typedef _Float16 e4 __attribute__((ext_vector_type(4)));
typedef _Float16 e8 __attribute__((ext_vector_type(8)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));

struct Dx3Args {
  const uint16_t* xs;  // split features [nslab_xs][2: hi, lo][P][16] f16 bits (bf16 kernel:
                       // the block's bf16 shadow [P][16 nslab_xs], pixel-major)
  int64_t P;           // pixels of the batch (B * H * W)
  int64_t xs_pix, xs_slab, xs_bytes;  // bytes: pixel to pixel, slab to slab, the whole buffer
  int32_t nslab_xs;    // slabs the split buffer holds
  int32_t C;           // input channels (slabs read: ceil(C / 16))
  const uint16_t* Wt;  // [nslab][ngroup][2: hi, lo][9 taps][NF][16 out][16 ch] f16 of w * 2^k
  int32_t nslab, ngroup;
  int32_t N;
  int32_t B, H, Wd;
  // packed tiling (dx3_plan)
  int32_t nbx, nby;     // images per band across / down
  int32_t tiles_x, tiles_y, ntiles, nblk_tiles;
  int32_t ch;           // canvas rows
  int32_t seg, segw, nseg;  // segment stride and width (slots), segments per canvas
  int32_t gut, wp, hp;  // 1: gutter packing -- images at pitch wp = W + 1 across, hp = H + 1
                        // down, the zero row / column between two images shared by both
  int32_t tilew, xskip; // packed columns per tile (16; 24 with xskip) and xskip: 2-wide images,
                        // lane j at image j / 2's column j % 2 (no lane on a gutter column)
  // split K
  int32_t nchunk, chunk_slabs;
  float* part;          // [nblk_tiles][ngroup][nchunk][waves][WR][NF][64 lanes] d4
  uint32_t* ctr;        // [nblk_tiles][ngroup], zero at the launch, left zero
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
  // the DenseBlock head fused into the layer (IdfDx3Head; nh = 0: none)
  const float* hw;      // [nh][ldhw] fp32 head weights (padded channel coordinates)
  int32_t ldhw, nh;
  float* hacc;          // [P][16] running head sums
  int32_t hlast, skip_f32, hmode, hn_mean;
  float* hout;
  int64_t hld_out;
  const float* hbase;
  int64_t hld_base;
  float *hmean, *hlogs, *hscale;
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
// timing-only block timeline (IDF_DX3_TL=1 builds): per block, wave 0 lane 0 -- s_memrealtime
// (100 MHz, chip-wide) at entry, after the bias table, after slab 0's barrier, at the loop's end,
// after the split-K hand-off (last block only) and at the end; read back with idf_dx3_timeline
#ifndef IDF_DX3_TL
#define IDF_DX3_TL 0
#endif
#if IDF_DX3_TL
__device__ unsigned long long g_dx3_tl[4096][8];
#define DX3_TL(j)                                                                          \
  do {                                                                                    \
    if (tid == 0 && blockIdx.x < 4096) g_dx3_tl[blockIdx.x][(j)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define DX3_TL(j) do { } while (0)
#endif
#ifndef IDF_DX3_KSPLIT
#define IDF_DX3_KSPLIT 4  // chunks of the split-K levels (timing A/B builds only: changes bits)
#endif
// split-K chunks at 16 x 16 (timing A/B builds only: changes bits)
#ifndef IDF_DX3_KSPLIT16
#define IDF_DX3_KSPLIT16 1
#endif
// two tiles per block from this many tiles up (every CU gets a block; timing A/B builds only)
#ifndef IDF_DX3_TWO_MIN
#define IDF_DX3_TWO_MIN 512
#endif
// 1: one tile per block at every geometry (timing A/B of the two block shapes)
#ifndef IDF_DX3_FORCE1
#define IDF_DX3_FORCE1 0
#endif

// the split slab schedule (see the kernel): 0 (the library's) [wh ; wh] . [xh | xl] per tap, 42
// weight-fragment reads a slab and wave; 1 pairs the hi weights' taps as the lo weights' are, 30
// reads at the same MFMA count -- L0 c = 496 1.4% faster, but its other summation order moves one
// teacher-forced coupling rounding of the imagenet64 B = 16 fixture from level 2 to level 1, so
// the latents differ from the reference's in 0 / 4 / 50 places instead of 0 / 0 / 0
// (profiles/r05/pairs/); a timing A/B build only
#ifndef IDF_DX3_PAIRS
#define IDF_DX3_PAIRS 0
#endif
// wave priority schedule in the split slab loop (timing A/B builds only; 0: none)
#ifndef IDF_DX3_PRIO
#define IDF_DX3_PRIO 0
#endif
#ifndef IDF_DX3_PRIO_K
#define IDF_DX3_PRIO_K 4
#endif
// mixed rows per wave in the two-tile split-f16 blocks (timing A/B builds only; dx3_block): 1 the
// older wave of a SIMD takes WR + 1 rows of its half tile, 2 WR - 1
#ifndef IDF_DX3_MIX
#define IDF_DX3_MIX 0
#endif
// waves per block (timing A/B: 16 = four per SIMD at 2 rows per wave)
#ifndef IDF_DX3_WAVES
#define IDF_DX3_WAVES 8
#endif
constexpr int kDxWaves = IDF_DX3_WAVES;
constexpr int kDxThreads = 64 * kDxWaves;
constexpr uint32_t kDxInvalid = 0xFFFFFFF0u;
// offset of an out-of-image halo slot: the halo DMA addresses one slab per buffer resource and
// a slab is under 2 GiB (checked on the host), so kDxOff lies past its end and the load returns
// zeros
constexpr uint32_t kDxOff = 0x80000000u;
// the split-f16 range guard on stored outputs: |y| < 8192, as wx3 (|x| < 32768 on block inputs
// is checked where the inputs are split, idf_dx3_split_cols)
constexpr float kDxInGuard = 32768.0f;
constexpr float kDxOutGuard = 8192.0f;

// The canvas shapes the library instantiates: (row pitch in slots, plane size in KiB).  18 /
// 11: one 16-wide tile of one image (18 x 18 halo); 10 / 13: 8-wide images, two segments of
// 10 x 20 (2 x 2 images of 8 x 8); 6 / 19: 4-wide images, four segments of 6 x 24; 26 / 17:
// widths with one image edge inside a tile (two segments side by side, the second 8 slots past
// the first's last lane: colbase = j mod 8); 25 / 15: 2-wide images gutter packed with every
// lane on an image column (xskip: 25 x 18 slots).
template <int NF, int WR, int PITCH, int PLANE_KIB, bool BF>
struct Dx3Lds {
  static constexpr int T = WR * kDxWaves / 16;     // tiles per block
  static constexpr int HR = WR + 2;                // canvas rows a wave reads
  // steps per slab (the schedule)
  static constexpr int NS = BF ? 2 * HR - 1 : IDF_DX3_PAIRS ? 3 * HR - 1 + 2 * WR : 5 * HR - 1;
  static constexpr int NPL = BF ? 1 : 2;           // planes per tile canvas: xh, xl / x
  static constexpr int PLANE = PLANE_KIB * 1024;   // one plane (xh or xl) of a tile's canvas
  static constexpr int SLOTS = PLANE / 32;
  static constexpr int WOFF = T * NPL * PLANE;     // weights within a stage
  static constexpr int WPART = 9 * NF * 512;       // one part (wh or wl) of a slab's weights
  // whole 1-KiB DMA pieces (the bf16 weights padded to them in HBM: packing.dxb_weights)
  static constexpr int WST = BF ? (WPART + 1023) / 1024 * 1024 : 2 * WPART;
  static constexpr int STAGE = WOFF + WST;
  static constexpr int ZOFF = 2 * STAGE;           // NF * 512 B of zeros (the odd tap's pair)
  static constexpr int BOFF = ZOFF + NF * 512;     // bias table [16 classes][NF * 16] f32
  static constexpr int HOFF = BOFF + 16 * NF * 16 * 4;  // fused head weights [16][NF * 16] f32
  static constexpr int FOFF = HOFF + 16 * NF * 16 * 4;  // the split-K "last block" flag
  static constexpr int BYTES = FOFF + 16;
  static constexpr int HPIECES = T * NPL * PLANE_KIB;      // halo DMA pieces per slab
  static constexpr int WPIECES = WST / 1024;               // weight pieces per slab
  // piece slots per wave: halo slots [0, PH) then weight slots [PH, PPW); slot i of wave w is
  // piece w + 8 i of its kind (some slots of the last row of each kind are empty)
  static constexpr int PH = (HPIECES + kDxWaves - 1) / kDxWaves;
  static constexpr int PPW = PH + (WPIECES + kDxWaves - 1) / kDxWaves;
};

typedef __attribute__((address_space(3))) void* dx_lds_ptr_t;

// f(integral_constant<int, T>) for T = 0, 1, ... in order: a compile-time unrolled schedule
template <typename F, int... T>
__device__ __forceinline__ void dx_unroll(F&& f, std::integer_sequence<int, T...>) {
  (f(std::integral_constant<int, T>{}), ...);
}

// A tile's place in the packed layout: band (nbx x nby images), first packed column u0 and row
// u0y; with segments, the image column ix0 / row iy0 they fall in, the first column's image x
// (xf0) and the canvas row 0's vertical coordinate vy0 (canvas row cr holds packed vertical
// coordinate vy0 + cr, image row vy / (H + 2)).
struct DxTile {
  int band, u0, ix0, xf0, u0y, iy0, vy0;
};

__device__ __forceinline__ DxTile dx_tile(const Dx3Args& g, int tile) {
  DxTile t;
  int q = tile;
  const int tx = q - udiv_s(q, g.tiles_x) * g.tiles_x;
  q = udiv_s(q, g.tiles_x);
  const int ty = q - udiv_s(q, g.tiles_y) * g.tiles_y;
  t.band = udiv_s(q, g.tiles_y);
  t.u0 = g.tilew * tx;
  t.ix0 = udiv_s(t.u0, g.Wd);
  t.xf0 = t.u0 - t.ix0 * g.Wd;
  t.u0y = 16 * ty;
  t.iy0 = udiv_s(t.u0y, g.H);
  if (t.iy0 > g.nby - 1) t.iy0 = g.nby - 1;
  t.vy0 = t.u0y + 2 * t.iy0;
  return t;
}

// One DenseLayer's own parameters (the rest of Dx3Args is the block's): a single-layer launch
// takes them from Dx3Args, the fused DenseBlock kernel (conv3_dx3_block_kernel) from its layer
// list.  nchunk / chunk_slabs: the layer's split-K cut (dx3_launch_shape; the fused kernel runs
// only geometries without one).
struct Dx3Layer {
  const uint16_t* Wt;
  const float *b3, *vtap, *bfull;
  float* out;
  float yscale;
  int32_t C, nslab, nchunk, chunk_slabs, hlast;
};

// The fused DenseBlock (conv3_dx3_block_kernel): every layer of a block in one launch, one
// workgroup per tile, for geometries whose tiles hold whole images (no halo crosses a tile:
// dx3_self_contained), so a tile's layers depend only on its own earlier layers.  With a fused
// head the running sums stay in registers from the head init (hx: the block input, fp32 rows of
// hld_x floats, hc0 channels; hb: the head bias) to the last layer's epilogue.
constexpr int kDxMaxLayers = 16;
struct Dx3MLArgs {
  Dx3Layer layer[kDxMaxLayers];
  int32_t nlayers, hc0;
  const float* hx;
  int64_t hld_x;
  const float* hb;
};

// The epilogue's two LDS tables: the bias table [16 border classes][NF * 16] (stage_bias's
// values: b3 plus the in-image taps' share of the folded 1x1 bias) and the fused head's weights
// on this layer's outputs [16][NF * 16] (zeros past nh and past N).  load() issues every global
// load at once (one memory round trip); the kernel calls it after the first slab's barrier and
// store() after the second's, so the loads overlap the first slab's MFMAs instead of holding the
// first barrier back (a slab barrier waits for every outstanding load, these included).
template <int NF>
struct Dx3Tables {
  static constexpr int NN = NF * 16, NE = 16 * NN;  // outputs of the group; entries per table
  static constexpr int HPER = (NE + kDxThreads - 1) / kDxThreads;  // head entries per thread
  float bt[11];     // thread n < NN: output n's b3, 9 tap biases and full bias (all 16 classes)
  float ht[HPER];   // head entries tid, tid + kDxThreads, ...

  __device__ __forceinline__ void load(const Dx3Args& g, const Dx3Layer& Ly, int grp, int tid) {
    const int n = grp * NN + tid, nc = n < g.N ? n : 0;
    if (tid < NN) {
      bt[0] = Ly.b3[nc];
      if (Ly.vtap) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) bt[1 + tap] = Ly.vtap[tap * g.ldv + nc];
        bt[10] = Ly.bfull[nc];
      }
    }
    if (g.nh > 0) {
#pragma unroll
      for (int i = 0; i < HPER; ++i) {
        const int e = tid + i * kDxThreads, o = e / NN, hn = grp * NN + e - o * NN;
        if (e < NE) ht[i] = g.hw[(int64_t)(o < g.nh ? o : 0) * g.ldhw + Ly.C + (hn < g.N ? hn : 0)];
      }
    }
  }

  __device__ __forceinline__ void store(float* btab, float* htab, const Dx3Args& g,
                                        const Dx3Layer& Ly, int grp, int tid) const {
    if (tid < NN) {
      const int n = grp * NN + tid;
#pragma unroll
      for (int cls = 0; cls < 16; ++cls) {
        float v = bt[0];
        if (Ly.vtap) {
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) {
            const int dy = tap / 3 - 1, dx = tap % 3 - 1;
            const bool ok = !((dy < 0 && (cls & 1)) || (dy > 0 && (cls & 2)) ||
                              (dx < 0 && (cls & 4)) || (dx > 0 && (cls & 8)));
            v = ok ? v + bt[1 + tap] : v;
          }
          v = cls == 0 ? bt[10] : v;
        }
        btab[cls * NN + tid] = n < g.N ? v : 0.0f;
      }
    }
    if (g.nh > 0) {
#pragma unroll
      for (int i = 0; i < HPER; ++i) {
        const int e = tid + i * kDxThreads, o = e / NN, hn = grp * NN + e - o * NN;
        if (e < NE) htab[e] = (o < g.nh && hn < g.N) ? ht[i] : 0.0f;
      }
    }
  }
};

// One launch's work: ML = false, one layer (conv3_dx3_kernel: a block = a chunk of the slabs of
// one output group of T tiles); ML = true, every layer of a DenseBlock for one tile
// (conv3_dx3_block_kernel, T = 1, one output group, no split K).
// WRW: the output rows of this wave (WR: of the block layout's waves).  WRW != WR ("mixed
// rows", IDF_DX3_MIX): the two waves of a SIMD share the 8 rows of one half tile unequally, the
// older (waves 0-3) WR + 1 rows, the younger WR - 1 -- the older wave runs ahead at the MFMA
// pipe (the hardware favours it) and waits at the slab barrier for the younger otherwise
// (profiles/r05/dma_issue/stamps.log).  Rows per wave change no output's summation order.
template <int NF, int WR, int PITCH, int PLANE_KIB, bool BF, bool ML, int WRW = WR>
__device__ __forceinline__ void dx3_block(const Dx3Args& g, const Dx3MLArgs* ml, char* lds) {
  using L = Dx3Lds<NF, WR, PITCH, PLANE_KIB, BF>;
  constexpr bool MIX = WRW != WR;
  constexpr int T = L::T, HR = WRW + 2;
  constexpr int NS = BF ? 2 * HR - 1 : IDF_DX3_PAIRS ? 3 * HR - 1 + 2 * WRW : 5 * HR - 1;
  static_assert(!MIX || (T == 2 && kDxWaves == 8 && !ML && (WRW == WR + 1 || WRW == WR - 1)),
                "mixed rows: two tiles of two SIMD pairs, per-layer launches");
  static_assert(L::WST % 1024 == 0, "weight stage must be whole 1-KiB DMA pieces");
  static_assert(L::BYTES <= 160 * 1024, "LDS");
  static_assert(HR >= 3, "the A-fragment reads of a phase take its last three steps");
  static_assert(IDF_DX3_DMAS == 0 || IDF_DX3_DMA0 + IDF_DX3_STAG + (L::PPW - 1) * IDF_DX3_DMAS < NS,
                "every DMA piece of a slab is issued within the slab's steps");
  int* last_flag = (int*)(lds + L::FOFF);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // block -> (chunk, output group, tile block), chunk-major: the blocks of one XCD (a
  // contiguous range, xcd_contiguous) mostly share a chunk and group, i.e. their weights
  const int bid = xcd_contiguous(blockIdx.x, gridDim.x);
  const int per_chunk = g.ngroup * g.nblk_tiles;
  const int chunk = udiv_s(bid, per_chunk);
  const int rem = bid - chunk * per_chunk;
  const int grp = udiv_s(rem, g.nblk_tiles);
  const int tb = rem - grp * g.nblk_tiles;
  // the wave's tile and first output row
  // (mixed rows: SIMD s = wave & 3 holds half tile s & 1 of tile s >> 1, its older wave the
  // first WR + 1 rows)
  const int tw = MIX ? (wave & 3) >> 1 : wave / (kDxWaves / T);
  constexpr int WR_OLD = IDF_DX3_MIX == 2 ? WR - 1 : WR + 1;  // the older wave's rows (MIX)
  const int r0 = MIX ? 2 * WR * (wave & 1) + ((wave & 4) ? WR_OLD : 0) : WR * (wave % (kDxWaves / T));
  d4 hreg[WRW];  // ML: the fused head's running sums, registers across the layers
  const int nlayers = ML ? ml->nlayers : 1;
  for (int li = 0; li < nlayers; ++li) {
  // (ML) the block's indices passed through an opaque asm: everything derived from them below
  // (DMA plan, canvas position, fragment offsets) is recomputed in every layer -- held across
  // the layer loop it doubled the kernel's VGPRs and spilled
  int tid_o = tid, lane_o = lane, wave_o = wave, tb_o = tb, tw_o = tw, r0_o = r0, grp_o = grp,
      chunk_o = chunk;
  if constexpr (ML) {
    asm volatile("" : "+v"(tid_o), "+v"(lane_o), "+v"(wave_o), "+v"(tb_o), "+v"(tw_o), "+v"(r0_o),
                 "+v"(grp_o), "+v"(chunk_o));
    wave_o = __builtin_amdgcn_readfirstlane(wave_o);  // (uniform again)
    tb_o = __builtin_amdgcn_readfirstlane(tb_o);
    tw_o = __builtin_amdgcn_readfirstlane(tw_o);
    r0_o = __builtin_amdgcn_readfirstlane(r0_o);
    grp_o = __builtin_amdgcn_readfirstlane(grp_o);
    chunk_o = __builtin_amdgcn_readfirstlane(chunk_o);
  }
  const int tid = tid_o, lane = lane_o, wave = wave_o, tb = tb_o, tw = tw_o, r0 = r0_o,
            grp = grp_o, chunk = chunk_o;
  const int lz = 0;
  Dx3Layer Ly;
  if constexpr (ML) {
    Ly = ml->layer[li];
  } else {
    Ly = Dx3Layer{g.Wt, g.b3, g.vtap, g.bfull, g.out, g.yscale, g.C, g.nslab, g.nchunk,
                  g.chunk_slabs, g.hlast};
  }
  const int tile = tb * T + tw + lz;

  // ---- DMA plan: piece k = wave + 8 i of each slab.  Halo pieces k < HPIECES: tile k /
  // (2 PLANE_KIB), plane (k / PLANE_KIB) % 2, canvas slots 32 (k % PLANE_KIB) .. +31 (lane:
  // slot + lane / 2, 8 channels (lane & 1)); weight pieces: 1 KiB of the slab's group weights.
  const int64_t plane_b = g.P * 32;                      // bytes of one plane of one slab
  // the halo DMA addresses one slab at a time (a buffer resource per slab: 32-bit offsets
  // within a slab, so the whole copy may exceed 4 GiB -- config 5's 2048-patch batches)
  const int xs_rec = (int)(g.xs_slab < (int64_t)kDxInvalid ? g.xs_slab : (int64_t)kDxInvalid);
  // Per slot: the source byte offset of slab 0 (halo: per lane; an out-of-image slot gets
  // kDxOff, which stays past the buffer's end for every slab -- the buffer returns zeros, no
  // select in the loop) or within a slab (weights); the LDS offset within a stage; whether the
  // slot holds a piece (wave-uniform).  The kind of slot i is a compile-time fact, so a DMA in
  // the loop is an address add, an M0 add and the load -- no per-piece branching.
  uint32_t pbase[L::PPW];
  int plo[L::PPW];
  bool pok[L::PPW];
#pragma unroll
  for (int i = 0; i < L::PPW; ++i) {
    const bool hk = i < L::PH;
    const int k = wave + kDxWaves * (hk ? i : i - L::PH);
    pok[i] = k < (hk ? L::HPIECES : L::WPIECES);
    pbase[i] = kDxOff;
    plo[i] = 0;
    if (hk && pok[i]) {
      const int t = k / (L::NPL * PLANE_KIB), pl = (k / PLANE_KIB) % L::NPL, pi = k % PLANE_KIB;
      plo[i] = (t * L::NPL + pl) * L::PLANE + pi * 1024;
      const int slot = 32 * pi + (lane >> 1);
      const int tt = tb * T + t;
      if (tt < g.ntiles) {
        const DxTile dt = dx_tile(g, tt);
        // canvas slot -> image (ix, iy) of the band and pixel (x, y)
        int ix, x, iy, y;
        bool ok;
        if (g.gut) {  // one 18 x 18 canvas of packed pixels; gutters and edges read zero
          const int cr = slot / PITCH, cc = slot - cr * PITCH;
          const int u = dt.u0 - 1 + cc, uy = dt.u0y - 1 + cr;
          ix = u >= 0 ? udiv_s(u, g.wp) : 0;
          x = u >= 0 ? u - ix * g.wp : -1;
          iy = uy >= 0 ? udiv_s(uy, g.hp) : 0;
          y = uy >= 0 ? uy - iy * g.hp : -1;
          ok = cr < g.ch && cc < g.segw;
        } else {  // canvas slot -> (segment, canvas row, segment column)
          const int sk = g.seg ? udiv_s(slot, g.seg) : 0;
          const int rr = slot - sk * g.seg;
          const int cr = rr / PITCH, cc = rr - cr * PITCH;
          ok = sk < g.nseg && cc < g.segw && cr < g.ch;
          ix = dt.ix0 + sk;
          x = (sk ? 0 : dt.xf0) - 1 + cc;
          const int vy = dt.vy0 + cr;
          iy = udiv_s(vy, g.H + 2);
          y = vy - iy * (g.H + 2) - 1;
        }
        const int b = (dt.band * g.nby + iy) * g.nbx + ix;
        ok = ok && x >= 0 && x < g.Wd && ix < g.nbx && y >= 0 && y < g.H && iy < g.nby && b < g.B;
        if (ok)
          pbase[i] = (uint32_t)(pl * plane_b + ((((int64_t)b * g.H + y) * g.Wd + x) * g.xs_pix) + (lane & 1) * 16);
      }
    } else if (!hk && pok[i]) {
      plo[i] = L::WOFF + k * 1024;
      pbase[i] = (uint32_t)(grp * L::WST + k * 1024 + lane * 16);
    }
  }
  DX3_TL(0);
  for (int e = tid; e < NF * 512 / 16; e += kDxThreads) *(d4*)(lds + L::ZOFF + 16 * e) = d4{0.f, 0.f, 0.f, 0.f};
  DX3_PHASE(0, __builtin_amdgcn_s_memtime());
  DX3_PHASE(4, __builtin_amdgcn_s_memrealtime());

  // ---- the wave's canvas position: lane j's column base (gutter packing: j; segments: its
  // segment's base + its offset in the segment, = j mod 8) and the wave's first canvas row
  // (segments: its rows lie in one image)
  const int j = lane & 15, q = lane >> 4;
  const DxTile dt = dx_tile(g, tile < g.ntiles ? tile : 0);
  const int jx = g.xskip ? 3 * (j >> 1) + (j & 1) : j;  // lane j's packed column in the tile
  const int uj = dt.u0 + jx;
  const int pw = g.gut ? g.wp : g.Wd;
  const int ixj = udiv_s(uj, pw);             // lane j's image column in the band
  const int xj = uj - ixj * pw;               // and its x (gutter packing: W = the gutter)
  const int kj = ixj - dt.ix0;                // its segment
  const int colb = g.gut ? jx : kj * g.seg + (kj ? j - (ixj * g.Wd - dt.u0) : j);
  const int uyw = dt.u0y + r0;
  int iyw = udiv_s(uyw, g.H);
  if (iyw > g.nby - 1) iyw = g.nby - 1;
  const int rowb = g.gut ? r0 : uyw + 2 * iyw - dt.vy0;  // canvas row of the wave's halo row 0

  // ---- fragment read offsets (bytes from a stage base).  B (pixels): lane (q = lane >> 4,
  // j = lane & 15) reads pixel j of a canvas row, 8 channels.  A (weights): output j, 8 channels.
  const int slot0 = rowb * PITCH + colb;
  const int tb0 = tw * L::NPL * L::PLANE;  // the wave's tile planes
  // [xh | xl] at (canvas row r0 + h, column j + dx): q 0,1 hi plane chunk q, q 2,3 lo plane chunk q-2
  const int oP = tb0 + (q >> 1) * L::PLANE + slot0 * 32 + (q & 1) * 16;
  // [xh(h, dx 0) | xh(h, dx 1)]
  const int oF = tb0 + slot0 * 32 + (q & 1) * 16 + (q >> 1) * 32;
  // [xh(h, dx 2) | xh(h + 1, dx 2)]
  const int oG = tb0 + slot0 * 32 + (q & 1) * 16 + 64 + (q >> 1) * PITCH * 32;
  // [wh(tap) ; wh(tap)] at tap t, fragment n: + (t * NF + n) * 512
  const int oAH = L::WOFF + j * 32 + (q & 1) * 16;
  // [wl(dy, 0) ; wl(dy, 1)]: + (3 dy * NF + n) * 512
  constexpr int WLO = BF ? 0 : L::WPART;  // the wl part (bf16 kernel: the only part)
  const int oAF = L::WOFF + WLO + j * 32 + (q & 1) * 16 + (q >> 1) * NF * 512;
  // [wl(0, 2) ; wl(1, 2)]: + n * 512
  const int oAG = L::WOFF + WLO + 2 * NF * 512 + j * 32 + (q & 1) * 16 + (q >> 1) * 3 * NF * 512;
  // [0 ; wl(2, 2)]: + n * 512; lanes q < 2 read the zero block (outside the stages)
  const int oAO = L::WOFF + WLO + 8 * NF * 512 + j * 32 + (q & 1) * 16;
  // [wh(dy, 0) ; wh(dy, 1)]: + (3 dy * NF + n) * 512, and [wh(0, 2) ; wh(1, 2)]: + n * 512
  const int oAHF = L::WOFF + j * 32 + (q & 1) * 16 + (q >> 1) * NF * 512;
  const int oAHG = L::WOFF + 2 * NF * 512 + j * 32 + (q & 1) * 16 + (q >> 1) * 3 * NF * 512;
  const bool zlane = q < 2;
  const char* zO = lds + L::ZOFF + j * 32 + (q & 1) * 16;

  // ---- ML: the wave's rows (as the epilogue's) and the fused head's running sums, kept in
  // registers across the layers from the head init on: per output o < n_head of pixel p,
  // bias[o] then c = 0 .. c0 - 1 in order, fmaf(w[o][c], x[p][c], .) -- dx3_head_init_kernel's
  // chain, so the sums carry the same bits as the split launches' HBM copy
  if constexpr (ML) if (li == 0) {
#pragma unroll
    for (int m = 0; m < WRW; ++m) hreg[m] = d4{0.f, 0.f, 0.f, 0.f};
    if (g.nh > 0) {
      const bool lane_ok0 = xj < g.Wd && ixj < g.nbx;
#pragma unroll
      for (int m = 0; m < WRW; ++m) {
        int iy = iyw, y = uyw + m - iyw * g.H;
        if (g.gut) {
          iy = udiv_s(uyw + m, g.hp);
          y = uyw + m - iy * g.hp;
        }
        const int img = (dt.band * g.nby + iy) * g.nbx + ixj;
        const bool ok = lane_ok0 && y < g.H && iy < g.nby && img < g.B;
        if (ok && 4 * q < g.nh) {
          const float* xr = ml->hx + (((int64_t)img * g.H + y) * g.Wd + xj) * ml->hld_x;
          d4 h;
#pragma unroll
          for (int i = 0; i < 4; ++i) h[i] = 4 * q + i < g.nh ? ml->hb[4 * q + i] : 0.0f;
          for (int c = 0; c < ml->hc0; c += 4) {
            const d4 xv = *(const d4*)(xr + c);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int o = 4 * q + i;
              if (o < g.nh) {
                const d4 wv = *(const d4*)(g.hw + (int64_t)o * g.ldhw + c);
#pragma unroll
                for (int k = 0; k < 4; ++k) h[i] = __builtin_fmaf(wv[k], xv[k], h[i]);
              }
            }
          }
          hreg[m] = h;
        }
      }
    }
  }

  // this block's slabs: a chunk of them (split launch), or all (ML: the chunks in order)
  const int s0 = ML ? 0 : chunk * Ly.chunk_slabs;
  const int s1 = ML ? Ly.nslab : min(Ly.nslab, s0 + Ly.chunk_slabs);
  const uint32_t wslab = (uint32_t)(g.ngroup * L::WST);  // weight bytes per slab
  const int64_t wbytes = (int64_t)Ly.nslab * wslab;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Ly.Wt, 0, (int)(wbytes < (int64_t)kDxInvalid ? wbytes : (int64_t)kDxInvalid), 0x00020000);
  // issue slot i's piece of slab s into stage st (a slab past the layer's reads zeros: the
  // loop's last slab issues its "next" DMA unconditionally, into a stage nothing reads again)
  auto dma = [&](int s, int st, int i) {
    if (!pok[i]) return;
    const bool halo = i < L::PH;
    if (halo ? (IDF_DX3_ABLATE & 1) : (IDF_DX3_ABLATE & 4)) return;
    // one call site for both kinds of piece (the LDS address formed from the __shared__ array
    // itself): the host pass of hipcc drops the kernel's launch stub otherwise
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)g.xs + (int64_t)s * g.xs_slab), 0, xs_rec, 0x00020000);
    const uint32_t off = pbase[i] + (halo ? 0u : (uint32_t)(s * g.ngroup) * (uint32_t)L::WST);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(halo ? xr : wr,
                                             (dx_lds_ptr_t)(lds + st * L::STAGE + plo[i]), 16,
                                             off, 0, 0, 0);
  };

  // the first slab's DMA first: the tables' dependent global loads then overlap its latency
  if (s1 > s0) {
#pragma unroll
    for (int i = 0; i < L::PPW; ++i) dma(s0, 0, i);
  }
  Dx3Tables<NF> tabs;  // loaded in the first slab, stored in the second (or after the loop)
  DX3_PHASE(1, __builtin_amdgcn_s_memtime());
  DX3_TL(1);


  d4 acc[WRW][NF];
#pragma unroll
  for (int m = 0; m < WRW; ++m)
#pragma unroll
    for (int n = 0; n < NF; ++n) acc[m][n] = d4{0.f, 0.f, 0.f, 0.f};

  auto rd = [](const char* p) { return *(const e8*)p; };
  auto mma = [](const e8& a, const e8& bb, d4& c) {
    if (IDF_DX3_ABLATE & 16) c[0] += (float)(a[0] * bb[0]);
    else if constexpr (BF)
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, bb),
                                                   c, 0, 0, 0);
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
  // the first three steps of the phase before it.  Two LDS stages: slab s reads stage
  // (s - s0) % 2; after the slab's barrier (every wave's DMA of slab s landed, every wave done
  // with slab s - 1) the waves DMA slab s + 1 into the other stage, one piece per step.
  constexpr int DB = IDF_DX3_DB, RB = DB + 1;
  e8 Bq[RB];
  e8 AS[2][3][NF];  // weight sets: P0 / P2 in 0, P1 / F in 1
  e8 AZ[2][NF];     // G: [wl(0,2) ; wl(1,2)] and [0 ; wl(2,2)]
  auto read_B = [&](const char* st, int t) -> e8 {
    if (t < 3 * HR) return rdB(st + oP + ((t % HR) * PITCH + t / HR) * 32);
    if (t < 4 * HR) return rdB(st + oF + (t - 3 * HR) * PITCH * 32);
    return rdB(st + oG + (t - 4 * HR) * PITCH * 32);
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
      if (m < 0 || m >= WRW) continue;
#pragma unroll
      for (int n = 0; n < NF; ++n) mma(A[dy][n], Bv, acc[m][n]);
    }
  };

  for (int s = s0; s < s1; ++s) {
    const char* cur = lds + ((s - s0) & 1) * L::STAGE;
    // this wave's DMA of slab s landed (vmcnt: LDS-DMA is a vector-memory load) and its LDS
    // writes -- the zero block, the epilogue tables -- are done (lgkmcnt); after the barrier every
    // wave's are, and every wave is done reading the other stage (slab s - 1).  The hardware
    // s_barrier waits for neither counter, and a wave's LDS write still in flight at the barrier
    // can land after another SIMD's wave has read the slot (the round-5 fused-head divergence:
    // tools/repro_lds/, DESIGN.md section 4 "LDS ordering audit").
    DX3_STAMP(s - s0, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (!(IDF_DX3_ABLATE & 8)) __builtin_amdgcn_s_barrier();
    DX3_STAMP(s - s0, 1);
    if (s == s0) DX3_TL(2);
    if (s == s0) tabs.load(g, Ly, grp, tid);
    if (s == s0 + 1) tabs.store((float*)(lds + L::BOFF), (float*)(lds + L::HOFF), g, Ly, grp, tid);
    __builtin_amdgcn_sched_barrier(0);
    const bool more = s + 1 < s1;
    const int nst = (s + 1 - s0) & 1;
    // slab s + 1's DMA at step t: one piece every IDF_DX3_DMAS steps from step IDF_DX3_DMA0
    auto dma_step = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int ds = IDF_DX3_DMAS > 0 ? IDF_DX3_DMAS : 1;
      auto dma_at = [&](auto dtc) {
        constexpr int dt_ = decltype(dtc)::value;
        if constexpr (IDF_DX3_DMAS == 0 && dt_ == 0) {  // the whole slab's pieces at once
          if (more) {
#pragma unroll
            for (int i = 0; i < L::PPW; ++i) dma(s + 1, nst, i);
          }
        } else if constexpr (IDF_DX3_DMAS > 0 && dt_ >= 0 && dt_ % ds == 0 && dt_ / ds < L::PPW) {
          if (more) dma(s + 1, nst, dt_ / ds);
        }
      };
      if (IDF_DX3_STAG == 0 || !(wave & 4)) dma_at(std::integral_constant<int, t - IDF_DX3_DMA0>{});
      else dma_at(std::integral_constant<int, t - IDF_DX3_DMA0 - IDF_DX3_STAG>{});
    };
    if constexpr (BF) {
      // bf16: one product per tap, the F / G phases of the split schedule on the one plane:
      //   steps [0, HR)       (F, h = t):      [w(dy,0) ; w(dy,1)] . [x(h,0) | x(h,1)]
      //   steps [HR, 2HR - 1) (G, h = t - HR): [w(0,2) ; w(1,2)] and [0 ; w(2,2)]
      //                                        . [x(h,2) | x(h+1,2)]
      // 5 MFMAs per 16 channels and row (4.5 the floor); the F weights read at the slab's
      // start, the G pairs in its steps 1 and 2
      auto read_Bf = [&](const char* st, int t) -> e8 {
        if (t < HR) return rdB(st + oF + t * PITCH * 32);
        return rdB(st + oG + (t - HR) * PITCH * 32);
      };
#pragma unroll
      for (int k = 0; k < (DB > 3 ? DB : 3); ++k) {  // in the order the first steps use them
        if (k < DB) Bq[k] = read_Bf(cur, k);
        if (k < 3) read_A(cur, 3, k, AS[1][k]);
      }
      auto stepb = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if (IDF_DX3_SB) __builtin_amdgcn_sched_barrier(0);
        dma_step(tc);
        if constexpr (t == 1 || t == 2) {
#pragma unroll
          for (int n = 0; n < NF; ++n) {
            if (t == 1) AZ[0][n] = rdA(cur + oAG + n * 512);
            else AZ[1][n] = rdA(zlane ? zO + n * 512 : cur + oAO + n * 512);
          }
        }
        if constexpr (t + DB < NS) Bq[(t + DB) % RB] = read_Bf(cur, t + DB);
        const e8& Bv = Bq[t % RB];
        if constexpr (t < HR) {
          mma_rows(AS[1], Bv, t);
        } else {
          constexpr int h = t - HR;
          if constexpr (h < WRW) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(AZ[0][n], Bv, acc[h][n]);
          }
          if constexpr (h > 0) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(AZ[1][n], Bv, acc[h - 1][n]);
          }
        }
      };
      dx_unroll(stepb, std::make_integer_sequence<int, NS>{});
      DX3_STAMP(s - s0, 3);
      continue;
    }
    if constexpr (IDF_DX3_PAIRS) {
      // The paired schedule: the hi weights' taps paired as the lo weights' are, so no weight
      // fragment is read twice ([wh ; wh] was: 42 weight-fragment reads a slab, now 30 -- the
      // CU's LDS read bandwidth co-bounds the loop), at the same 14 MFMAs per row and fragment:
      //   F_h [0, HR)          h = t:            [wh(dy,0) ; wh(dy,1)], [wl(dy,0) ; wl(dy,1)]
      //                                          . [xh(h,0) | xh(h,1)]
      //   F_l [HR, 2HR)        h = t - HR:       [wh(dy,0) ; wh(dy,1)] . [xl(h,0) | xl(h,1)]
      //   G_h [2HR, 3HR-1)     h = t - 2HR:      [wh(0,2) ; wh(1,2)], [wl(0,2) ; wl(1,2)] (row h),
      //                                          [0 ; wl(2,2)] (row h - 1) . [xh(h,2) | xh(h+1,2)]
      //   G_l [3HR-1, +WRW)     h = t - 3HR + 1:  [wh(0,2) ; wh(1,2)] . [xl(h,2) | xl(h+1,2)]
      //   P   [TP, NS)         m = t - TP:       [wh(2,2) ; wh(2,2)] . [xh | xl](m + 2, 2)
      constexpr int TL = HR, TG = 2 * HR, TGL = 3 * HR - 1, TP = TGL + WRW;
      static_assert(BF || TP + WRW == NS, "the paired schedule's steps");
      e8 AH[3][NF], AL[3][NF], GH[NF], GL[NF], GZ[NF], PW[NF];
      auto read_Bp = [&](const char* st, int t) -> e8 {
        if (t < TL) return rdB(st + oF + t * PITCH * 32);
        if (t < TG) return rdB(st + oF + L::PLANE + (t - TL) * PITCH * 32);
        if (t < TGL) return rdB(st + oG + (t - TG) * PITCH * 32);
        if (t < TP) return rdB(st + oG + L::PLANE + (t - TGL) * PITCH * 32);
        return rdB(st + oP + ((t - TP + 2) * PITCH + 2) * 32);
      };
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int n = 0; n < NF; ++n) AH[dy][n] = rdA(cur + oAHF + (3 * dy * NF + n) * 512);
#pragma unroll
      for (int n = 0; n < NF; ++n) AL[0][n] = rdA(cur + oAF + n * 512);
#pragma unroll
      for (int k = 0; k < DB; ++k) Bq[k] = read_Bp(cur, k);
      auto stepp = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if (IDF_DX3_SB) __builtin_amdgcn_sched_barrier(0);
        dma_step(tc);
        // weights one phase ahead where a register set is free: the lo F pairs dy = 1, 2 in steps
        // 0, 1 (first used in steps 1, 2, after that step's hi products); the G sets in F_l
        // (the lo F pairs are dead); the P set in G_h (the hi F pairs are dead)
        if constexpr (t < 2) {
#pragma unroll
          for (int n = 0; n < NF; ++n) AL[t + 1][n] = rdA(cur + oAF + (3 * (t + 1) * NF + n) * 512);
        }
        if constexpr (t >= TL && t < TL + 3) {
#pragma unroll
          for (int n = 0; n < NF; ++n) {
            if constexpr (t == TL) GH[n] = rdA(cur + oAHG + n * 512);
            else if constexpr (t == TL + 1) GL[n] = rdA(cur + oAG + n * 512);
            else GZ[n] = rdA(zlane ? zO + n * 512 : cur + oAO + n * 512);
          }
        }
        if constexpr (t == TG) {
#pragma unroll
          for (int n = 0; n < NF; ++n) PW[n] = rdA(cur + oAH + (8 * NF + n) * 512);
        }
        if constexpr (t + DB < NS) Bq[(t + DB) % RB] = read_Bp(cur, t + DB);
        const e8& Bv = Bq[t % RB];
        if constexpr (t < TL) {
          mma_rows(AH, Bv, t);
          mma_rows(AL, Bv, t);
        } else if constexpr (t < TG) {
          mma_rows(AH, Bv, t - TL);
        } else if constexpr (t < TGL) {
          constexpr int h = t - TG;
          if constexpr (h < WRW) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(GH[n], Bv, acc[h][n]);
          }
          if constexpr (h > 0) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(GZ[n], Bv, acc[h - 1][n]);
          }
          if constexpr (h < WRW) {
#pragma unroll
            for (int n = 0; n < NF; ++n) mma(GL[n], Bv, acc[h][n]);
          }
        } else if constexpr (t < TP) {
          constexpr int h = t - TGL;
#pragma unroll
          for (int n = 0; n < NF; ++n) mma(GH[n], Bv, acc[h][n]);
        } else {
          constexpr int m = t - TP;
#pragma unroll
          for (int n = 0; n < NF; ++n) mma(PW[n], Bv, acc[m][n]);
        }
      };
      dx_unroll(stepp, std::make_integer_sequence<int, NS>{});
      DX3_STAMP(s - s0, 3);
      continue;
    }
    // the slab's first reads interleaved in the order the first steps use them (step h needs
    // kernel rows dy <= h and pixel fragment h): the first MFMA waits for two reads, not twelve
#pragma unroll
    for (int k = 0; k < (DB > 3 ? DB : 3); ++k) {
      if (k < DB) Bq[k] = read_B(cur, k);
      if (k < 3) read_A(cur, 0, k, AS[0][k]);
    }
    auto step = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if (IDF_DX3_SB) __builtin_amdgcn_sched_barrier(0);  // keep the schedule: steps do not mix
      if constexpr (t == 9) DX3_STAMP(s - s0, 2);
      // timing knob: wave priority by step (1: the SIMD's two waves alternate the lead every
      // step; 2: every IDF_DX3_PRIO_K steps; 3: the younger wave leads the slab's first half)
      if constexpr (IDF_DX3_PRIO == 1) {
        if (((t & 1) != 0) == ((wave & 4) != 0)) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      } else if constexpr (IDF_DX3_PRIO == 2) {
        if (((t / IDF_DX3_PRIO_K) & 1) == ((wave >> 2) & 1)) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      } else if constexpr (IDF_DX3_PRIO == 3) {
        if constexpr (t == 0) { if (wave & 4) __builtin_amdgcn_s_setprio(1); }
        if constexpr (t == NS / 2) __builtin_amdgcn_s_setprio(0);
      }
      dma_step(tc);
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
        if constexpr (h < WRW) {
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
    DX3_STAMP(s - s0, 3);
  }
  DX3_PHASE(2, __builtin_amdgcn_s_memtime());
  DX3_TL(3);
  // the tables in LDS before any epilogue reads them: stored here when the loop had no second
  // slab, and ordered by one more barrier when no slab barrier followed the store
  if (s1 - s0 <= 1) {
    if (s1 == s0) tabs.load(g, Ly, grp, tid);
    tabs.store((float*)(lds + L::BOFF), (float*)(lds + L::HOFF), g, Ly, grp, tid);
  }
  if (s1 - s0 <= 2) __syncthreads();

  // ---- split K: every chunk's block stores its raw sums; the tile's last block to finish
  // adds them in chunk order (its own from registers -- the same bits) and runs the epilogue.
  // The hand-off within the launch (MI355X_MICROARCH.md "Valid forms", table row 1): payload
  // stored write-through (sc1, 16 B a lane), every storing wave drained (vmcnt 0), a workgroup
  // barrier, ONE lane's agent-scope atomic add on the tile's counter; the block whose add
  // returns nchunk - 1 is last, resets the counter and reads every chunk with sc1 loads (which
  // bypass this CU's L1) -- no release / acquire fences, whose L2 write-back costs microseconds
  // per block.
  // (compiled only into the one-tile blocks: the host splits K only with T = 1)
  if constexpr (T == 1 && !ML) if (Ly.nchunk > 1) {
    constexpr int FR = kDxWaves * WR * NF;  // fragments per block
    const uint32_t pb = (uint32_t)((tb * g.ngroup + grp) * Ly.nchunk) * (FR * 1024u);  // bytes
    const int64_t pbytes = (int64_t)g.nblk_tiles * g.ngroup * Ly.nchunk * FR * 1024;
    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)g.part, 0, (int)(pbytes < (int64_t)kDxInvalid ? pbytes : (int64_t)kDxInvalid), 0x00020000);
    auto poff = [&](int c, int m, int n) -> uint32_t {
      return pb + (uint32_t)((c * FR + (tw * 16 + r0 + m) * NF + n) * 1024 + lane * 16);
    };
#pragma unroll
    for (int m = 0; m < WRW; ++m)
#pragma unroll
      for (int n = 0; n < NF; ++n)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[m][n]), pr, poff(chunk, m, n),
                                               0, 16 /* sc1 */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (tid == 0) {
      const uint32_t old = __hip_atomic_fetch_add(g.ctr + tb * g.ngroup + grp, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      const bool last = old == (uint32_t)(Ly.nchunk - 1);
      if (last)  // no other block touches it again in this launch: zero for the next one
        __hip_atomic_store(g.ctr + tb * g.ngroup + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_flag = last;
    }
    __syncthreads();
    DX3_TL(6);
    if (!*last_flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
    // every other chunk's fragments in flight at once (one memory round trip, not nchunk), then
    // the sums in chunk order; chunk slots past nchunk and the block's own read nothing
    static_assert(IDF_DX3_KSPLIT <= 4, "the reduction holds up to 4 chunks");
    d4 pv[4][WRW][NF];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int m = 0; m < WRW; ++m)
#pragma unroll
        for (int n = 0; n < NF; ++n)
          pv[c][m][n] = (c < Ly.nchunk && c != chunk)
                            ? __builtin_bit_cast(d4, __builtin_amdgcn_raw_buffer_load_b128(pr, poff(c, m, n), 0, 16))
                            : acc[m][n];
#pragma unroll
    for (int m = 0; m < WRW; ++m)
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        d4 sum = pv[0][m][n];
#pragma unroll
        for (int c = 1; c < 4; ++c)
          if (c < Ly.nchunk) sum = sum + pv[c][m][n];
        acc[m][n] = sum;
      }
    DX3_TL(4);
  }

  // ---- epilogue: lane holds outputs 16 (grp NF + n) + 4q .. +3 of packed pixel (row r0 + m,
  // column j) of its tile.  fp32 outputs to out (unless skip_f32); their split pairs to XS at
  // channel C + that output (zeros for the padding outputs >= N and -- the last group -- on to
  // the next 16-channel boundary past C + N, so the next layer's last slab reads finite values;
  // never past the split buffer).  With a fused head every lane of the wave takes part in the
  // head's cross-lane sums, so lanes without an output (gutter columns, rows past the image,
  // images past the batch) compute and only skip their stores.
  if (tile >= g.ntiles) return;
  const bool lane_ok = xj < g.Wd && ixj < g.nbx;  // a gutter column or past the band: no output
  const WAct act(g.act, g.slope);
  const float* btab = (const float*)(lds + L::BOFF);
  const float* htab = (const float*)(lds + L::HOFF);
  const bool fh = g.nh > 0;
  bool out_ok = true;
  const int zr = (Ly.C + g.N + 15) / 16 * 16, zend = zr < 16 * g.nslab_xs ? zr : 16 * g.nslab_xs;
  const bool lastg = grp == g.ngroup - 1;
  char* xsb = (char*)g.xs;
  // the wave's rows: image, y, pixel, whether the lane has an output there
  int r_img[WRW], r_y[WRW];
  int64_t r_pix[WRW];
  bool r_ok[WRW];
#pragma unroll
  for (int m = 0; m < WRW; ++m) {
    int iy = iyw, y = uyw + m - iyw * g.H;
    if (g.gut) {
      iy = udiv_s(uyw + m, g.hp);
      y = uyw + m - iy * g.hp;
    }
    r_img[m] = (dt.band * g.nby + iy) * g.nbx + ixj;
    r_y[m] = y;
    r_ok[m] = lane_ok && y < g.H && iy < g.nby && r_img[m] < g.B;
    r_pix[m] = ((int64_t)r_img[m] * g.H + y) * g.Wd + xj;
  }
  // the head's running sums of the wave's rows, loaded before any store of the epilogue (a
  // store may alias them for all the compiler knows, so a load after one would wait it out)
  d4 hprev[WRW];
#pragma unroll
  for (int m = 0; m < WRW; ++m) {
    hprev[m] = d4{0.f, 0.f, 0.f, 0.f};
    if constexpr (ML) hprev[m] = hreg[m];  // (zeros where the head init left them)
    else if (fh && r_ok[m] && 4 * q < g.nh) hprev[m] = *(const d4*)(g.hacc + r_pix[m] * 16 + 4 * q);
  }
  // outputs: bias, activation, the fp32 and split stores; acc[m][n] becomes the output (zeros
  // past N), which the head's shares below read
#pragma unroll
  for (int m = 0; m < WRW; ++m) {
    const bool row_ok = r_ok[m];
    if (!row_ok && !fh) continue;
    const int cls = bias_class(r_y[m], xj, g.H, g.Wd);
    const int64_t pix = r_pix[m];
    float* dst = Ly.out + pix * g.ldo;
#pragma unroll
    for (int n = 0; n <= NF; ++n) {
      if (n == NF && !lastg) break;
      const int nl = 16 * n + 4 * q;              // within the group
      const int n0 = 16 * grp * NF + nl;          // output column
      d4 v = d4{0.f, 0.f, 0.f, 0.f};
      if (n < NF && n0 < g.N) {
        const d4 bv = *(const d4*)(btab + cls * (NF * 16) + nl);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float t = acc[m][n][k] * Ly.yscale + bv[k];
          v[k] = act.tanh_ ? wact(t, g.act, g.slope) : act(t);
          if (!BF && row_ok) out_ok = out_ok && fabsf(v[k]) < kDxOutGuard;
        }
        if (row_ok && !g.skip_f32) {
          if (n0 + 4 <= g.N) {
            *(d4*)(dst + n0) = v;
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (n0 + k < g.N) dst[n0 + k] = v[k];
          }
        }
        for (int k = g.N - n0; k < 4; ++k) v[k] = 0.0f;
      }
      if (n < NF) acc[m][n] = v;
      const int c = Ly.C + n0;  // split channel of v[0]; c % 4 == 0, so v stays in one slab
      if (row_ok && !(IDF_DX3_ABLATE & 128) && c < zend) {
        if constexpr (BF) {  // the bf16 copy, round to nearest even
          typedef __bf16 b4 __attribute__((ext_vector_type(4)));
          *(b4*)(xsb + (int64_t)(c >> 4) * g.xs_slab + pix * g.xs_pix + (c & 15) * 2) =
              __builtin_convertvector(v, b4);
        } else {
          const e4 h = __builtin_convertvector(v, e4);
          const e4 l = __builtin_convertvector(v - __builtin_convertvector(h, d4), e4);
          char* p = xsb + (int64_t)(c >> 4) * 2 * plane_b + pix * 32 + (c & 15) * 2;
          *(e4*)p = h;
          *(e4*)(p + plane_b) = l;
        }
      }
    }
  }
  if (fh) {
    // this lane's share of the head sums of its pixels (its 4 x NF channels): each head weight
    // quad read from LDS once and applied to the wave's WRW rows (per row and output: channels
    // in order, fragments in order; zero weights past N) -- one read per row cost the epilogue
    // ~8k cycles of LDS bandwidth per block
    float hp[WRW][16];
#pragma unroll
    for (int m = 0; m < WRW; ++m)
#pragma unroll
      for (int o = 0; o < 16; ++o) hp[m][o] = 0.0f;
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int nl = 16 * n + 4 * q;
      if (16 * grp * NF + nl >= g.N) continue;
#pragma unroll
      for (int o = 0; o < 16; ++o) {
        if (o < g.nh) {  // (no early exit: the loop must unroll, hp stays in registers)
          const d4 wv = *(const d4*)(htab + o * (NF * 16) + nl);
#pragma unroll
          for (int m = 0; m < WRW; ++m)
#pragma unroll
            for (int k = 0; k < 4; ++k) hp[m][o] = __builtin_fmaf(wv[k], acc[m][n][k], hp[m][o]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < WRW; ++m) {
      // the pixel's 4 lanes (q) reduce-scatter their shares: lane q ends with the sums of head
      // outputs 4q .. 4q + 3 -- (h_q + h_q^2) then + the pair q^1 -- one fixed order per output
      float r8[8], r4[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float mine = q < 2 ? hp[m][i] : hp[m][8 + i];
        const float give = q < 2 ? hp[m][8 + i] : hp[m][i];
        r8[i] = mine + __shfl_xor(give, 32);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float mine = (q & 1) ? r8[4 + i] : r8[i];
        const float give = (q & 1) ? r8[i] : r8[4 + i];
        r4[i] = mine + __shfl_xor(give, 16);
      }
      if (r_ok[m] && 4 * q < g.nh) {
        const int64_t pix = r_pix[m];
        d4* ap = (d4*)(g.hacc + pix * 16 + 4 * q);
        const d4 prev = hprev[m];
        d4 hv;
#pragma unroll
        for (int i = 0; i < 4; ++i) hv[i] = prev[i] + r4[i];
        if (!Ly.hlast) {
          if constexpr (ML) hreg[m] = hv;
          else *ap = hv;
        } else {  // the complete head: its epilogue (flow_kernels.hip gemm_f32_kernel's)
          const int b_img = r_img[m];
          const int64_t hw_ = (int64_t)g.H * g.Wd, rem = (int64_t)r_y[m] * g.Wd + xj;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int o = 4 * q + i;
            if (o >= g.nh) break;
            const float vv = hv[i];
            if (g.hmode == IDF_EPI_COUPLE_ADD || g.hmode == IDF_EPI_COUPLE_SUB) {
              const float r = __builtin_rintf(vv * 256.0f) / 256.0f;  // roundlib.py:34-38
              const float bsv = g.hbase[pix * g.hld_base + o];
              g.hout[pix * g.hld_out + o] = g.hmode == IDF_EPI_COUPLE_ADD ? bsv + r : bsv - r;
            } else if (g.hmode == IDF_EPI_PRIOR) {
              if (o < g.hn_mean) {
                g.hmean[((int64_t)b_img * g.hn_mean + o) * hw_ + rem] = vv;
              } else {
                const int64_t oi = ((int64_t)b_img * g.hn_mean + (o - g.hn_mean)) * hw_ + rem;
                g.hlogs[oi] = vv;
                g.hscale[oi] = expf_glibc(vv);
              }
            } else {
              g.hout[pix * g.hld_out + o] = vv;
            }
          }
        }
      }
    }
  }
  if (!out_ok && g.flag) atomicOr(g.flag, 1u);
  DX3_TL(5);
  DX3_PHASE(3, __builtin_amdgcn_s_memtime());
  DX3_PHASE(5, __builtin_amdgcn_s_memrealtime());
  if constexpr (ML) {
    // the layer's outputs (split copy, fp32 rows) stored and its LDS reads done before the next
    // layer's DMA reads them / overwrites the stages and tables: every wave drained, one barrier
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  }  // layers
}

template <int NF, int WR, int PITCH, int PLANE_KIB, bool BF>
__global__ void __launch_bounds__(kDxThreads, 1) conv3_dx3_kernel(Dx3Args g) {
  __shared__ __attribute__((aligned(16))) char lds[Dx3Lds<NF, WR, PITCH, PLANE_KIB, BF>::BYTES];
  if constexpr (IDF_DX3_MIX && !BF && WR * kDxWaves == 32 && WR >= 2) {
    constexpr int D = IDF_DX3_MIX == 2 ? -1 : 1;  // 1: the older waves take WR + 1 rows, 2: WR - 1
    if (threadIdx.x < 256) dx3_block<NF, WR, PITCH, PLANE_KIB, BF, false, WR + D>(g, nullptr, lds);
    else dx3_block<NF, WR, PITCH, PLANE_KIB, BF, false, WR - D>(g, nullptr, lds);
  } else {
    dx3_block<NF, WR, PITCH, PLANE_KIB, BF, false>(g, nullptr, lds);
  }
}

// The fused DenseBlock: every layer of a block, one workgroup per tile (Dx3MLArgs)
template <int NF, int PITCH, int PLANE_KIB, bool BF>
__global__ void __launch_bounds__(kDxThreads, 1) conv3_dx3_block_kernel(Dx3Args g, Dx3MLArgs ml) {
  __shared__ __attribute__((aligned(16))) char lds[Dx3Lds<NF, 16 / kDxWaves, PITCH, PLANE_KIB, BF>::BYTES];
  dx3_block<NF, 16 / kDxWaves, PITCH, PLANE_KIB, BF, true>(g, &ml, lds);
}

// Block-input split: XS channels [c0, c1) of every pixel from the fp32 rows x (ld_x floats),
// zeros for [c1, round16(c1)) (the first layer's own output slab: other blocks of that
// layer's launch read it -- as halo -- while its own blocks write it, so the value a reader
// sees depends on timing; it is only ever multiplied by exactly-zero weights (packing
// dx3_weights asserts the weights of channels >= C are +0) and every value written there is
// finite (these zeros, and outputs under the |y| < 8192 guard), so the product is +-0 either
// way and the sum's bits do not depend on which value was read);
// ORs bit 0 of flag for a value that is NaN or |x| >= 32768 (the f16 pairs' range).  One
// thread per (pixel, 4 channels).  Threads [0, nzero) also clear zero[] (the split-K tile
// counters of the block's dx3 layers, idf_conv3x3_dx3: zero before a block's first layer).
// With hacc (c0 = 0; the fused head of a block run as per-layer launches) the same launch
// starts the head's running sums, dx3_head_init_kernel's arithmetic: the thread of a pixel's
// quad k < 4 forms outputs 4k .. 4k + 3, each bias[o] then c = 0 .. c1 - 1 in order,
// fmaf(w[o][c], x[c], .) -- the same chain, so the same bits (one thread per pixel and 16
// outputs in its own range of the launch measured slower: 24.2 vs 20.3 ms over the bench
// profile, against 14.2 + 9.5 for the two launches, profiles/r06/head_split/).
// pixel p's running head sums from the block input (dx3_head_init_kernel's per-pixel body)
__device__ __forceinline__ void dx3_head_init_pixel(int64_t p, int32_t C0, const float* __restrict__ x,
                                                    int64_t ld_x, const float* __restrict__ w,
                                                    int32_t ldw, const float* __restrict__ bias,
                                                    int32_t nh, float* __restrict__ acc) {
  float h[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) h[o] = o < nh ? bias[o] : 0.0f;
  const float* xr = x + p * ld_x;
  for (int c = 0; c < C0; c += 4) {
    const d4 xv = *(const d4*)(xr + c);
#pragma unroll
    for (int o = 0; o < 16; ++o) {
      if (o >= nh) break;
      const d4 wv = *(const d4*)(w + (int64_t)o * ldw + c);  // uniform: one scalar 16-B load
#pragma unroll
      for (int k = 0; k < 4; ++k) h[o] = __builtin_fmaf(wv[k], xv[k], h[o]);
    }
  }
  d4* ap = (d4*)(acc + p * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) ap[i] = d4{h[4 * i], h[4 * i + 1], h[4 * i + 2], h[4 * i + 3]};
}

struct Dx3HeadInit {
  const float* w;
  int32_t ldw;
  const float* bias;
  int32_t nh;
  float* acc;  // [P][16]
};
__global__ void __launch_bounds__(256) dx3_split_cols_kernel(int64_t P, int32_t c0, int32_t c1,
                                                             const float* __restrict__ x,
                                                             int64_t ld_x, uint16_t* __restrict__ xs,
                                                             uint32_t* __restrict__ flag,
                                                             uint32_t* __restrict__ zero,
                                                             int32_t nzero, Dx3HeadInit hi) {
  const int nq = ((c1 + 15) / 16 * 16 - c0) / 4;  // channel quads per pixel
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < nzero) zero[g] = 0u;
  if (g >= P * nq) return;
  const int64_t pix = g / nq;
  const int kq = (int)(g - pix * nq);
  const int c = c0 + 4 * kq;
  if (hi.acc && kq < 4) {
    d4 h;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = 4 * kq + i < hi.nh ? hi.bias[4 * kq + i] : 0.0f;
    const float* xr = x + pix * ld_x;
    for (int cc = 0; cc < c1; cc += 4) {
      const d4 xv = *(const d4*)(xr + cc);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (4 * kq + i >= hi.nh) break;
        const d4 wv = *(const d4*)(hi.w + (int64_t)(4 * kq + i) * hi.ldw + cc);
#pragma unroll
        for (int k = 0; k < 4; ++k) h[i] = __builtin_fmaf(wv[k], xv[k], h[i]);
      }
    }
    *(d4*)(hi.acc + pix * 16 + 4 * kq) = h;
  }
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

// Block-input bf16 copy for the bf16 direct conv: XB channels [c0, c1) of every pixel, slab-major
// [slab][P][16] bf16 (round to nearest even), zeros for [c1, round16(c1)).  One thread per
// (pixel, 4 channels); threads [0, nzero) also clear zero[] (the split-K counters).
__global__ void __launch_bounds__(256) dxb_cols_kernel(int64_t P, int32_t c0, int32_t c1,
                                                       const float* __restrict__ x, int64_t ld_x,
                                                       uint16_t* __restrict__ xb,
                                                       uint32_t* __restrict__ zero, int32_t nzero) {
  const int nq = ((c1 + 15) / 16 * 16 - c0) / 4;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < nzero) zero[g] = 0u;
  if (g >= P * nq) return;
  const int64_t pix = g / nq;
  const int c = c0 + 4 * (int)(g - pix * nq);
  d4 v = d4{0.f, 0.f, 0.f, 0.f};
  if (c < c1) v = *(const d4*)(x + pix * ld_x + c);
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  *(b4*)((char*)xb + ((int64_t)(c >> 4) * P + pix) * 32 + (c & 15) * 2) = __builtin_convertvector(v, b4);
}

// ---- geometry plan (host): how a (H, W, N) layer tiles, packs and splits.  A function of the
// image geometry, the output count and C only -- never of the batch -- so an encoder and its
// decoder run every layer with the same tiles, chunks and summation order.
struct Dx3Plan {
  int ok, pitch, plane_kib, nbx, nby, ch, seg, segw, nseg, gut, wp, hp, nf, ngroup, split, tilew,
      xskip;
};

static int dx3_gcd(int a, int b) { return b ? dx3_gcd(b, a % b) : a; }

static Dx3Plan dx3_plan(int H, int W, int N, bool bf = false) {
  Dx3Plan p = {};
  p.tilew = 16;
  if (H < 1 || W < 1 || N < 1 || N > 1024) return p;
  const int nft = (N + 15) / 16;
  p.nf = nft <= 4 ? nft : 4;
  p.ngroup = (nft + p.nf - 1) / p.nf;
  if (W % 16 == 0) {  // 16-wide tiles of one image, any H (16-row tiles)
    p.nbx = 1; p.nby = 1; p.pitch = 18; p.ch = 18; p.segw = 18; p.nseg = 1; p.plane_kib = 11;
    p.ok = 1;
  } else if (W == 4 || W == 8) {
    // 16 / W images across a tile, one canvas segment each (every lane an output); H = 2, 4, 8
    // stacked down the tile too, with gutter rows in the segment
    p.nbx = 16 / W; p.pitch = W + 2; p.segw = W + 2; p.nseg = p.nbx;
    p.plane_kib = W == 8 ? 13 : 19;
    if (H == 2 || H == 4 || H == 8) {
      p.nby = 16 / H;
      p.ch = p.nby * (H + 2);
    } else {
      p.nby = 1;
      p.ch = 18;
    }
    // segment stride = W (mod 8) slots: lane j's column base is then j (mod 8) in every
    // segment, so the fragment reads stay bank-conflict-free
    int sg = p.ch * p.pitch;
    while ((sg - W) % 8) ++sg;
    p.seg = sg;
    p.ok = (p.nseg * sg * 32 + 1023) / 1024 <= p.plane_kib;
  }
  if (!p.ok) {
    // gutter packing (any other geometry): images at pitch W + 1 across and H + 1 down in bands
    // of nbx x nby whose packed extent is a whole number of 16-pixel tiles where that fits in
    // 8 tiles; the one zero column / row between two images is both images' padding, so the
    // canvas is the plain 18 x 18 one and a gutter lane's output is simply not stored
    p.gut = 1; p.wp = W + 1; p.hp = H + 1;
    p.nbx = 16 / dx3_gcd(p.wp, 16);
    while (p.nbx > 1 && p.nbx * p.wp > 128) p.nbx /= 2;
    p.nby = 16 / dx3_gcd(p.hp, 16);
    while (p.nby > 1 && p.nby * p.hp > 128) p.nby /= 2;
    p.pitch = 18; p.ch = 18; p.segw = 18; p.nseg = 1; p.seg = 0; p.plane_kib = 11;
    p.ok = 1;
    if (W == 2 && !bf) {
      // 2-wide images (config 4's 2 x 2 level): the 16 lanes on 8 images' real columns, not on
      // 16 packed columns of which a third are gutters -- a tile spans 24 packed columns, its
      // canvas 25 x 18 slots (lane j's column base 3 (j / 2) + j % 2); the rows stay packed
      p.xskip = 1; p.tilew = 24; p.pitch = 25; p.segw = 25; p.plane_kib = 15;
    }
  }
  // split K where a level's tiles are few for any batch the bench runs (imagenet64's 8 x 8:
  // 64 tiles per 256 images): by the geometry alone
  p.split = (H * W <= 64 && p.nbx * p.nby <= 4) ? IDF_DX3_KSPLIT
            : (H == 16 && W == 16) ? IDF_DX3_KSPLIT16 : 1;
  return p;
}

}  // namespace idf

using namespace idf;

#if IDF_DX3_TL
extern "C" int idf_dx3_timeline(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dx3_tl), sizeof(g_dx3_tl)) == hipSuccess ? 0 : 2;
}
#endif

#if IDF_DX3_STAMPS
extern "C" int idf_dx3_stamps(unsigned long long* host) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dx3_stamp), sizeof(g_dx3_stamp)) != hipSuccess) return 2;
  return hipMemcpyFromSymbol(host + 8 * 40 * 4, HIP_SYMBOL(g_dx3_phase), sizeof(g_dx3_phase)) == hipSuccess ? 0 : 2;
}
#endif

namespace {

// tiles across / down one band of the plan's packing
int dx3_tiles_x(const Dx3Plan& p, int W) {
  return (p.nbx * (p.gut ? p.wp : W) + p.tilew - 1) / p.tilew;
}
int dx3_tiles_y(const Dx3Plan& p, int H) { return (p.nby * (p.gut ? p.hp : H) + 15) / 16; }

struct Dx3Launch {
  Dx3Plan pl;
  int64_t ntiles;
  int T, nblk_tiles, nslab, nchunk, chunk_slabs;
  int64_t ctr_bytes, part_bytes;
};

// the launch shape of a layer: tiles, tiles per block (two where every CU still gets a block,
// at the 16-wide canvas), split-K chunks and the workspace they need
Dx3Launch dx3_launch_shape(int B, int H, int W, int C, int N, bool bf = false) {
  Dx3Launch s = {};
  s.pl = dx3_plan(H, W, N, bf);
  if (!s.pl.ok || B < 1) return s;
  const int64_t nbands = (B + s.pl.nbx * s.pl.nby - 1) / (s.pl.nbx * s.pl.nby);
  const int tiles_x = dx3_tiles_x(s.pl, W), tiles_y = dx3_tiles_y(s.pl, H);
  s.ntiles = nbands * tiles_x * tiles_y;
  s.nslab = (C + 15) / 16;
  s.chunk_slabs = s.nslab > 0 ? (s.nslab + s.pl.split - 1) / s.pl.split : 1;
  s.nchunk = s.nslab > 0 ? (s.nslab + s.chunk_slabs - 1) / s.chunk_slabs : 1;
  const bool two = s.pl.pitch == 18 && s.pl.nf <= 3 && s.nchunk == 1 && s.ntiles >= IDF_DX3_TWO_MIN &&
                   !IDF_DX3_FORCE1;
  s.T = two ? 2 : 1;  // two tiles (4 rows per wave) or one (2 rows)
  s.nblk_tiles = (int)((s.ntiles + s.T - 1) / s.T);
  if (s.nchunk > 1) {
    const int64_t fr = (int64_t)kDxWaves * (16 / kDxWaves) * s.pl.nf;  // fragments per block
    s.ctr_bytes = ((int64_t)s.nblk_tiles * s.pl.ngroup * 4 + 255) / 256 * 256;
    // room for the most chunks any C up to this one splits into (nchunk is not monotonic in
    // C: 7 slabs make 4 chunks of 2, 9 slabs 3 of 3), so one workspace serves a block's layers
    const int most = s.nslab < s.pl.split ? s.nslab : s.pl.split;
    s.part_bytes = (int64_t)s.nblk_tiles * s.pl.ngroup * most * fr * 64 * 16;
  }
  return s;
}

}  // namespace

extern "C" int idf_conv3x3_dx3_supported(int32_t H, int32_t W, int32_t N) {
  return dx3_plan(H, W, N).ok;
}

extern "C" int64_t idf_dx3_split_bytes(int64_t P, int32_t channels) {
  if (P < 0 || channels < 0) return -1;
  return (int64_t)((channels + 15) / 16) * 2 * P * 32;
}

extern "C" int64_t idf_conv3x3_dx3_counter_bytes(int32_t B, int32_t H, int32_t W, int32_t N) {
  const Dx3Launch s = dx3_launch_shape(B, H, W, 16 * 64, N);  // the widest split: every chunk count
  if (!s.pl.ok) return -1;
  if (s.pl.split <= 1) return 0;
  return ((int64_t)s.nblk_tiles * s.pl.ngroup * 4 + 255) / 256 * 256;
}

extern "C" int64_t idf_conv3x3_dx3_workspace(int32_t B, int32_t H, int32_t W, int32_t C, int32_t N) {
  const Dx3Launch s = dx3_launch_shape(B, H, W, C, N);
  if (!s.pl.ok) return -1;
  if (s.nchunk <= 1) return 0;
  return idf_conv3x3_dx3_counter_bytes(B, H, W, N) + s.part_bytes;
}

// the split (and, with head, the head init fused into the same launch)
static int dx3_split_cols_run(void* stream, int64_t P, int32_t c0, int32_t c1, const float* x,
                              int64_t ld_x, uint16_t* xs, int32_t nslab_xs, uint32_t* d_flag,
                              uint32_t* d_zero, int32_t nzero, const Dx3HeadInit& head) {
  if (P < 0 || c1 < c0 || nzero < 0 || (nzero && !d_zero)) return IDF_ERR_ARG;
  if (head.acc) {  // idf_dx3_head_init's contract, over the block input c0 = 0 .. c1
    if (P == 0) return IDF_OK;
    if (c0 != 0 || c1 <= 0 || !head.w || !head.bias || head.nh < 1 || head.nh > 16 || c1 > 64 ||
        head.ldw < c1 || (head.ldw & 3) || (uintptr_t)head.w % 16 || (uintptr_t)head.acc % 16)
      return IDF_ERR_ARG;
  }
  if (P == 0 || c1 == c0) {
    if (nzero) return hipMemsetAsync(d_zero, 0, 4 * (size_t)nzero, (hipStream_t)stream) == hipSuccess
                          ? IDF_OK : IDF_ERR_HIP;
    return IDF_OK;
  }
  if (!x || !xs || (c0 & 15) || (c1 & 3) || (ld_x & 3) || (uintptr_t)x % 16) return IDF_ERR_ARG;
  if ((c1 + 15) / 16 > nslab_xs) return IDF_ERR_ARG;
  int64_t n = P * (((c1 + 15) / 16 * 16 - c0) / 4);
  if (n < nzero) n = nzero;
  hipLaunchKernelGGL(dx3_split_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P, c0, c1, x, ld_x, xs, d_flag, d_zero, nzero, head);
  return idf_last_error();
}

extern "C" int idf_dx3_split_cols(void* stream, int64_t P, int32_t c0, int32_t c1, const float* x,
                                  int64_t ld_x, uint16_t* xs, int32_t nslab_xs, uint32_t* d_flag,
                                  uint32_t* d_zero, int32_t nzero) {
  return dx3_split_cols_run(stream, P, c0, c1, x, ld_x, xs, nslab_xs, d_flag, d_zero, nzero,
                            Dx3HeadInit{});
}

// the block input's split copy and the fused head's running sums in one launch (flow_kernels
// dense_block_run; the same bits as idf_dx3_split_cols + idf_dx3_head_init)
extern "C" int idf_dx3_split_cols_head(void* stream, int64_t P, int32_t c1, const float* x, int64_t ld_x,
                            uint16_t* xs, int32_t nslab_xs, uint32_t* d_flag, uint32_t* d_zero,
                            int32_t nzero, const float* w, int32_t ldw, const float* bias,
                            int32_t n_head, float* acc) {
  if (!acc) return IDF_ERR_ARG;
  return dx3_split_cols_run(stream, P, 0, c1, x, ld_x, xs, nslab_xs, d_flag, d_zero, nzero,
                            Dx3HeadInit{w, ldw, bias, n_head, acc});
}

#ifndef IDF_HEAD_INIT_EXTERNAL  // tools/repro_lds builds link a variant head init instead
// The fused head's running sums start from the block input: acc[p][o] = bias[o] + sum over
// c < C0 of w[o][c] x[p][c] (c in order), o < n_head; 0 for n_head <= o < 16.  One thread per
// pixel, scalar FMAs on the weights read from global memory (wave-uniform, cached).  A version
// staging the weights in LDS (packed FMAs on broadcast ds_read_b128) returned different sums for
// runs of 16 pixels when it ran beside another stream's dx3 layers on the same CUs -- the table
// itself checked intact before and after -- so two decode lanes diverged (profiles/r05/
// fused_head/lds_coresidency.txt; tests/test_gpu_lanes.py test_fused_blocks_two_streams).
__global__ void __launch_bounds__(256) dx3_head_init_kernel(int64_t P, int32_t C0,
                                                            const float* __restrict__ x,
                                                            int64_t ld_x, const float* __restrict__ w,
                                                            int32_t ldw, const float* __restrict__ bias,
                                                            int32_t nh, float* __restrict__ acc) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  dx3_head_init_pixel(p, C0, x, ld_x, w, ldw, bias, nh, acc);
}

extern "C" int idf_dx3_head_init(void* stream, int64_t P, int32_t C0, const float* x, int64_t ld_x,
                                 const float* w, int32_t ldw, const float* bias, int32_t n_head,
                                 float* acc) {
  if (P <= 0) return P < 0 ? IDF_ERR_ARG : IDF_OK;
  if (!x || !w || !bias || !acc || n_head < 1 || n_head > 16 || C0 < 0 || C0 > 64 || (C0 & 3) ||
      (ld_x & 3) || (uintptr_t)x % 16 || (uintptr_t)acc % 16 || ldw < C0 || (ldw & 3) ||
      (uintptr_t)w % 16)
    return IDF_ERR_ARG;
  hipLaunchKernelGGL(dx3_head_init_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P, C0, x, ld_x, w, ldw, bias, n_head, acc);
  return idf_last_error();
}
#endif  // IDF_HEAD_INIT_EXTERNAL

// the bf16 kernel's geometries: the 16-wide canvas (tiles and gutter packing) and the 8 x 8
// level's segments, one output group of up to 3 fragments (the bf16 blocks' growth <= 48)
static bool dxb_plan_ok(const Dx3Plan& p) {
  return p.ok && p.nf <= 3 && p.ngroup == 1 && (p.pitch == 18 || p.pitch == 10);
}

extern "C" int idf_conv3x3_dxb_supported(int32_t H, int32_t W, int32_t N) {
  return dxb_plan_ok(dx3_plan(H, W, N, true)) ? 1 : 0;
}

// A dx3 launch's arguments, split-f16 (bf = false: xs the split copy) or bf16 (bf = true: xs the
// bf16 shadow).  xs_pix / xs_slab / xs_bytes: the buffer's pixel and slab strides and size,
// bytes.  ml: the fused DenseBlock's first layer (no split-K workspace; one tile per block).
static int dx3_args(Dx3Args& g, Dx3Launch& sh, bool ml, bool bf, int32_t B, int32_t H, int32_t W,
                    int32_t C, uint16_t* xs, int64_t xs_pix, int64_t xs_slab, int64_t xs_bytes,
                    int32_t nslab_xs, const uint16_t* w, int32_t nft, float yscale, const float* b3,
                    const float* vtap, int32_t ldv, const float* bfull, int32_t N, float* out,
                    int64_t ld_out, int32_t act, float slope, uint32_t* d_flag, void* d_workspace,
                    int64_t workspace_bytes, const IdfDx3Head* head) {
  if (C <= 0 || (C & 3) || !w || !xs || !out || !b3) return IDF_ERR_ARG;
  sh = dx3_launch_shape(B, H, W, C, N, bf);
  if (!sh.pl.ok || (bf && !dxb_plan_ok(sh.pl))) return IDF_ERR_UNSUPPORTED;
  if (ml) {  // one tile per workgroup, every chunk in it
    sh.T = 1;
    sh.nblk_tiles = (int)sh.ntiles;
  }
  // the weights hold exactly the kernel's fragments: ngroup groups of nf, nft = ngroup * nf
  if (nft != sh.pl.ngroup * sh.pl.nf) return IDF_ERR_ARG;
  if (vtap && (!bfull || ldv < N)) return IDF_ERR_ARG;
  if ((uintptr_t)out % 16 || ld_out % 4) return IDF_ERR_ARG;  // 16-B output stores
  if ((C + 15) / 16 > nslab_xs) return IDF_ERR_ARG;          // the input slabs must exist
  const int64_t P = (int64_t)B * H * W;
  // 32-bit buffer offsets within a slab, and kDxOff past the end of every slab: one slab of the
  // copy must span < 2 GiB (P < 32M pixels)
  if (xs_slab >= (int64_t)kDxOff) return IDF_ERR_UNSUPPORTED;
  const int64_t nblk = (int64_t)sh.nblk_tiles * sh.pl.ngroup * (ml ? 1 : sh.nchunk);
  if (sh.ntiles >= (1 << 20) || nblk >= (1 << 20)) return IDF_ERR_UNSUPPORTED;  // udiv_s operands
  g = {};
  if (sh.nchunk > 1 && !ml) {
    // split K: the kernel addresses the partial sums with 32-bit offsets through one buffer
    // resource (kDxInvalid records at most), nblk blocks x fragments x 1 KiB
    if (nblk * (int64_t)(kDxWaves * (16 / kDxWaves) * sh.pl.nf) * 1024 >= (int64_t)kDxInvalid)
      return IDF_ERR_UNSUPPORTED;
    const int64_t cb = idf_conv3x3_dx3_counter_bytes(B, H, W, N);
    if (!d_workspace || (uintptr_t)d_workspace % 256 || workspace_bytes < cb + sh.part_bytes)
      return IDF_ERR_WORKSPACE;
    g.ctr = (uint32_t*)d_workspace;
    g.part = (float*)((char*)d_workspace + cb);
  }
  g.xs = xs; g.P = P; g.nslab_xs = nslab_xs; g.C = C;
  g.xs_pix = xs_pix; g.xs_slab = xs_slab; g.xs_bytes = xs_bytes;
  g.Wt = w; g.nslab = sh.nslab; g.ngroup = sh.pl.ngroup; g.N = N;
  g.B = B; g.H = H; g.Wd = W;
  g.nbx = sh.pl.nbx; g.nby = sh.pl.nby;
  g.tiles_x = dx3_tiles_x(sh.pl, W);
  g.tiles_y = dx3_tiles_y(sh.pl, H);
  g.ntiles = (int32_t)sh.ntiles;
  g.nblk_tiles = sh.nblk_tiles;
  g.ch = sh.pl.ch; g.seg = sh.pl.seg; g.segw = sh.pl.segw; g.nseg = sh.pl.nseg;
  g.gut = sh.pl.gut; g.wp = sh.pl.wp; g.hp = sh.pl.hp;
  g.tilew = sh.pl.tilew; g.xskip = sh.pl.xskip;
  g.nchunk = sh.nchunk; g.chunk_slabs = sh.chunk_slabs;
  g.b3 = b3; g.vtap = vtap; g.bfull = bfull; g.ldv = ldv; g.act = act; g.slope = slope;
  g.out = out; g.ldo = ld_out; g.yscale = yscale; g.flag = d_flag;
  if (head && head->n_head > 0) {
    // one block writes a pixel's running head sums: one output group only; <= 16 outputs
    if (head->n_head > 16 || sh.pl.ngroup != 1 || !head->w || (!head->acc && !ml) ||
        head->ldw < C + N || (uintptr_t)head->acc % 16)
      return IDF_ERR_ARG;
    const IdfHeadOut& o = head->out;
    if (head->last || ml) {
      if (o.mode == IDF_EPI_PRIOR ? (!o.mean || !o.logscale || !o.scale || o.n_mean < 0 ||
                                     2 * o.n_mean != head->n_head)
                                  : (!o.out || ((o.mode == IDF_EPI_COUPLE_ADD ||
                                                 o.mode == IDF_EPI_COUPLE_SUB) && !o.base)))
        return IDF_ERR_ARG;
    }
    g.hw = head->w; g.ldhw = head->ldw; g.nh = head->n_head; g.hacc = head->acc;
    g.hlast = head->last; g.skip_f32 = head->skip_f32; g.hmode = o.mode; g.hn_mean = o.n_mean;
    g.hout = o.out; g.hld_out = o.ld_out; g.hbase = o.base; g.hld_base = o.ld_base;
    g.hmean = o.mean; g.hlogs = o.logscale; g.hscale = o.scale;
  } else if (head && head->skip_f32) {
    g.skip_f32 = 1;
  }
  return IDF_OK;
}

// One dx3 launch (one layer).
static int dx3_run(void* stream, bool bf, int32_t B, int32_t H, int32_t W, int32_t C, uint16_t* xs,
                   int64_t xs_pix, int64_t xs_slab, int64_t xs_bytes, int32_t nslab_xs,
                   const uint16_t* w, int32_t nft, float yscale, const float* b3,
                   const float* vtap, int32_t ldv, const float* bfull, int32_t N, float* out,
                   int64_t ld_out, int32_t act, float slope, uint32_t* d_flag, void* d_workspace,
                   int64_t workspace_bytes, const IdfDx3Head* head) {
  if (B <= 0 || H <= 0 || W <= 0 || N <= 0) return IDF_OK;
  Dx3Args g;
  Dx3Launch sh;
  if (int rc = dx3_args(g, sh, false, bf, B, H, W, C, xs, xs_pix, xs_slab, xs_bytes, nslab_xs, w,
                        nft, yscale, b3, vtap, ldv, bfull, N, out, ld_out, act, slope, d_flag,
                        d_workspace, workspace_bytes, head))
    return rc;
  const int64_t nblk = (int64_t)sh.nblk_tiles * sh.pl.ngroup * sh.nchunk;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)nblk), blk(kDxThreads);
#define IDF_DX3_GO(nf_, wr_, pitch_, kib_) \
  hipLaunchKernelGGL((conv3_dx3_kernel<nf_, wr_, pitch_, kib_, false>), grid, blk, 0, s, g)
#define IDF_DXB_GO(nf_, wr_, pitch_, kib_) \
  hipLaunchKernelGGL((conv3_dx3_kernel<nf_, wr_, pitch_, kib_, true>), grid, blk, 0, s, g)
#define IDF_DX3_NF(wr_, pitch_, kib_)                      \
  switch (sh.pl.nf) {                                      \
    case 1: IDF_DX3_GO(1, wr_, pitch_, kib_); break;       \
    case 2: IDF_DX3_GO(2, wr_, pitch_, kib_); break;       \
    case 3: IDF_DX3_GO(3, wr_, pitch_, kib_); break;       \
    default: IDF_DX3_GO(4, wr_, pitch_, kib_); break;      \
  }
  constexpr int W2 = 16 / kDxWaves, W4 = 32 / kDxWaves;  // rows per wave: one tile / two tiles
  if (bf) {
#define IDF_DXB_NF(wr_, pitch_, kib_)                 \
  switch (sh.pl.nf) {                                 \
    case 1: IDF_DXB_GO(1, wr_, pitch_, kib_); break;  \
    case 2: IDF_DXB_GO(2, wr_, pitch_, kib_); break;  \
    default: IDF_DXB_GO(3, wr_, pitch_, kib_); break; \
  }
    if (sh.T == 2) {
      IDF_DXB_NF(W4, 18, 11)
    } else if (sh.pl.pitch == 18) {
      IDF_DXB_NF(W2, 18, 11)
    } else {
      IDF_DXB_NF(W2, 10, 13)
    }
#undef IDF_DXB_NF
  } else if (sh.T == 2) {
    switch (sh.pl.nf) {
      case 1: IDF_DX3_GO(1, W4, 18, 11); break;
      case 2: IDF_DX3_GO(2, W4, 18, 11); break;
      default: IDF_DX3_GO(3, W4, 18, 11); break;
    }
  } else if (sh.pl.pitch == 18) {
    IDF_DX3_NF(W2, 18, 11)
  } else if (sh.pl.pitch == 10) {
    IDF_DX3_NF(W2, 10, 13)
  } else if (sh.pl.pitch == 25) {
    IDF_DX3_NF(W2, 25, 15)
  } else {
    IDF_DX3_NF(W2, 6, 19)
  }
#undef IDF_DX3_NF
#undef IDF_DX3_GO
#undef IDF_DXB_GO
  return idf_last_error();
}


// tiles that hold whole images (no halo crosses a tile: a tile's layers need only its own earlier
// layers): one image per tile (16-wide images up to 16 rows) or the 4- / 8-wide segments, whose
// canvases hold whole images with zero gutters.  Not the split-K geometries (imagenet64's 8 x 8
// level): there one workgroup per tile runs every chunk of every layer in turn, measured 473 vs
// 308 us per DenseBlock (1.54x the per-layer launches' latency, bench -3%, profiles/r06/fused/).
static bool dx3_self_contained(const Dx3Plan& p, int H, int W) {
  if (!p.ok || p.gut || p.ngroup != 1 || p.split > 1) return false;
  if (W % 16 == 0) return W == 16 && H <= 16;
  return p.nby > 1 || H <= 16;
}

extern "C" int idf_dx3_block_supported(int32_t H, int32_t W, int32_t N, int32_t bf) {
  const Dx3Plan p = dx3_plan(H, W, N, bf != 0);
  if (bf && !dxb_plan_ok(p)) return 0;
  return dx3_self_contained(p, H, W) && (p.pitch == 18 || p.pitch == 10 || (!bf && p.pitch == 6));
}

int idf_dx3_block_launch(void* stream, const IdfDx3BlockDesc* d) {
  if (!d || d->nlayers < 1 || d->nlayers > kDxMaxLayers || !d->C || !d->w || !d->b3 || !d->feat)
    return IDF_ERR_ARG;
  if (d->B <= 0 || d->H <= 0 || d->W <= 0 || d->N <= 0) return IDF_OK;
  if (!idf_dx3_block_supported(d->H, d->W, d->N, d->bf)) return IDF_ERR_UNSUPPORTED;
  const bool bf = d->bf != 0;
  const int64_t P = (int64_t)d->B * d->H * d->W;
  const int64_t xs_slab = bf ? P * 32 : 2 * P * 32;
  const int64_t xs_bytes = bf ? idf_dxb_bytes(P, 16 * d->nslab_xs) : idf_dx3_split_bytes(P, 16 * d->nslab_xs);
  const bool fh = d->head && d->head->n_head > 0;
  if (fh && (!d->hx || !d->hb || d->hc0 < 0 || d->hc0 > 64 || (d->hc0 & 3) || (d->hld_x & 3) ||
             (uintptr_t)d->hx % 16 || (uintptr_t)d->head->w % 16 || (d->head->ldw & 3)))
    return IDF_ERR_ARG;
  Dx3Args g;
  Dx3Launch sh;
  IdfDx3Head h0 = {};
  if (fh) {
    h0 = *d->head;
    h0.last = d->nlayers == 1;
  }
  // the block's fields, checked and set from layer 0 (the plan depends on H, W, N only)
  if (int rc = dx3_args(g, sh, true, bf, d->B, d->H, d->W, d->C[0], d->xs, 32, xs_slab, xs_bytes,
                        d->nslab_xs, d->w[0], d->nft, bf ? 1.0f : d->yscale[0], d->b3[0],
                        d->vtap ? d->vtap[0] : nullptr, d->ldv, d->bfull ? d->bfull[0] : nullptr,
                        d->N, d->feat + d->C[0], d->ld_feat, d->act, d->slope, bf ? nullptr : d->flag,
                        nullptr, 0, fh ? &h0 : (d->head ? d->head : nullptr)))
    return rc;
  Dx3MLArgs ml = {};
  ml.nlayers = d->nlayers;
  for (int i = 0; i < d->nlayers; ++i) {
    const int C = d->C[i];
    if (C <= 0 || (C & 3) || !d->w[i] || !d->b3[i] || (C + 15) / 16 > d->nslab_xs) return IDF_ERR_ARG;
    if (d->vtap && d->vtap[i] && (!d->bfull || !d->bfull[i])) return IDF_ERR_ARG;
    if (fh && d->head->ldw < C + d->N) return IDF_ERR_ARG;
    const Dx3Launch li = dx3_launch_shape(d->B, d->H, d->W, C, d->N, bf);
    Dx3Layer& L = ml.layer[i];
    L.Wt = d->w[i]; L.b3 = d->b3[i]; L.vtap = d->vtap ? d->vtap[i] : nullptr;
    L.bfull = d->bfull ? d->bfull[i] : nullptr; L.out = d->feat + C;
    L.yscale = bf ? 1.0f : d->yscale[i];
    L.C = C; L.nslab = li.nslab; L.nchunk = li.nchunk; L.chunk_slabs = li.chunk_slabs;
    L.hlast = fh && i == d->nlayers - 1;
  }
  if (fh) {
    ml.hx = d->hx; ml.hld_x = d->hld_x; ml.hc0 = d->hc0; ml.hb = d->hb;
  }
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)sh.ntiles), blk(kDxThreads);
#define IDF_DX3B_GO(nf_, pitch_, kib_, bf_) \
  hipLaunchKernelGGL((conv3_dx3_block_kernel<nf_, pitch_, kib_, bf_>), grid, blk, 0, s, g, ml)
#define IDF_DX3B_NF(pitch_, kib_, bf_)                              \
  switch (sh.pl.nf) {                                              \
    case 1: IDF_DX3B_GO(1, pitch_, kib_, bf_); break;              \
    case 2: IDF_DX3B_GO(2, pitch_, kib_, bf_); break;              \
    case 3: IDF_DX3B_GO(3, pitch_, kib_, bf_); break;              \
    default: if (!bf_) IDF_DX3B_GO(4, pitch_, kib_, false); break; \
  }
  if (bf) {
    if (sh.pl.pitch == 18) IDF_DX3B_NF(18, 11, true)
    else IDF_DX3B_NF(10, 13, true)
  } else if (sh.pl.pitch == 18) {
    IDF_DX3B_NF(18, 11, false)
  } else if (sh.pl.pitch == 10) {
    IDF_DX3B_NF(10, 13, false)
  } else {
    IDF_DX3B_NF(6, 19, false)
  }
#undef IDF_DX3B_NF
#undef IDF_DX3B_GO
  return idf_last_error();
}

extern "C" int idf_conv3x3_dx3(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                               uint16_t* xs, int32_t nslab_xs, const uint16_t* w, int32_t nft,
                               float yscale, const float* b3, const float* vtap, int32_t ldv,
                               const float* bfull, int32_t N, float* out, int64_t ld_out,
                               int32_t act, float slope, uint32_t* d_flag, void* d_workspace,
                               int64_t workspace_bytes, const IdfDx3Head* head) {
  const int64_t P = (int64_t)B * H * W;
  return dx3_run(stream, false, B, H, W, C, xs, 32, 2 * P * 32, idf_dx3_split_bytes(P, 16 * nslab_xs),
                 nslab_xs, w, nft, yscale, b3, vtap, ldv, bfull, N, out, ld_out, act, slope, d_flag,
                 d_workspace, workspace_bytes, head);
}

extern "C" int64_t idf_dxb_bytes(int64_t P, int32_t channels) {
  if (P < 0 || channels < 0) return -1;
  return (int64_t)((channels + 15) / 16) * P * 32;
}

extern "C" int idf_dxb_cols(void* stream, int64_t P, int32_t c0, int32_t c1, const float* x,
                            int64_t ld_x, uint16_t* xb, int32_t nslab_xb, uint32_t* d_zero,
                            int32_t nzero) {
  if (P < 0 || c1 < c0 || nzero < 0 || (nzero && !d_zero)) return IDF_ERR_ARG;
  if (P == 0 || c1 == c0) {
    if (nzero) return hipMemsetAsync(d_zero, 0, 4 * (size_t)nzero, (hipStream_t)stream) == hipSuccess
                          ? IDF_OK : IDF_ERR_HIP;
    return IDF_OK;
  }
  if (!x || !xb || (c0 & 15) || (c1 & 3) || (ld_x & 3) || (uintptr_t)x % 16) return IDF_ERR_ARG;
  if ((c1 + 15) / 16 > nslab_xb) return IDF_ERR_ARG;
  int64_t n = P * (((c1 + 15) / 16 * 16 - c0) / 4);
  if (n < nzero) n = nzero;
  hipLaunchKernelGGL(dxb_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P, c0, c1, x, ld_x, xb, d_zero, nzero);
  return idf_last_error();
}

extern "C" int idf_conv3x3_dxb(void* stream, int32_t B, int32_t H, int32_t W, int32_t C,
                               uint16_t* xb, int32_t nslab_xb, const uint16_t* w, int32_t nft,
                               const float* b3, const float* vtap, int32_t ldv, const float* bfull,
                               int32_t N, float* out, int64_t ld_out, int32_t act, float slope,
                               void* d_workspace, int64_t workspace_bytes,
                               const IdfDx3Head* head) {
  if ((uintptr_t)xb % 16) return IDF_ERR_ARG;
  const int64_t P = (int64_t)B * H * W;
  return dx3_run(stream, true, B, H, W, C, xb, 32, P * 32, idf_dxb_bytes(P, 16 * nslab_xb), nslab_xb,
                 w, nft, 1.0f, b3, vtap, ldv, bfull, N, out, ld_out, act, slope, nullptr,
                 d_workspace, workspace_bytes, head);
}
