// Reproducer for the round-5 fused-head divergence (profiles/r05/fused_head/lds_coresidency.txt):
// the DenseBlock head init (conv3_dx3.hip dx3_head_init_kernel's arithmetic -- h[o] = bias[o],
// then c in order, fmaf(w[o][c], x[p][c], h[o])) with its 16 x 64 weight table staged in LDS and
// read by broadcast ds_read_b128, in four forms that differ ONLY in how the table fill is ordered
// before the block barrier:
//   1 ds_write fill, then s_barrier with no wait       (the LDS writes may still be in flight)
//   2 ds_write fill, s_waitcnt lgkmcnt(0), s_barrier    (correct)
//   3 LDS-DMA fill (buffer_load ... lds), s_barrier     (the DMA is counted by vmcnt: in flight)
//   4 LDS-DMA fill, s_waitcnt vmcnt(0), s_barrier       (correct)
// The barrier is written as inline asm so the compiler adds no wait of its own (a hardware
// s_barrier on gfx950 does not wait for the wave's outstanding memory operations); the committed
// ISA check (check_isa.py) proves which waits sit between the fill and the barrier.
// Timing-only test infrastructure: never linked into libidfcodec.so.
// Build: make -C tools/repro_lds   (-> tools/repro_lds/librepro_lds.so, gfx950)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

#pragma clang fp contract(off)

template <int V>
__global__ void __launch_bounds__(256) head_init_lds(int64_t P, int32_t C0, const float* __restrict__ x,
                                                     int64_t ld_x, const float* __restrict__ w,
                                                     int32_t ldw, const float* __restrict__ bias, int32_t nh,
                                                     float* __restrict__ acc) {
  __shared__ __attribute__((aligned(16))) float tab[16 * 64];
  const int tid = threadIdx.x;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + tid;
  // every kernel argument the thread needs is read before the fill, so no scalar-load wait
  // (lgkmcnt(0), which would also drain the LDS writes) falls between the fill and the barrier
  const int64_t pc = p < P ? p : P - 1;
  const float* xr = x + pc * ld_x;
  float h[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) h[o] = o < nh ? bias[o] : 0.0f;
  d4 x0 = *(const d4*)xr;  // the first channel quad in flight across the barrier
  asm volatile("" ::: "memory");
  if constexpr (V == 1 || V == 2) {
    // ds_write fill: 4 entries a thread, zeros past (nh, C0)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, o = e >> 6, c = e & 63;
      tab[e] = (o < nh && c < C0) ? w[o * ldw + c] : 0.0f;
    }
    if constexpr (V == 1) asm volatile("s_barrier" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    // LDS-DMA fill: wave k writes table bytes [1 KiB k, 1 KiB (k + 1)), lane l the entries
    // 256 k + 4 l .. + 3 (o, c .. c + 3), gathered from w's rows; entries past (nh, C0) read
    // an offset past the buffer's end, i.e. zeros
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int e = 256 * wave + 4 * lane, o = e >> 6, c = e & 63;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, nh * ldw * 4, 0x00020000);
    const uint32_t off = (o < nh && c < C0) ? (uint32_t)(o * ldw + c) * 4u : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)((char*)tab + 1024 * wave), 16, off, 0, 0, 0);
    if constexpr (V == 3) asm volatile("s_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (p >= P) return;
  for (int c = 0; c < C0; c += 4) {
    const d4 xv = c == 0 ? x0 : *(const d4*)(xr + c);
#pragma unroll
    for (int o = 0; o < 16; ++o) {
      if (o >= nh) break;
      const d4 wv = *(const d4*)(tab + o * 64 + c);  // uniform address: a broadcast read
#pragma unroll
      for (int k = 0; k < 4; ++k) h[o] = __builtin_fmaf(wv[k], xv[k], h[o]);
    }
  }
  d4* ap = (d4*)(acc + p * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) ap[i] = d4{h[4 * i], h[4 * i + 1], h[4 * i + 2], h[4 * i + 3]};
}

static int launch_variant(int variant, void* stream, int64_t P, int32_t C0, const float* x,
                          int64_t ld_x, const float* w, int32_t ldw, const float* bias, int32_t nh,
                          float* acc) {
  if (P <= 0 || C0 < 4 || C0 > 64 || (C0 & 3) || nh < 1 || nh > 16 || (ld_x & 3) || (ldw & 3)) return 1;
  const dim3 grid((unsigned)((P + 255) / 256)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 1: hipLaunchKernelGGL(head_init_lds<1>, grid, blk, 0, s, P, C0, x, ld_x, w, ldw, bias, nh, acc); break;
    case 2: hipLaunchKernelGGL(head_init_lds<2>, grid, blk, 0, s, P, C0, x, ld_x, w, ldw, bias, nh, acc); break;
    case 3: hipLaunchKernelGGL(head_init_lds<3>, grid, blk, 0, s, P, C0, x, ld_x, w, ldw, bias, nh, acc); break;
    case 4: hipLaunchKernelGGL(head_init_lds<4>, grid, blk, 0, s, P, C0, x, ld_x, w, ldw, bias, nh, acc); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// the four forms, called directly (run_repro.py: beside the product's dx3 block)
extern "C" int repro_head_init(int variant, void* stream, int64_t P, int32_t C0, const float* x,
                               int64_t ld_x, const float* w, int32_t ldw, const float* bias,
                               int32_t nh, float* acc) {
  return launch_variant(variant, stream, P, C0, x, ld_x, w, ldw, bias, nh, acc);
}

#ifdef IDF_HEAD_INIT_VARIANT
// a whole library with this form as its head init (Makefile: libidfcodec_v<N>.so, conv3_dx3.hip
// built with IDF_HEAD_INIT_EXTERNAL): the round-5 reduced case exactly, two fused blocks on two
// streams (tools/dbg_block_conc.py with IDF_LIB_PATH)
extern "C" int idf_dx3_head_init(void* stream, int64_t P, int32_t C0, const float* x, int64_t ld_x,
                                 const float* w, int32_t ldw, const float* bias, int32_t n_head,
                                 float* acc) {
  if (P <= 0) return P < 0 ? 1 : 0;
  return launch_variant(IDF_HEAD_INIT_VARIANT, stream, P, C0, x, ld_x, w, ldw, bias, n_head, acc) ? 2 : 0;
}
#endif
