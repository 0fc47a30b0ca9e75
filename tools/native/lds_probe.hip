// LDS bank-conflict probe (timing/counter tool, not part of the library): one block of 64
// lanes repeats one LDS access pattern; rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS per
// kernel instantiation tells which lane->address maps of conv3_wino.hip's epilogue conflict.
//   0 staging write b64, plain    (n = lane & 15, tile 4 * (lane >> 4), slot 2w)
//   1 staging write b64, swapped  (slot (2w) ^ (2 * ((lane >> 4) & 1)))
//   2 scalar read b128, e_grp/e_nn remap      3 scalar read b128, plain lane >> 4 / lane & 15
//   4 vector read b128 (v_t, v_nq, v_r)       5 write b64 at 2 * lane   6 read b128 at 4 * lane
//   7 staging write b64, slot (2w) ^ (2 * (n >> 3 & 1))    8 read b128 at 4 * (lane & 15)
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int TPI = 20, ERW = 64 * TPI + 4;

template <int PAT, int W>
__global__ void __launch_bounds__(64) lds_probe(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float lds[16 * ERW + 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 16 * ERW + 64; i += 64) lds[i] = (float)i;
  __syncthreads();
  int a = 0;
  if (PAT == 0 || PAT == 1 || PAT == 7) {
    const int lr = lane & 15, t = (lane >> 4) * 4;
    const int slot = PAT == 0 ? 2 * W : PAT == 1 ? (2 * W) ^ (2 * ((lane >> 4) & 1))
                                                 : (2 * W) ^ (2 * ((lr >> 3) & 1));
    a = lr * ERW + t * TPI + slot;
  } else if (PAT == 2 || PAT == 3) {
    int e_grp = lane >> 4 & 3, e_nn = lane & 15;
    if (PAT == 2) {
      const int m = lane & 31;
      const bool g0 = m < 4 || (m >= 12 && m < 16) || (m >= 20 && m < 28);
      e_grp = 2 * (lane >> 5) + (g0 ? 0 : 1);
      e_nn = m < 4 ? m : m < 12 ? m - 4 : m < 16 ? m - 8 : m < 20 ? m - 8 : m < 28 ? m - 12 : m - 16;
    }
    a = e_nn * ERW + (4 * W + e_grp) * TPI;
  } else if (PAT == 4) {
    const int v_t = 8 * W + (((lane >> 2) & 1) | (((lane >> 3) & 1) << 1) | ((lane & 1) << 2));
    const int v_nq = ((lane >> 4) & 1) | (((lane >> 1) & 1) << 1), v_r = (lane >> 5) & 1;
    a = (4 * v_nq) * ERW + v_t * TPI + 4 * v_r;
  } else if (PAT == 5) {
    a = 2 * lane;
  } else if (PAT == 6) {
    a = 4 * lane;
  } else {
    a = 4 * (lane & 15);
  }
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  // byte address in LDS; the accesses are inline asm so that the compiler neither hoists nor
  // splits them (a b128 it cannot prove aligned becomes two b64s)
  const unsigned ba = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)&lds[a];
  for (int it = 0; it < iters; ++it) {
    if (PAT == 0 || PAT == 1 || PAT == 5 || PAT == 7) {
      const f2 v = f2{(float)it, acc[0]};
      asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(ba), "v"(v) : "memory");
    } else {
      f4 v;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ba) : "memory");
      acc += v;
    }
  }
  out[lane] = acc[0] + acc[1] + acc[2] + acc[3] + lds[a];
}

int main() {
  float* out;
  if (hipMalloc(&out, 64 * 4) != hipSuccess) return 1;
  const int iters = 1000;
#define RUN(p, w) hipLaunchKernelGGL((lds_probe<p, w>), dim3(1), dim3(64), 0, 0, out, iters)
  RUN(0, 0); RUN(0, 1); RUN(1, 0); RUN(1, 1); RUN(2, 0); RUN(2, 1); RUN(3, 0); RUN(4, 0);
  RUN(5, 0); RUN(6, 0); RUN(7, 0); RUN(7, 1); RUN(8, 0);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("ok (%d iterations per probe; read the counters per kernel)\n", iters);
  return 0;
}
