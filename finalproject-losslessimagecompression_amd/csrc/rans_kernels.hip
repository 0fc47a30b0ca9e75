// rans_kernels.hip -- CDNA4 (gfx950) rANS coder, bit-identical to the
// reference Cython coder (/root/reference/rans/rans.pyx:37-110) per stream.
//
// A "stream" is one reference encode()/decode() call: symbols
// [sym_off[k], sym_off[k+1]) coded from init_state[k].  Many independent
// streams run at once (one reference-format stream per lane/wave).
//
// Kernels
//   rans_cdf_freq   : pass 1 of encode (rans.pyx:50-56), one thread per symbol,
//                     fully parallel, HBM-bound (12 B in, 8 B out per symbol).
//   rans_encode     : pass 2 (rans.pyx:61-66), one lane per stream; the serial
//                     state chain with an exact 64/24-bit division done by a
//                     double-precision reciprocal estimate plus integer correction.
//   rans_decode     : rans.pyx:69-110, ONE WAVE per stream.  The reference's
//                     11-12 step binary search over the 2048-bin window is
//                     replaced by a two-round 64-ary search (round 1: 64 lanes
//                     probe the last bin of each 32-bin block; round 2: 33 lanes
//                     probe the chosen block and its left neighbour).  The CDF is
//                     strictly increasing in s for scale > 0 (part2 steps by 1,
//                     part1 is monotone: glibc expf verified monotone on every
//                     float), so both searches return the same s; scale <= 0 or
//                     NaN falls back to the reference's serial binary search.
//   gather_words    : compacts per-stream word runs into one contiguous buffer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "idf_cdf.h"
#include "idf_codec_internal.h"

#pragma clang fp contract(off)

namespace idf {

static constexpr uint64_t kRansL = 0x100000000ull;

__device__ __forceinline__ void window_check(float x, int lower, int32_t* flag) {
  // symbol index s = x*256 must satisfy lower <= s <= lower+2047 to round-trip
  float s = x * 256.0f;
  if (!(s >= (float)lower && s <= (float)(lower + 2047))) *flag |= IDF_STREAM_OUT_OF_WINDOW;
}

// ---------------------------------------------------------------- pass 1
__global__ void __launch_bounds__(256) rans_cdf_freq_kernel(int64_t n, const float* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ scale,
                                                            int32_t* __restrict__ start,
                                                            int32_t* __restrict__ freq) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float xi = x[i], mi = mean[i], si = scale[i];
  if (si == 0.0f) {  // ZeroDivisionError("float division"), rans.cpp:1435-1438
    start[i] = 0;
    freq[i] = IDF_FREQ_SCALE_ZERO;
    return;
  }
  int lo = rans_lower_int(mi);
  float lower = rans_lower_f(lo);  // rans.pyx:51
  float xm = (float)((double)xi - 1.0 / 256.0);
  int s = rans_cdf(xm, mi, si, lower);  // rans.pyx:52
  int e = rans_cdf(xi, mi, si, lower);  // rans.pyx:53
  start[i] = s;
  freq[i] = e - s;
}

// ---------------------------------------------------------------- pass 2
// Exact q = state / f, r = state % f for f in [1, 2^24], state < 2^64 with q < 2^40
// (guaranteed after renormalisation).  The double estimate is within +-1.
__device__ __forceinline__ void divmod_u64_u24(uint64_t state, uint32_t f, double rcp, uint64_t& q,
                                               uint64_t& r) {
  uint64_t qe = (uint64_t)((double)state * rcp);
  int64_t rr = (int64_t)(state - qe * (uint64_t)f);
  if (rr < 0) {
    qe -= 1;
    rr += f;
  } else if (rr >= (int64_t)f) {
    qe += 1;
    rr -= f;
  }
  q = qe;
  r = (uint64_t)rr;
}

__global__ void __launch_bounds__(64) rans_encode_kernel(
    int64_t nstreams, const int64_t* __restrict__ sym_off, const float* __restrict__ x,
    const float* __restrict__ mean, const int32_t* __restrict__ start,
    const int32_t* __restrict__ freq, const uint64_t* __restrict__ init_state,
    uint64_t* __restrict__ final_state, uint32_t* __restrict__ words, int64_t* __restrict__ nwords,
    int32_t* __restrict__ status) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nstreams) return;
  const int64_t b = sym_off[k], e = sym_off[k + 1];
  uint64_t state = init_state[k];
  uint32_t* out = words + b;
  int64_t nw = 0;
  int32_t flag = 0;
  for (int64_t i = b; i < e; ++i) {
    int32_t st = start[i];
    int32_t fr = freq[i];
    if (fr == IDF_FREQ_SCALE_ZERO && st == 0) {
      flag |= IDF_STREAM_SCALE_ZERO;
      break;
    }
    uint64_t cdf = (uint64_t)(int64_t)st;  // vector<ull>.push_back(int)
    uint64_t f = (uint64_t)(int64_t)fr;
    if (state >= (f << 40)) {  // rans.pyx:62-64
      out[nw++] = (uint32_t)(state & 0xffffffffull);
      state >>= 32;
    }
    if (f == 0) {  // ZeroDivisionError, rans.cpp:1825-1834
      flag |= IDF_STREAM_FREQ_ZERO;
      break;
    }
    uint64_t q, r;
    if (f <= (1ull << 24)) {
      divmod_u64_u24(state, (uint32_t)f, 1.0 / (double)(uint32_t)f, q, r);
    } else {  // only reachable out of window / corrupted input: exact slow path
      q = state / f;
      r = state % f;
    }
    state = (q << 24) + r + cdf;  // rans.pyx:65
    window_check(x[i], rans_lower_int(mean[i]), &flag);
  }
  final_state[k] = state;
  nwords[k] = nw;
  status[k] = flag;
}

// ---------------------------------------------------------------- decode
__device__ __forceinline__ float sym_x(int s) { return (float)((double)s / 256.0); }

// Reference binary search (rans.pyx:96-104) for the non-monotone corner
// (scale <= 0 or NaN).  Returns s and flags.
__device__ int ref_binary_search(uint64_t mod, int lower, float mean, float scale, float lf,
                                 int32_t* flag) {
  int upper = lower + 0x7FF;
  while (lower <= upper) {
    int s = (lower + upper) >> 1;
    int c = rans_cdf(sym_x(s), mean, scale, lf);
    if (c < 0) *flag |= IDF_STREAM_NEG_CDF;
    if ((uint64_t)(int64_t)c > mod) upper = s - 1;
    else lower = s + 1;
  }
  return lower;
}

__global__ void __launch_bounds__(64) rans_decode_kernel(
    int64_t nstreams, const int64_t* __restrict__ sym_off, const int64_t* __restrict__ word_off,
    const int64_t* __restrict__ nwords, const uint32_t* __restrict__ words,
    const float* __restrict__ mean, const float* __restrict__ scale,
    const uint64_t* __restrict__ init_state, uint64_t* __restrict__ final_state,
    float* __restrict__ out, int32_t* __restrict__ status) {
  const int64_t k = blockIdx.x;
  if (k >= nstreams) return;
  const int lane = threadIdx.x;
  const int64_t b = sym_off[k], n = sym_off[k + 1] - b;
  const uint32_t* w = words + word_off[k];
  int64_t pos = nwords[k];
  uint64_t state = init_state[k];
  int32_t flag = 0;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t i = b + n - 1 - j;
    if (state < kRansL) {  // rans.pyx:86-89 (buffer read in reverse)
      if (pos <= 0) {
        flag |= IDF_STREAM_UNDERFLOW;
        break;
      }
      state = (state << 32) | (uint64_t)w[--pos];
    }
    const uint64_t mod = state & 0xffffffull;
    const float mi = mean[i], si = scale[i];
    const int lower = rans_lower_int(mi);  // rans.pyx:91
    const float lf = rans_lower_f(lower);  // rans.pyx:93
    int s;
    int c_lo, c_hi;
    if (!(si > 0.0f)) {
      if (si == 0.0f) {
        flag |= IDF_STREAM_SCALE_ZERO;
        break;
      }
      s = ref_binary_search(mod, lower, mi, si, lf, &flag);
      c_lo = rans_cdf(sym_x(s - 1), mi, si, lf);
      c_hi = rans_cdf(sym_x(s), mi, si, lf);
    } else {
      // round 1: lane L probes the last bin of block L
      int p1 = lower + 32 * lane + 31;
      int c1 = rans_cdf(sym_x(p1), mi, si, lf);
      uint64_t m1 = __ballot((uint64_t)(int64_t)c1 > mod);
      if (m1 == 0) {
        // no bin in the window has CDF > mod: reference leaves s = lower + 2048
        s = lower + 2048;
        int q = s - 1 + (lane & 1);
        int cq = rans_cdf(sym_x(q), mi, si, lf);
        c_lo = __shfl(cq, 0);
        c_hi = __shfl(cq, 1);
      } else {
        int blk = __ffsll((unsigned long long)m1) - 1;
        int base = lower + 32 * blk - 1;  // probe base-1 .. base+31 (33 points)
        int q = base + (lane <= 32 ? lane : 32);
        int cq = rans_cdf(sym_x(q), mi, si, lf);
        uint64_t m2 = __ballot(lane >= 1 && lane <= 32 && (uint64_t)(int64_t)cq > mod);
        int kk = __ffsll((unsigned long long)m2) - 1;  // >= 1
        s = base + kk;
        c_lo = __shfl(cq, kk - 1);
        c_hi = __shfl(cq, kk);
      }
    }
    if (c_lo < 0 || c_hi - c_lo < 0) flag |= IDF_STREAM_NEG_CDF;
    const uint64_t cdf_s = (uint64_t)(int64_t)c_lo;
    const uint64_t freq_s = (uint64_t)(int64_t)(c_hi - c_lo);
    state = (state >> 24) * freq_s + (state & 0xffffffull) - cdf_s;  // rans.pyx:108
    if (lane == 0) out[i] = sym_x(s);  // message.push_back(s / 256.)
  }
  if (lane == 0) {
    final_state[k] = state;
    status[k] = flag | (pos != 0 ? IDF_STREAM_WORDS_LEFT : 0);
  }
}

// ---------------------------------------------------------------- compaction
__global__ void __launch_bounds__(256) gather_words_kernel(int64_t nstreams,
                                                           const int64_t* __restrict__ src_off,
                                                           const int64_t* __restrict__ nwords,
                                                           const int64_t* __restrict__ dst_off,
                                                           const uint32_t* __restrict__ src,
                                                           uint32_t* __restrict__ dst) {
  int64_t k = blockIdx.x;
  if (k >= nstreams) return;
  const uint32_t* s = src + src_off[k];
  uint32_t* d = dst + dst_off[k];
  for (int64_t i = threadIdx.x; i < nwords[k]; i += blockDim.x) d[i] = s[i];
}

__global__ void expf_kernel(int64_t n, const float* __restrict__ in, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = expf_glibc(in[i]);
}

// Exhaustive device check: order-independent checksum over a range of float
// bit patterns, same formula as tests/native/expf_check.cpp.
__global__ void __launch_bounds__(256) expf_checksum_kernel(uint64_t lo, uint64_t hi,
                                                            unsigned long long* acc) {
  uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long sum = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (; i < hi; i += stride) {
    float a = expf_glibc(u2f((uint32_t)i));
    uint32_t h = (a != a) ? 0x7fc00000u : f2u(a);
    sum += (unsigned long long)h * ((uint64_t)i * 2654435761ull | 1ull);
  }
  // wave reduce
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_down(sum, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(acc, sum);
}

}  // namespace idf

// ============================================================== C-ABI
using namespace idf;

extern "C" {

int idf_rans_cdf_freq(void* stream, int64_t n, const float* x, const float* mean,
                      const float* scale, int32_t* start, int32_t* freq) {
  if (n < 0) return IDF_ERR_ARG;
  if (n == 0) return IDF_OK;
  int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(rans_cdf_freq_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, n, x, mean, scale, start, freq);
  return idf_last_error();
}

int64_t idf_rans_encode_workspace_bytes(int64_t nsym) {
  return 2 * (int64_t)sizeof(int32_t) * (nsym > 0 ? nsym : 1);
}

int idf_rans_encode_streams(void* stream, int64_t nstreams, int64_t nsym, const int64_t* sym_off,
                            const float* x, const float* mean, const float* scale,
                            const uint64_t* init_state, uint64_t* final_state, uint32_t* words,
                            int64_t* nwords, int32_t* status, void* workspace,
                            int64_t workspace_bytes) {
  if (nstreams < 0 || nsym < 0) return IDF_ERR_ARG;
  if (nstreams == 0) return IDF_OK;
  if (workspace_bytes < idf_rans_encode_workspace_bytes(nsym)) return IDF_ERR_WORKSPACE;
  int32_t* st = (int32_t*)workspace;
  int32_t* fr = st + (nsym > 0 ? nsym : 1);
  int rc = idf_rans_cdf_freq(stream, nsym, x, mean, scale, st, fr);
  if (rc) return rc;
  int64_t blocks = (nstreams + 63) / 64;
  hipLaunchKernelGGL(rans_encode_kernel, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream,
                     nstreams, sym_off, x, mean, st, fr, init_state, final_state, words, nwords,
                     status);
  return idf_last_error();
}

int idf_rans_decode_streams(void* stream, int64_t nstreams, const int64_t* sym_off,
                            const int64_t* word_off, const int64_t* nwords, const uint32_t* words,
                            const float* mean, const float* scale, const uint64_t* init_state,
                            uint64_t* final_state, float* out, int32_t* status) {
  if (nstreams < 0) return IDF_ERR_ARG;
  if (nstreams == 0) return IDF_OK;
  hipLaunchKernelGGL(rans_decode_kernel, dim3((unsigned)nstreams), dim3(64), 0,
                     (hipStream_t)stream, nstreams, sym_off, word_off, nwords, words, mean, scale,
                     init_state, final_state, out, status);
  return idf_last_error();
}

int idf_gather_words(void* stream, int64_t nstreams, const int64_t* src_off, const int64_t* nwords,
                     const int64_t* dst_off, const uint32_t* src, uint32_t* dst) {
  if (nstreams < 0) return IDF_ERR_ARG;
  if (nstreams == 0) return IDF_OK;
  hipLaunchKernelGGL(gather_words_kernel, dim3((unsigned)nstreams), dim3(256), 0,
                     (hipStream_t)stream, nstreams, src_off, nwords, dst_off, src, dst);
  return idf_last_error();
}

int idf_expf_glibc(void* stream, int64_t n, const float* in, float* out) {
  if (n <= 0) return n < 0 ? IDF_ERR_ARG : IDF_OK;
  hipLaunchKernelGGL(expf_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, n, in, out);
  return idf_last_error();
}

int idf_expf_checksum(void* stream, uint64_t lo, uint64_t hi, unsigned long long* acc) {
  hipLaunchKernelGGL(expf_checksum_kernel, dim3(8192), dim3(256), 0, (hipStream_t)stream, lo, hi,
                     acc);
  return idf_last_error();
}

// ---- host-buffer convenience: exactly one reference call (rans.pyx:37 / :69)
#define CK(expr)                                   \
  do {                                             \
    if ((expr) != hipSuccess && rc == IDF_OK) rc = IDF_ERR_HIP; \
  } while (0)
int idf_rans_encode(uint64_t* state_io, int64_t n, const float* x, const float* mean,
                    const float* scale, uint32_t* words, int64_t* nwords_out, int32_t* status_out) {
  if (n < 0 || !state_io) return IDF_ERR_ARG;
  hipStream_t s = nullptr;
  int64_t nn = n > 0 ? n : 1;
  int rc = IDF_OK;
  char* dbuf = nullptr;
  size_t bytes = 3 * nn * 4 + 2 * 8 + 8 + 8 + 8 + 4 + nn * 4 + (size_t)idf_rans_encode_workspace_bytes(n) + 64;
  if (hipMalloc(&dbuf, bytes) != hipSuccess) return IDF_ERR_HIP;
  char* p = dbuf;
  auto take = [&](size_t b) { char* r = p; p += (b + 15) & ~(size_t)15; return r; };
  float* dx = (float*)take(nn * 4);
  float* dm = (float*)take(nn * 4);
  float* ds = (float*)take(nn * 4);
  int64_t* doff = (int64_t*)take(16);
  uint64_t* dst = (uint64_t*)take(8);
  uint64_t* dfs = (uint64_t*)take(8);
  int64_t* dnw = (int64_t*)take(8);
  int32_t* dstat = (int32_t*)take(4);
  uint32_t* dw = (uint32_t*)take(nn * 4);
  void* ws = take((size_t)idf_rans_encode_workspace_bytes(n));
  int64_t off[2] = {0, n};
  if (n > 0) {
    CK(hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dm, mean, n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ds, scale, n * 4, hipMemcpyHostToDevice));
  }
  CK(hipMemcpy(doff, off, 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dst, state_io, 8, hipMemcpyHostToDevice));
  if (rc == IDF_OK)
    rc = idf_rans_encode_streams(s, 1, n, doff, dx, dm, ds, dst, dfs, dw, dnw, dstat, ws,
                               idf_rans_encode_workspace_bytes(n));
  int64_t nw = 0;
  int32_t stat = 0;
  if (rc == IDF_OK) {
    CK(hipMemcpy(state_io, dfs, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&nw, dnw, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&stat, dstat, 4, hipMemcpyDeviceToHost));
    if (nw > 0) CK(hipMemcpy(words, dw, nw * 4, hipMemcpyDeviceToHost));
    if (hipDeviceSynchronize() != hipSuccess) rc = IDF_ERR_HIP;
  }
  CK(hipFree(dbuf));
  if (nwords_out) *nwords_out = nw;
  if (status_out) *status_out = stat;
  return rc;
}

int idf_rans_decode(uint64_t* state_io, const uint32_t* words, int64_t nwords, int64_t n,
                    const float* mean, const float* scale, float* out, int32_t* status_out) {
  if (n < 0 || nwords < 0 || !state_io) return IDF_ERR_ARG;
  int64_t nn = n > 0 ? n : 1, nwn = nwords > 0 ? nwords : 1;
  int rc = IDF_OK;
  char* dbuf = nullptr;
  size_t bytes = 3 * nn * 4 + nwn * 4 + 16 + 8 * 4 + 4 + 128;
  if (hipMalloc(&dbuf, bytes) != hipSuccess) return IDF_ERR_HIP;
  char* p = dbuf;
  auto take = [&](size_t b) { char* r = p; p += (b + 15) & ~(size_t)15; return r; };
  float* dm = (float*)take(nn * 4);
  float* ds = (float*)take(nn * 4);
  float* dout = (float*)take(nn * 4);
  uint32_t* dw = (uint32_t*)take(nwn * 4);
  int64_t* doff = (int64_t*)take(16);
  int64_t* dwoff = (int64_t*)take(8);
  int64_t* dnw = (int64_t*)take(8);
  uint64_t* dst = (uint64_t*)take(8);
  uint64_t* dfs = (uint64_t*)take(8);
  int32_t* dstat = (int32_t*)take(4);
  int64_t off[2] = {0, n}, zero = 0;
  if (n > 0) {
    CK(hipMemcpy(dm, mean, n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ds, scale, n * 4, hipMemcpyHostToDevice));
  }
  if (nwords > 0) CK(hipMemcpy(dw, words, nwords * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(doff, off, 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dwoff, &zero, 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dnw, &nwords, 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dst, state_io, 8, hipMemcpyHostToDevice));
  if (rc == IDF_OK) rc = idf_rans_decode_streams(nullptr, 1, doff, dwoff, dnw, dw, dm, ds, dst, dfs, dout, dstat);
  int32_t stat = 0;
  if (rc == IDF_OK) {
    CK(hipMemcpy(state_io, dfs, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&stat, dstat, 4, hipMemcpyDeviceToHost));
    if (n > 0) CK(hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost));
    if (hipDeviceSynchronize() != hipSuccess) rc = IDF_ERR_HIP;
  }
  CK(hipFree(dbuf));
  if (status_out) *status_out = stat;
  return rc;
}

}  // extern "C"
