// idf_codec_internal.h -- shared internals of libidfcodec (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/idf_codec.h"

// marker written by rans_cdf_freq for scale == 0 (freq can never be INT32_MIN)
#define IDF_FREQ_SCALE_ZERO ((int32_t)0x80000000)

static inline int idf_last_error() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? IDF_OK : IDF_ERR_HIP;
}
