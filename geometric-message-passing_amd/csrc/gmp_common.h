// Shared helpers for the gfx950 kernels of libgmp (HIP, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gmp.h"

namespace gmp {

// last HIP error seen by any entry point (diagnostics only)
extern thread_local int g_last_hip_error;

inline int hip_check(hipError_t e) {
  if (e != hipSuccess) {
    g_last_hip_error = static_cast<int>(e);
    return GMP_ERR_HIP;
  }
  return GMP_OK;
}

inline int launch_status() { return hip_check(hipGetLastError()); }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Number of CUs on the device the stream belongs to (cached per process; MI355X: 256).
int device_cu_count();

}  // namespace gmp

#define GMP_CHECK_ARG(cond) \
  do {                      \
    if (!(cond)) return GMP_ERR_ARG; \
  } while (0)
