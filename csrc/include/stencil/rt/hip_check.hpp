#pragma once
// HIP error checking. Parity: reference include/stencil/cuda_runtime.hpp:8-17 (checkCuda / CUDA_RUNTIME /
// CudaErrorsFatal). Errors are rank-tagged and throw stencil::Error instead of exit(-1).
#include <hip/hip_runtime_api.h>

#include "stencil/rt/logging.hpp"

enum class HipErrorsFatal { NO, YES };

#define HIP_CHECK(stmt)                                                                                            \
  do {                                                                                                             \
    hipError_t _e = (stmt);                                                                                        \
    if (_e != hipSuccess) {                                                                                        \
      (void)hipGetLastError(); /* a caught failure must not resurface in the next hipGetLastError() check */       \
      LOG_FATAL("HIP error " << int(_e) << " (" << hipGetErrorString(_e) << ") in `" #stmt "`");                    \
    }                                                                                                              \
  } while (0)

// non-fatal variant: logs and returns the error
#define HIP_TRY(stmt)                                                                                              \
  ([&]() {                                                                                                         \
    hipError_t _e = (stmt);                                                                                        \
    if (_e != hipSuccess) (void)hipGetLastError();                                                                 \
    if (_e != hipSuccess) LOG_DEBUG("HIP error " << int(_e) << " (" << hipGetErrorString(_e) << ") in `" #stmt "`"); \
    return _e;                                                                                                     \
  }())
