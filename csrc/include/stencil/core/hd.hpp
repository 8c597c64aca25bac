#pragma once
// Host/device qualifier shim for headers shared by host-only TUs (g++/pybind11) and
// hipcc device TUs. Only the qualifiers are switched; there is no second code path.
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define STENCIL_HD __host__ __device__
#define STENCIL_DEVICE_COMPILE 1
#else
#define STENCIL_HD
#define STENCIL_DEVICE_COMPILE 0
#endif

#define STENCIL_HDI STENCIL_HD inline
