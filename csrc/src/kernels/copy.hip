// Descriptor-driven strided box copies for gfx950 (see stencil/kernels/copy.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "stencil/kernels/copy.hpp"
#include "stencil/rt/hip_check.hpp"

namespace stencil {

static inline bool aligned(uint64_t v, uint32_t a) { return (v & (a - 1)) == 0; }

CopySeg make_copy_seg(const StridedBox &src, const StridedBox &dst, const Dim3 &ext, int64_t elemSize) {
  CopySeg s{};
  s.src = src.base;
  s.dst = dst.base;
  s.src_ystride = src.ystride;
  s.src_zstride = src.zstride;
  s.dst_ystride = dst.ystride;
  s.dst_zstride = dst.zstride;
  const uint64_t rowBytes = uint64_t(ext.x) * uint64_t(elemSize);
  uint32_t vec = 16;
  while (vec > 1) {
    if (aligned(rowBytes, vec) && aligned(uint64_t(uintptr_t(src.base)), vec) &&
        aligned(uint64_t(uintptr_t(dst.base)), vec) && aligned(uint64_t(src.ystride), vec) &&
        aligned(uint64_t(src.zstride), vec) && aligned(uint64_t(dst.ystride), vec) && aligned(uint64_t(dst.zstride), vec))
      break;
    vec >>= 1;
  }
  s.vec = vec;
  s.row_units = uint32_t(rowBytes / vec);
  s.ny = uint32_t(ext.y);
  s.units = (ext.x > 0 && ext.y > 0 && ext.z > 0) ? uint64_t(s.row_units) * uint64_t(ext.y) * uint64_t(ext.z) : 0;
  return s;
}

uint64_t finalize_segs(std::vector<CopySeg> &segs) {
  // drop empty segments, keep order
  segs.erase(std::remove_if(segs.begin(), segs.end(), [](const CopySeg &s) { return s.units == 0; }), segs.end());
  uint64_t acc = 0;
  for (auto &s : segs) {
    s.unit_begin = acc;
    acc += s.units;
  }
  return acc;
}

void copy_segs_host(const std::vector<CopySeg> &segs) {
  for (const auto &s : segs) {
    if (!s.units) continue;
    const uint64_t rowBytes = uint64_t(s.row_units) * s.vec;
    const uint64_t rows = s.units / s.row_units;
    for (uint64_t r = 0; r < rows; ++r) {
      const uint64_t y = r % s.ny, z = r / s.ny;
      std::memmove(s.dst + z * s.dst_zstride + y * s.dst_ystride, s.src + z * s.src_zstride + y * s.src_ystride,
                   rowBytes);
    }
  }
}

template <uint32_t V> struct VecOf;
template <> struct VecOf<16> { using T = uint4; };
template <> struct VecOf<8> { using T = uint2; };
template <> struct VecOf<4> { using T = uint32_t; };
template <> struct VecOf<2> { using T = uint16_t; };
template <> struct VecOf<1> { using T = uint8_t; };

template <uint32_t V> __device__ __forceinline__ void copy_unit(char *dst, const char *src) {
  using T = typename VecOf<V>::T;
  *reinterpret_cast<T *>(dst) = *reinterpret_cast<const T *>(src);
}

// One launch walks every segment. Units are assigned with a grid-stride loop over the flattened unit space;
// the owning segment is found by binary search over unit_begin (segments are few and L1/L2 resident).
// All index math past the segment base is 32-bit (a segment holds < 2^32 units) to keep VALU cost per 16-B unit
// well under the HBM-bound budget.
__global__ __launch_bounds__(256) void copy_segs_kernel(const CopySeg *__restrict__ segs, int nsegs, uint64_t total) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t u = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; u < total; u += stride) {
    int lo = 0, hi = nsegs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (segs[mid].unit_begin <= u)
        lo = mid;
      else
        hi = mid - 1;
    }
    const CopySeg &s = segs[lo];
    const uint32_t lu = uint32_t(u - s.unit_begin);
    const uint32_t c = lu % s.row_units;
    const uint32_t r = lu / s.row_units;
    const uint32_t y = r % s.ny;
    const uint32_t z = r / s.ny;
    const uint32_t vec = s.vec;
    const char *sp = s.src + int64_t(z) * s.src_zstride + int64_t(y) * s.src_ystride + uint64_t(c) * vec;
    char *dp = s.dst + int64_t(z) * s.dst_zstride + int64_t(y) * s.dst_ystride + uint64_t(c) * vec;
    switch (vec) {
    case 16:
      copy_unit<16>(dp, sp);
      break;
    case 8:
      copy_unit<8>(dp, sp);
      break;
    case 4:
      copy_unit<4>(dp, sp);
      break;
    case 2:
      copy_unit<2>(dp, sp);
      break;
    default:
      copy_unit<1>(dp, sp);
      break;
    }
  }
}

void copy_segs_device(const CopySeg *dsegs, int nsegs, uint64_t totalUnits, hipStream_t stream) {
  if (!nsegs || !totalUnits) return;
  const int threads = 256;
  // enough blocks to cover the units, capped at 8 blocks/CU over 256 CUs (grid-stride for the rest)
  const uint64_t want = (totalUnits + threads - 1) / threads;
  const int blocks = int(std::min<uint64_t>(want, 2048));
  hipLaunchKernelGGL(copy_segs_kernel, dim3(blocks), dim3(threads), 0, stream, dsegs, nsegs, totalUnits);
  HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// device flags
// ------------------------------------------------------------------------------------------------
struct FlagList {
  uint64_t *p[kMaxFlagsPerLaunch];
  int n;
};

__global__ void wait_flags_kernel(FlagList f, uint64_t target, int *err, int code, uint64_t timeoutTicks) {
  const int i = threadIdx.x;
  if (i < f.n) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime(); // 100 MHz constant clock
    while (true) {
      const uint64_t v = __hip_atomic_load(f.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v >= target) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeoutTicks) {
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
}

__global__ void signal_flags_kernel(FlagList f, uint64_t value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); // system scope: prior kernels' peer stores are ordered before
  const int i = threadIdx.x;
  if (i < f.n) __hip_atomic_store(f.p[i], value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static FlagList to_list(const std::vector<uint64_t *> &flags) {
  STENCIL_REQUIRE(flags.size() <= size_t(kMaxFlagsPerLaunch), "too many flags in one launch: " << flags.size());
  FlagList f{};
  f.n = int(flags.size());
  for (size_t i = 0; i < flags.size(); ++i) f.p[i] = flags[i];
  return f;
}

void wait_flags_device(const std::vector<uint64_t *> &flags, uint64_t target, int *err, int code, double timeout_s,
                       hipStream_t stream) {
  if (flags.empty()) return;
  const uint64_t ticks = uint64_t(timeout_s * 1e8);
  hipLaunchKernelGGL(wait_flags_kernel, dim3(1), dim3(64), 0, stream, to_list(flags), target, err, code, ticks);
  HIP_CHECK(hipGetLastError());
}

void signal_flags_device(const std::vector<uint64_t *> &flags, uint64_t value, hipStream_t stream) {
  if (flags.empty()) return;
  hipLaunchKernelGGL(signal_flags_kernel, dim3(1), dim3(64), 0, stream, to_list(flags), value);
  HIP_CHECK(hipGetLastError());
}

} // namespace stencil
