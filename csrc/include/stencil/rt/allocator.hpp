#pragma once
// STL allocators over HIP memory: device (hipMalloc on a chosen GPU), managed (hipMallocManaged) and pinned host
// (hipHostMalloc, portable + coherent, used for host-staged transfers).
// Parity: reference include/stencil/device_allocator.hpp:7-64 (DeviceAllocator over cudaMalloc on a given GPU)
// and managed_allocator.hpp:7-64 (ManagedAllocator over cudaMallocManaged). Both are stateless in the reference
// except for the device; here equality also compares the device so containers never free on the wrong GPU.
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <limits>
#include <new>

#include "stencil/rt/hip_check.hpp"

namespace stencil {

namespace detail {
// allocate with `dev` current, restoring the caller's device afterwards
template <typename F> inline void *with_device(int dev, F &&f) {
  int prev = 0;
  HIP_CHECK(hipGetDevice(&prev));
  if (dev >= 0) HIP_CHECK(hipSetDevice(dev));
  void *p = f();
  if (dev >= 0) HIP_CHECK(hipSetDevice(prev));
  return p;
}
} // namespace detail

// Device memory on GPU `dev` (-1 = current device). Elements are never constructed on the host: use with
// containers of trivially constructible types only (std::vector<T, DeviceAllocator<T>> v(n) must not be used to
// value-initialise; use reserve() + a device fill, or Array<T> below).
template <typename T> class DeviceAllocator {
public:
  using value_type = T;
  int dev = -1;
  DeviceAllocator() noexcept = default;
  explicit DeviceAllocator(int d) noexcept : dev(d) {}
  template <typename U> DeviceAllocator(const DeviceAllocator<U> &o) noexcept : dev(o.dev) {}
  T *allocate(size_t n) {
    if (n > std::numeric_limits<size_t>::max() / sizeof(T)) throw std::bad_array_new_length();
    return static_cast<T *>(detail::with_device(dev, [&] {
      void *p = nullptr;
      HIP_CHECK(hipMalloc(&p, n * sizeof(T)));
      return p;
    }));
  }
  void deallocate(T *p, size_t) noexcept { (void)hipFree(p); }
  template <typename U> bool operator==(const DeviceAllocator<U> &o) const noexcept { return dev == o.dev; }
  template <typename U> bool operator!=(const DeviceAllocator<U> &o) const noexcept { return dev != o.dev; }
};

// Unified (managed) memory, accessible from host and device; attached to GPU `dev` at allocation time.
template <typename T> class ManagedAllocator {
public:
  using value_type = T;
  int dev = -1;
  ManagedAllocator() noexcept = default;
  explicit ManagedAllocator(int d) noexcept : dev(d) {}
  template <typename U> ManagedAllocator(const ManagedAllocator<U> &o) noexcept : dev(o.dev) {}
  T *allocate(size_t n) {
    if (n > std::numeric_limits<size_t>::max() / sizeof(T)) throw std::bad_array_new_length();
    return static_cast<T *>(detail::with_device(dev, [&] {
      void *p = nullptr;
      HIP_CHECK(hipMallocManaged(&p, n * sizeof(T), hipMemAttachGlobal));
      return p;
    }));
  }
  void deallocate(T *p, size_t) noexcept { (void)hipFree(p); }
  template <typename U> bool operator==(const ManagedAllocator<U> &o) const noexcept { return dev == o.dev; }
  template <typename U> bool operator!=(const ManagedAllocator<U> &o) const noexcept { return dev != o.dev; }
};

// Page-locked host memory (DMA-able by every GPU of the node): the staging buffers of the host-staged transport.
template <typename T> class PinnedAllocator {
public:
  using value_type = T;
  PinnedAllocator() noexcept = default;
  template <typename U> PinnedAllocator(const PinnedAllocator<U> &) noexcept {}
  T *allocate(size_t n) {
    if (n > std::numeric_limits<size_t>::max() / sizeof(T)) throw std::bad_array_new_length();
    void *p = nullptr;
    HIP_CHECK(hipHostMalloc(&p, n * sizeof(T), hipHostMallocPortable));
    return static_cast<T *>(p);
  }
  void deallocate(T *p, size_t) noexcept { (void)hipHostFree(p); }
  template <typename U> bool operator==(const PinnedAllocator<U> &) const noexcept { return true; }
  template <typename U> bool operator!=(const PinnedAllocator<U> &) const noexcept { return false; }
};

} // namespace stencil
