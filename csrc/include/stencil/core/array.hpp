#pragma once
// Array<T, Mem>: a sized owning buffer on the host or on one GPU.
// Parity: reference include/stencil/array.hpp:10-49 (host new[] array with size/resize/[]/begin/end/==/swap). The
// reference's GPU specialisation (:52-83) is behind a macro that is never defined and does not compile; here the
// device variant is real: hipMalloc on a chosen GPU, with explicit host<->device copies (no element access from the
// host).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <initializer_list>
#include <type_traits>
#include <utility>
#include <vector>

#include "stencil/rt/hip_check.hpp"

namespace stencil {

enum class Mem { Host, Device };

template <typename T, Mem M = Mem::Host> class Array;

template <typename T> class Array<T, Mem::Host> {
  T *data_ = nullptr;
  size_t n_ = 0;

public:
  Array() = default;
  explicit Array(size_t n) : data_(n ? new T[n]() : nullptr), n_(n) {}
  Array(size_t n, const T &v) : Array(n) { std::fill(begin(), end(), v); }
  Array(std::initializer_list<T> il) : Array(il.size()) { std::copy(il.begin(), il.end(), begin()); }
  Array(const Array &o) : Array(o.n_) { std::copy(o.begin(), o.end(), begin()); }
  Array(Array &&o) noexcept { swap(o); }
  Array &operator=(Array o) noexcept {
    swap(o);
    return *this;
  }
  ~Array() { delete[] data_; }
  void swap(Array &o) noexcept {
    std::swap(data_, o.data_);
    std::swap(n_, o.n_);
  }
  // keeps the first min(n, size()) elements
  void resize(size_t n) {
    Array t(n);
    std::copy(begin(), begin() + std::min(n, n_), t.begin());
    swap(t);
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T *data() { return data_; }
  const T *data() const { return data_; }
  T &operator[](size_t i) { return data_[i]; }
  const T &operator[](size_t i) const { return data_[i]; }
  T *begin() { return data_; }
  T *end() { return data_ + n_; }
  const T *begin() const { return data_; }
  const T *end() const { return data_ + n_; }
  bool operator==(const Array &o) const { return n_ == o.n_ && std::equal(begin(), end(), o.begin()); }
  bool operator!=(const Array &o) const { return !(*this == o); }
};

template <typename T> class Array<T, Mem::Device> {
  static_assert(std::is_trivially_copyable<T>::value, "device arrays hold trivially copyable elements");
  T *data_ = nullptr;
  size_t n_ = 0;
  int dev_ = -1;

  static T *alloc(size_t n, int dev) {
    if (!n) return nullptr;
    int prev = 0;
    HIP_CHECK(hipGetDevice(&prev));
    if (dev >= 0) HIP_CHECK(hipSetDevice(dev));
    void *p = nullptr;
    HIP_CHECK(hipMalloc(&p, n * sizeof(T)));
    if (dev >= 0) HIP_CHECK(hipSetDevice(prev));
    return static_cast<T *>(p);
  }

public:
  Array() = default;
  explicit Array(size_t n, int dev = -1) : n_(n), dev_(dev) {
    if (dev_ < 0) HIP_CHECK(hipGetDevice(&dev_));
    data_ = alloc(n, dev_);
  }
  // upload a host vector
  explicit Array(const std::vector<T> &h, int dev = -1) : Array(h.size(), dev) { from_host(h.data(), h.size()); }
  Array(const Array &) = delete;
  Array &operator=(const Array &) = delete;
  Array(Array &&o) noexcept { swap(o); }
  Array &operator=(Array &&o) noexcept {
    Array t(std::move(o));
    swap(t);
    return *this;
  }
  ~Array() {
    if (data_) (void)hipFree(data_);
  }
  void swap(Array &o) noexcept {
    std::swap(data_, o.data_);
    std::swap(n_, o.n_);
    std::swap(dev_, o.dev_);
  }
  size_t size() const { return n_; }
  int device() const { return dev_; }
  T *data() { return data_; }
  const T *data() const { return data_; }
  void from_host(const T *src, size_t n, hipStream_t s = nullptr) {
    STENCIL_REQUIRE(n <= n_, "Array::from_host: " << n << " > " << n_);
    HIP_CHECK(hipMemcpyAsync(data_, src, n * sizeof(T), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  std::vector<T> to_host(hipStream_t s = nullptr) const {
    std::vector<T> h(n_);
    if (n_) {
      HIP_CHECK(hipMemcpyAsync(h.data(), data_, n_ * sizeof(T), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
    }
    return h;
  }
  // byte-wise fill (hipMemset semantics)
  void memset(int v, hipStream_t s = nullptr) {
    if (n_) HIP_CHECK(hipMemsetAsync(data_, v, n_ * sizeof(T), s));
  }
};

} // namespace stencil
