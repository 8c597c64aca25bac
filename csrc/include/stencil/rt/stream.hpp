#pragma once
// Shared-ownership HIP stream / event handles.
// Parity: reference include/stencil/rcstream.hpp + src/rcstream.cpp:21-45 (ref-counted non-blocking stream,
// Priority::HIGH = max device priority, implicit conversion to the native stream handle, device()).
#include <hip/hip_runtime_api.h>

#include <memory>

#include "stencil/rt/hip_check.hpp"

namespace stencil {

enum class Priority { DEFAULT, HIGH };

class Stream {
  struct Impl {
    hipStream_t s = nullptr;
    int dev = -1;
    ~Impl() {
      if (s) {
        (void)hipSetDevice(dev);
        (void)hipStreamDestroy(s);
      }
    }
  };
  std::shared_ptr<Impl> impl_;

public:
  Stream() = default;
  explicit Stream(int dev, Priority prio = Priority::DEFAULT) : impl_(std::make_shared<Impl>()) {
    impl_->dev = dev;
    HIP_CHECK(hipSetDevice(dev));
    if (prio == Priority::HIGH) {
      int lo = 0, hi = 0;
      HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_CHECK(hipStreamCreateWithPriority(&impl_->s, hipStreamNonBlocking, hi));
    } else {
      HIP_CHECK(hipStreamCreateWithFlags(&impl_->s, hipStreamNonBlocking));
    }
  }
  operator hipStream_t() const { return impl_ ? impl_->s : nullptr; }
  hipStream_t get() const { return impl_ ? impl_->s : nullptr; }
  int device() const { return impl_ ? impl_->dev : -1; }
  long use_count() const { return impl_.use_count(); }
  explicit operator bool() const { return bool(impl_); }
  void sync() const {
    if (impl_) HIP_CHECK(hipStreamSynchronize(impl_->s));
  }
};

class Event {
  struct Impl {
    hipEvent_t e = nullptr;
    int dev = -1;
    ~Impl() {
      if (e) {
        (void)hipSetDevice(dev);
        (void)hipEventDestroy(e);
      }
    }
  };
  std::shared_ptr<Impl> impl_;

public:
  Event() = default;
  explicit Event(int dev, bool timing = false) : impl_(std::make_shared<Impl>()) {
    impl_->dev = dev;
    HIP_CHECK(hipSetDevice(dev));
    HIP_CHECK(hipEventCreateWithFlags(&impl_->e, timing ? hipEventDefault : hipEventDisableTiming));
  }
  operator hipEvent_t() const { return impl_ ? impl_->e : nullptr; }
  int device() const { return impl_ ? impl_->dev : -1; }
  void record(hipStream_t s) const { HIP_CHECK(hipEventRecord(impl_->e, s)); }
  void wait_on(hipStream_t s) const { HIP_CHECK(hipStreamWaitEvent(s, impl_->e, 0)); }
  void sync() const { HIP_CHECK(hipEventSynchronize(impl_->e)); }
  explicit operator bool() const { return bool(impl_); }
};

} // namespace stencil
