#pragma once
// roctx ranges for rocprofv3 --marker-trace.
// Parity: reference nvtxRangePush/Pop sites (92 of them, e.g. src/stencil.cu:672-850, local_domain.cu:42).
// roctx is resolved with dlopen at first use (librocprofiler-sdk-roctx.so, then libroctx64.so), so the library has
// no hard link dependency on the profiler; ranges are no-ops unless STENCIL_TRACE=1 or a roctx library loads.
namespace stencil {
namespace trace {
void push(const char *name);
void pop();
bool enabled();
} // namespace trace

struct TraceRange {
  explicit TraceRange(const char *name) { trace::push(name); }
  ~TraceRange() { trace::pop(); }
  TraceRange(const TraceRange &) = delete;
  TraceRange &operator=(const TraceRange &) = delete;
};
} // namespace stencil
