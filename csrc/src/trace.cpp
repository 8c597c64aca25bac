#include "stencil/rt/trace.hpp"
#include "stencil/rt/env.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace stencil {
namespace trace {

namespace {
using PushFn = int (*)(const char *);
using PopFn = int (*)();
struct Roctx {
  PushFn push = nullptr;
  PopFn pop = nullptr;
  bool on = false;
  Roctx() {
    if (env::get_int("STENCIL_TRACE", 0) == 0) return;
    const char *libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                          "libroctx64.so"};
    for (const char *l : libs) {
      void *h = dlopen(l, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
      if (push && pop) {
        on = true;
        return;
      }
    }
  }
};
Roctx &roctx() {
  static Roctx r;
  return r;
}
} // namespace

bool enabled() { return roctx().on; }
void push(const char *name) {
  auto &r = roctx();
  if (r.on) r.push(name);
}
void pop() {
  auto &r = roctx();
  if (r.on) r.pop();
}

} // namespace trace
} // namespace stencil
