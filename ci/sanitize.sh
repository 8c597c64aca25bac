#!/bin/bash
# Host-side AddressSanitizer + UBSan build of the runtime and the native tests, run on the CPU backend
# (device ASan / xnack+ runs are not available on the MI355X pool, so sanitizers cover host code).
# -fsanitize applies to host code only (CMake: -Xarch_host -fsanitize=...).
set -euo pipefail
cd "$(dirname "$0")/.."
B=build-asan
cmake -S . -B $B -G Ninja -DCMAKE_HIP_ARCHITECTURES=gfx950 -DCMAKE_BUILD_TYPE=RelWithDebInfo \
  -DSTENCIL_HOST_SANITIZE=ON -DSTENCIL_BUILD_PYTHON=OFF -DSTENCIL_BUILD_APPS=OFF > /dev/null
ninja -C $B -j"${MAX_JOBS:-8}" stencil_ctest
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 $B/bin/stencil_ctest --cpu
