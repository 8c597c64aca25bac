#!/bin/bash
# remote-halo overlap probe (bench_stencil --only ovl): pinned-memory "link", reserve / CU-mask variants
set -o pipefail
mkdir -p gpurun_out/ovlprobe
timeout -k 10 100 ./build/bin/bench_stencil --only ovl --reps 1 --iters 10 > gpurun_out/ovlprobe/ovl.log 2>&1
rc=$?; cat gpurun_out/ovlprobe/ovl.log; exit $rc
