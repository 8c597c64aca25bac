#!/bin/bash
# 1-GPU bench variants: stores (nt), z-march alternation, rows per lane, overlap
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/bv
run() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 64 --warmup 16 "$@" > gpurun_out/bv/$name.log 2>&1 || { echo "$name FAILED"; tail -5 gpurun_out/bv/$name.log; return 1; }
  python - "$name" gpurun_out/bv/$name.log <<'PY'
import json,sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d=json.loads(l); print(f"{sys.argv[1]:18s} {d['value']:8.1f} Gcells/s  {d['ms_per_step']*1e3:7.1f} us/step  xchg {d['extra']['exchange_ms']*1e3:6.1f} us")
PY
}
run base &&
run nt0 --nt 0 &&
run altz0 --altz 0 &&
run nt0_altz0 --nt 0 --altz 0 &&
run ty4 --ty 4 &&
run ty4_nt0 --ty 4 --nt 0 &&
run overlap --overlap on &&
run overlap_nt0 --overlap on --nt 0 &&
run base2
echo "done rc=$?"
