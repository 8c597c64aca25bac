#!/bin/bash
# race canary timing (2 ranks on one GPU, IPC / staged with jitter), then the GPU suite with per-test durations
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_canary}; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "race_canary" --durations=0 > $D/canary.log 2>&1; rc=$?
grep -E "PASSED|FAILED|s call" $D/canary.log | head; echo "canary rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --durations=15 > $D/pytest_gpu.log 2>&1; rc=$?
tail -22 $D/pytest_gpu.log; echo "suite rc=$rc"; exit $rc
