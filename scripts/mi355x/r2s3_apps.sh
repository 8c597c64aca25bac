#!/bin/bash
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r2s3_apps}; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_apps_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -15 $D/tests.log; exit $rc
