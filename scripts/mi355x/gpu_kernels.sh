#!/bin/bash
# stencil kernel sweep vs the streaming roofline, plus HBM byte counters of the default variant
set -o pipefail
export STENCIL_SKIP_BUILD=1 STENCIL_PLAN_FILE=0 PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -k 10 300 ./build/bin/bench_stencil > gpurun_out/bench_stencil.csv 2>&1 && cat gpurun_out/bench_stencil.csv &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d gpurun_out/pmc/bytes -o pmc --output-format csv -- ./build/bin/bench_stencil --only lds --iters 2 > gpurun_out/pmc/bytes.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d gpurun_out/pmc/sq -o pmc --output-format csv -- ./build/bin/bench_stencil --only lds --iters 2 > gpurun_out/pmc/sq.log 2>&1
echo "done rc=$?"
