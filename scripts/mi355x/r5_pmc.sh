# PMC passes (one counter group per run) over bench.py's fused sweep: pair (--temporal 2) vs triple (--temporal 3)
set -o pipefail
O=gpurun_out/r5/${PMC_TAG:-c}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
for t in ${PMC_TEMPORALS:-2 3}; do
  for p in 1 2 3 4; do
    case $p in 1) C="$P1";; 2) C="$P2";; 3) C="FETCH_SIZE";; 4) C="WRITE_SIZE";; esac
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/p${p}_t$t -o pmc -- python bench.py --temporal $t --steps 18 --warmup 0 --exchange-iters 1 --with-exchange off ${PMC_ARGS:-} > $O/p${p}_t$t.log 2>&1 || exit 1
  done
done
