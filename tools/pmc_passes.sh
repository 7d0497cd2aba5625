#!/bin/bash
# PMC counter passes over the benchmark (one rocprofv3 run per counter group;
# counters never combined with runtime/sys tracing). Usage: tools/pmc_passes.sh OUTDIR [bench args]
set -e
OUT=$GRAFT_REPO_ROOT/$1; shift
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
ARGS="--steps 3 --warmup 1 --cpu-sample 0 $*"
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT -o pass$i -- python3 bench.py $ARGS > $OUT/pass$i.log 2>&1
  echo "pass $i rc=$?"
done
