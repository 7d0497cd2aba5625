#!/bin/bash
# Two SQ counter passes over the serial benchmark (every kernel alone on the
# chip), one rocprofv3 run per counter group. Usage: tools/pmc_sq.sh OUTDIR [bench args]
set -e
OUT=$GRAFT_REPO_ROOT/$1; shift
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
ARGS="--steps 3 --warmup 1 --cpu-sample 0 --serial --pool 64 --no-latency --no-host-stream $*"
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT -o pass$i -- python3 bench.py $ARGS > $OUT/pass$i.log 2>&1
  echo "pass $i rc=$?"
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
