#!/bin/bash
# Pyramid LDS counters (bank conflicts, LDS-active cycles, VALU, LDS instructions) of
# the serial bench, base vs the runs-of-4 variant (tools/variant.sh prun4).
set -e
cd "$GRAFT_REPO_ROOT"
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for v in base prun4; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/psq_$v -o pass1 -- python3 bench.py --allow-diag --steps 3 --warmup 1 --cpu-sample 0 --serial --pool 64 --no-latency --no-host-stream > gpurun_out/psq_$v.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/psq_$v > gpurun_out/psq_$v.txt
  echo "== $v"; grep -A5 pyr_band gpurun_out/psq_$v.txt
done
