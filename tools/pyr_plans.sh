#!/bin/bash
# Pyramid band plans: the planned (bands, cost, LDS) list and phase clocks of the
# default pick, then serial rocprof averages of pyr_band_kernel per forced plan.
# Usage: tools/pyr_plans.sh TAG [plan indices...]
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
ORBX_PYR_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 2>&1 | grep "^pyr_band" | tail -2
for i in "$@"; do
  OUT=gpurun_out/pp_${TAG}_$i
  ORBX_PYR_PLAN=$i timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --allow-diag --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream > $OUT.log 2>&1 || { echo "plan $i failed"; tail -3 $OUT.log; exit 1; }
  echo "plan $i: $(python3 tools/stats_brief.py $OUT/run_kernel_stats.csv | grep pyr_band)"
done
