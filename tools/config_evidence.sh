#!/bin/bash
# Bench lines and rocprofv3 kernel stats for every config DESIGN.md quotes
# (C2 extract only, C4 stereo, C5 per-GPU EuRoC, C3 + ComputeBoW + SearchByBoW),
# fresh SQ counters of the serial C3 bench, and the search_init phase clocks.
# Stops at the first failing step. Usage: tools/config_evidence.sh
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/cfg
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 "$@" > $OUT/$name.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- \
    python3 bench.py --cpu-sample 0 --no-latency --no-host-stream --steps 30 --warmup 5 "$@" > $OUT/${name}_prof.log 2>&1
  echo "$name done"
}
run c2 --no-match
run c4 --config stereo
run c5 --config euroc
run bowmatch --bow-match
run bowmatch_serial --bow-match --serial
timeout -k 10 120 python3 tools/init_timing.py 64 > $OUT/init_prof.log 2>&1
timeout -k 10 120 python3 tools/init_timing.py 64 >> $OUT/init_prof.log 2>&1
bash tools/pmc_sq.sh $OUT/pmc_sq > $OUT/pmc_sq.log 2>&1
echo all-done
