#!/bin/bash
# FAST under several launch settings (env assignments, "-" = none): phase
# clocks and the clean serial per-kernel averages (no single-frame legs).
# Usage: ORBX_LIB_VARIANT=... tools/fast_env.sh "-" "ORBX_FAST_WAVES_PER_CU=16" ...
cd "$GRAFT_REPO_ROOT"
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
i=0
for e in "$@"; do
  i=$((i+1))
  echo "== $e"
  [ "$e" = "-" ] && e=""
  env $e ORBX_FAST_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 > /tmp/fe.log 2>&1 || { tail -5 /tmp/fe.log; exit 1; }
  grep "^fast" /tmp/fe.log | head -1; grep "^fast" /tmp/fe.log | tail -1
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fe$i -o run -- python3 bench.py --allow-diag --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream > /tmp/fes.log 2>&1 || { tail -5 /tmp/fes.log; exit 1; }
  python3 tools/stats_brief.py gpurun_out/fe$i/run_kernel_stats.csv | grep -E "fast"
done
