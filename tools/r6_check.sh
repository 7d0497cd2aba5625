#!/bin/bash
# Round-6 edit-measure step: named GPU tests, quadtree phase clocks, serial
# rocprof stats, the matcher per-call leg and a pipelined bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6c}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 \
    || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
if [ -z "$NO_PROF" ]; then
  ORBX_QT_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 $BENCH_ARGS > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  grep "^quadtree" $O/prof.log | tail -10 | cut -c1-240
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
    python3 bench.py --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream $BENCH_ARGS \
    > $O/serial.log 2>&1 || { tail -5 $O/serial.log; exit 1; }
  python3 tools/stats_brief.py $O/serial/run_kernel_stats.csv
fi
if [ -n "$TRACE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pipe -o run -- \
    python3 bench.py --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream $BENCH_ARGS \
    > $O/pipe.log 2>&1 || { tail -5 $O/pipe.log; exit 1; }
  python3 tools/trace_overlap.py $O/pipe/run_kernel_trace.csv
fi
if [ -n "$MLAT" ]; then
  timeout -k 10 300 python3 -c "
import json, bench
print(json.dumps(bench.shim_matcher_latency_leg(0)))
" > $O/mlat.json 2>&1 || { tail -5 $O/mlat.json; exit 1; }
  cat $O/mlat.json | cut -c1-1500
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream $BENCH_ARGS > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep -o '"value": [0-9.]*' $O/bench.log
fi
