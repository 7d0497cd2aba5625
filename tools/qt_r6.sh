#!/bin/bash
# Round-6 quadtree step: extraction parity (sorted path + fallback), per-level
# phase clocks (ORBX_QT_PROF=1) and a short pipelined bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-qt6}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_extract.py} > $O/tests.log 2>&1 \
  || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ORBX_QT_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep "^quadtree" $O/prof.log | tail -8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
  python3 bench.py --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream \
  > $O/serial.log 2>&1 || { tail -5 $O/serial.log; exit 1; }
python3 tools/stats_brief.py $O/serial/run_kernel_stats.csv
timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench.log
