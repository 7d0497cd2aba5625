#!/bin/bash
# One GPU call for an edit-measure step: the named GPU test files, the drop-in
# shim's per-call latency (bench.py's shim_latency leg) and a serial rocprofv3
# run (every kernel alone). Stops at the first failing step.
# Usage: OUT=r5x TESTS="tests/test_gpu_extract.py ..." tools/gpu_check.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-check}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 \
    || { echo TESTFAIL; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
if [ -z "$NO_SHIM" ]; then
  timeout -k 10 300 python -c "
import json, bench
from orb_slam_cuda_amd.synth import SynthSequence
print(json.dumps(bench.shim_latency_leg(list(SynthSequence(1, 1241, 376).frames(32)), 1241, 376, 0)))
" > $O/shim.json 2>&1 || { tail -5 $O/shim.json; exit 1; }
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
  python3 bench.py --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream $BENCH_ARGS \
  > $O/serial.log 2>&1 || { tail -5 $O/serial.log; exit 1; }
python3 tools/stats_brief.py $O/serial/run_kernel_stats.csv
