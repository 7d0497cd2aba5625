#!/bin/bash
# One GPU call for an A/B step: selected GPU tests, the serial per-kernel
# rocprofv3 averages, and the default bench line (no CPU baseline).
# Usage: tools/quick_eval.sh TAG "pytest targets"
set -e
TAG=$1; TESTS=${2:-tests/test_gpu_match.py}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q_$TAG
timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/q_$TAG/tests.log 2>&1 || { tail -n 40 gpurun_out/q_$TAG/tests.log; exit 1; }
tail -n 2 gpurun_out/q_$TAG/tests.log
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q_$TAG/serial -o run -- python3 bench.py --serial --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream > gpurun_out/q_$TAG/serial.log 2>&1
python3 tools/stats_brief.py gpurun_out/q_$TAG/serial/run_kernel_stats.csv
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > gpurun_out/q_$TAG/bench.log 2>&1
python3 -c "import json,sys;d=json.loads(open('gpurun_out/q_$TAG/bench.log').read().strip().splitlines()[-1]);print('VALUE',d['value'],d['ms_per_step'],d['stage_ms_per_batch'],d.get('match_roofline'))"
