#!/bin/bash
# One GPU call for an extraction A/B step: the extraction parity tests, the
# serial per-kernel rocprofv3 averages (32-frame launches, no latency leg) and
# the FAST phase clocks. Usage: tools/ext_quick.sh TAG [pytest targets]
set -e
TAG=$1; TESTS=${2:-tests/test_gpu_extract.py}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/x_$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial -o run -- python3 bench.py --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream > $OUT/serial.log 2>&1
python3 tools/stats_brief.py $OUT/serial/run_kernel_stats.csv
ORBX_FAST_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 2>&1 | grep "^fast" | tail -1
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $OUT/bench.log 2>&1
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print('VALUE',d['value'],d['ms_per_step'],d['stage_ms_per_batch'])"
