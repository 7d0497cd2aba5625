#!/bin/bash
# SearchByBoW batch A/B step: the BoW parity tests, the pipelined C3 + BoW bench
# line, serial per-kernel rocprof averages and the BoW phase clocks.
# Usage: tools/bow_quick.sh TAG [variant]
set -e
TAG=$1; V=${2:-}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bow_$TAG
mkdir -p $OUT
if [ -n "$V" ]; then export ORBX_LIB_VARIANT=$V; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_bow_batch.py tests/test_gpu_pipeline.py -k "bow" -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
timeout -k 10 200 python3 bench.py --allow-diag --bow-match --steps 50 --warmup 10 --cpu-sample 0 --no-latency --no-host-stream > $OUT/bench.log 2>&1
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print('VALUE',d['value'],d['ms_per_step'],d['stage_ms_per_batch'],'bow_nm',d['bow_matches_per_pair'])"
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial -o run -- python3 bench.py --allow-diag --bow-match --serial --steps 10 --warmup 2 --cpu-sample 0 --no-latency --no-host-stream > $OUT/serial.log 2>&1
python3 tools/stats_brief.py $OUT/serial/run_kernel_stats.csv | grep -v rocclr
ORBX_BOW_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --bow-match --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 2>&1 | grep "^bow" | tail -1
