#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/init5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py "tests/test_gpu_pipeline.py::test_timed_pipeline_matches_oracle[kitti]" -x -q --timeout 120 --timeout-method thread > $O/match.log 2>&1 || { tail -n 30 $O/match.log; exit 1; }
tail -n 1 $O/match.log
ORBX_INIT_PROF=1 timeout -k 10 120 python3 tools/init_timing.py 64 > $O/prof.log 2>&1
tail -n 2 $O/prof.log
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alone -o run -- python3 tools/init_timing.py 64 > $O/alone.log 2>&1
grep "ms_per_call" $O/alone.log
python3 tools/stats_brief.py $O/alone/run_kernel_stats.csv | grep search_init
for r in 1 2; do
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench$r.log 2>&1
python3 -c "import json;d=json.loads(open('$O/bench$r.log').read().strip().splitlines()[-1]);print('VALUE',d['value'],d['stage_ms_per_batch'])"
done
tools/host_ab.sh
