#!/bin/bash
# search_init timing alone, the default bench line, the link microbench, then
# the shipped-config parity and the FAST variants' extraction parity.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/init2; mkdir -p $O
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alone -o run -- python3 tools/init_timing.py 64 > $O/alone.log 2>&1
grep "ms_per_call" $O/alone.log
python3 tools/stats_brief.py $O/alone/run_kernel_stats.csv
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench.log 2>&1
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('VALUE',d['value'],d['ms_per_step'],d['stage_ms_per_batch'])"
timeout -k 10 120 python3 tools/h2d_bench.py > $O/h2d.json 2> $O/h2d.err || { tail -20 $O/h2d.err; exit 1; }
cat $O/h2d.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py "tests/test_gpu_pipeline.py::test_timed_pipeline_matches_oracle" -x -q --timeout 240 --timeout-method thread > $O/cfg.log 2>&1 || { tail -n 40 $O/cfg.log; exit 1; }
tail -n 2 $O/cfg.log
