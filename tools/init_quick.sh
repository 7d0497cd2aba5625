#!/bin/bash
# search_init A/B: the matcher GPU tests, the pipelined timed-region parity, the
# 64-pair timing alone under a kernel trace, and the default bench line.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/init; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py "tests/test_gpu_pipeline.py::test_timed_pipeline_matches_oracle[kitti]" tests/test_shim.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 60 $O/tests.log; exit 1; }
tail -n 3 $O/tests.log
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alone -o run -- python3 tools/init_timing.py 64 > $O/alone.log 2>&1
cat $O/alone.log | tail -2
cut -d, -f1-4 $O/alone/run_kernel_stats.csv | head -8
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench.log 2>&1
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('VALUE',d['value'],d['ms_per_step'],d['stage_ms_per_batch'])"
timeout -k 10 120 python3 tools/h2d_bench.py > $O/h2d.json 2> $O/h2d.err || { tail -20 $O/h2d.err; exit 1; }
cat $O/h2d.json
