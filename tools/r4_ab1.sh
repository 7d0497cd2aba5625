#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/init3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread > $O/match.log 2>&1 || { tail -n 30 $O/match.log; exit 1; }
tail -n 1 $O/match.log
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alone -o run -- python3 tools/init_timing.py 64 > $O/alone.log 2>&1
grep "ms_per_call" $O/alone.log
python3 tools/stats_brief.py $O/alone/run_kernel_stats.csv | grep search_init
tools/fast_ab.sh r4a base c8 band bandc8
