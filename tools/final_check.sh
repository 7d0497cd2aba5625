#!/bin/bash
# Round-end check on the final commit: the GPU suite, smoke(), the default
# bench line, the single-frame latency evidence and the stereo-frame timeline.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -n 30 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.log 2>&1
tail -n 1 $O/bench_default.log | cut -c1-200
OUT=$O/lat TESTS=tests/test_gpu_dropin.py bash tools/lat_check.sh > $O/lat_check.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/stereo_prof -o run -- python3 tools/stereo_frame_prof.py 300 > $O/stereo_prof.log 2>&1
echo all-done
