#!/bin/bash
# Everything the round's evidence needs, in one GPU call: the GPU test suite,
# smoke(), the default bench line, and the rocprofv3 summaries of the bench
# and of the matcher tools. Stops at the first failing step.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ev
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ev/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/ev/bench_default.log 2>&1
bash tools/profile_round.sh main --steps 30 --warmup 5 > gpurun_out/ev/prof_main.txt 2>&1
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/serial -o run -- python3 bench.py --serial --steps 30 --warmup 5 --cpu-sample 0 > gpurun_out/ev/serial.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/pose -o run -- python3 tools/pose_timing.py 64 last 2000 > gpurun_out/ev/pose.log 2>&1
echo all-done
