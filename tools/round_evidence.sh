#!/bin/bash
# Everything the round's evidence needs, in one GPU call: the GPU test suite,
# smoke(), the default bench line, the rocprofv3 summaries (pipelined stats +
# FETCH_SIZE / WRITE_SIZE passes, serial stats), the SQ counters, FAST phase
# clocks and the C3 + BoW line. Stops at the first failing step.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ev
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/ev/gpu_tests.log 2>&1
tail -n 1 gpurun_out/ev/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log 2>&1
cat gpurun_out/ev/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/ev/bench_default.log 2>&1
tail -n 1 gpurun_out/ev/bench_default.log | cut -c1-200
bash tools/profile_round.sh main --steps 30 --warmup 5 > gpurun_out/ev/prof_main.txt 2>&1
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/serial -o run -- python3 bench.py --serial --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream > gpurun_out/ev/serial.log 2>&1
bash tools/pmc_sq.sh gpurun_out/ev/sq > gpurun_out/ev/sq.log 2>&1
ORBX_FAST_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 2>&1 | grep "^fast" > gpurun_out/ev/fast_phases.txt
timeout -k 10 300 python3 bench.py --bow-match --cpu-sample 0 --no-latency --no-host-stream > gpurun_out/ev/bench_bow.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev/bowserial -o run -- python3 bench.py --bow-match --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream > gpurun_out/ev/bowserial.log 2>&1
echo all-done
