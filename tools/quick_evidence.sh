#!/bin/bash
# The short form of tools/round_evidence.sh for a crowded GPU pool: the default
# bench line, the pipelined rocprofv3 stats of the C3 bench and the serial
# (every kernel alone) stats. Stops at the first failing step.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/q
mkdir -p $OUT
timeout -k 10 300 python3 bench.py > $OUT/bench_default.log 2>&1
tail -n 1 $OUT/bench_default.log | cut -c1-200
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
ARGS="--cpu-sample 0 --no-latency --no-host-stream --steps 30 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial -o run -- python3 bench.py --serial $ARGS > $OUT/serial.log 2>&1
echo all-done
