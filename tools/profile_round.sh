#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the bench command,
# then separate FETCH_SIZE and WRITE_SIZE passes (counters never combined
# with runtime/sys tracing). Usage: tools/profile_round.sh TAG [bench args]
set -e
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
ARGS="--cpu-sample 0 --no-latency --no-host-stream $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/pmc_traffic.py $OUT/pmc_traffic.json $OUT/fetch $OUT/write > $OUT/traffic.txt
echo done
