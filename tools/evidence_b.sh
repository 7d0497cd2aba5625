#!/bin/bash
# A round's evidence, part B (ROUND=rNN, PART=1|2|all; run after part A and tools/collect.sh): per-config bench lines + rocprofv3 stats (C2, C4,
# C5, C3 + BoW, the KITTI14 / intcatch-1080p settings), SQ counters of the
# serial C3 bench, FAST and search_init phase clocks, the link microbench.
set -e
cd "$GRAFT_REPO_ROOT"
R=${ROUND:-r05}
O=gpurun_out/ev_${R}b; mkdir -p $O
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --no-latency --no-host-stream "$@" > $O/$name.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- \
    python3 bench.py --cpu-sample 0 --no-latency --no-host-stream --steps 30 --warmup 5 "$@" > $O/${name}_prof.log 2>&1
  python3 -c "import json;d=json.loads(open('$O/$name.log').read().strip().splitlines()[-1]);print('$name',d['value'],d['unit'])"
}
PART=${PART:-all}  # 1: the config lines and their stats, 2: counters, phases, link, final line
if [ $PART != 2 ]; then
run c2 --no-match
run c4 --config stereo
run c5 --config euroc
run bowmatch --bow-match
run bowmatch_serial --bow-match --serial
run kitti14 --config kitti14
run intcatch1080 --config intcatch1080
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/intcatch1080_serial -o run -- \
  python3 bench.py --cpu-sample 0 --no-latency --no-host-stream --steps 30 --warmup 5 --serial --config intcatch1080 \
  > $O/intcatch1080_serial.log 2>&1
fi
[ $PART = 1 ] && { echo part-1-done; exit 0; }
bash tools/qt_prof.sh > $O/qt_phases.txt 2>&1
bash tools/pmc_sq.sh $O/sq > $O/sq.log 2>&1
python3 tools/sq_valu.py $O/sq/summary.txt $O/sq_valu.json
ORBX_FAST_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 2>&1 | grep "^fast" > $O/fast_phases.txt
ORBX_INIT_PROF=1 timeout -k 10 100 python3 tools/init_timing.py 64 > $O/init_phases.txt 2>&1
timeout -k 10 120 python3 tools/h2d_bench.py > $O/h2d.json
# the default bench line again, now reading this commit's counter files
# (pmc_traffic.json from part A, collected into profiles/ before this call;
# sq_valu.json from the passes above)
cp $O/sq_valu.json profiles/sq_valu.json
mkdir -p gpurun_out/ev_${R}c
timeout -k 10 400 python3 bench.py > gpurun_out/ev_${R}c/bench_default.log 2>&1
tail -n 1 gpurun_out/ev_${R}c/bench_default.log | cut -c1-200
echo all-done
