#!/bin/bash
# A/B of the fused front path against the per-stage kernels in one GPU call:
# serial per-kernel rocprofv3 averages and the pipelined bench line for each.
# Usage: tools/ab_front.sh TAG
set -e
TAG=$1
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/abf_$TAG
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for MODE in 1 0; do
  ORBX_FRONT=$MODE timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial$MODE -o run -- python3 bench.py --serial --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream > $OUT/serial$MODE.log 2>&1
  echo "== ORBX_FRONT=$MODE serial"
  python3 tools/stats_brief.py $OUT/serial$MODE/run_kernel_stats.csv
done
for MODE in 1 0 1 0; do
  ORBX_FRONT=$MODE timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $OUT/bench$MODE.log 2>&1
  python3 -c "import json;d=json.loads(open('$OUT/bench$MODE.log').read().strip().splitlines()[-1]);print('FRONT=$MODE VALUE',d['value'],d['ms_per_step'],d['stage_ms_per_batch'],d['roofline']['frac'])"
done
