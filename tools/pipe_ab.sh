#!/bin/bash
# Pipeline-shape A/B on the default C3 bench (2 interleaved rounds).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pipe; mkdir -p $O
run() {  # name, env, args
  n=$1; shift; e=$1; shift
  env $e timeout -k 10 150 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]);print('$n',d['value'],d['stage_ms_per_batch'])"
}
for r in 1 2; do
run base_$r X=1
run pfbqo_$r ORBX_EXTRACT_ORDER=pfbqo
run pfqbo_$r ORBX_EXTRACT_ORDER=pfqbo
run b128_$r X=1 --batch 128
run b128s4_$r X=1 --batch 128 --split 4
run b96s3_$r X=1 --batch 96 --split 3
done
