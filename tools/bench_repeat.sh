#!/bin/bash
# The default C3 line N times in one GPU call (run-to-run spread of `value`).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rep; mkdir -p $O
for i in $(seq 1 ${1:-5}); do
  timeout -k 10 200 python3 bench.py --cpu-sample 0 --no-latency --no-host-stream > $O/bench_$i.log 2>&1 || { echo "run $i failed"; tail -5 $O/bench_$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]);print('run $i',d['value'],d['ms_per_step'])"
done
