#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pipe2; mkdir -p $O
run() {  # name, args
  n=$1; shift
  timeout -k 10 150 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]);s=d['stage_ms_per_batch'];print('$n',d['value'],'top2',s['hamming_top2'],'init',s['search_init'])"
}
for r in 1 2 3; do
run base_$r
run noprio_$r --no-match-priority
run initfirst_$r --match-order init,top2,bow
run ms2_$r --match-streams 2
done
