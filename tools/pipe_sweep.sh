#!/bin/bash
# Pipelined bench under stream options, two runs each (run-to-run spread is a few %).
cd $GRAFT_REPO_ROOT
for a in "" "--priority" "--split 1" "--split 4" "--carry ext" ""; do
  for r in 1 2; do
    timeout -k 10 120 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 $a > /tmp/ps.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('/tmp/ps.log').read().strip().splitlines()[-1]);print('[$a]', d['value'], d['ms_per_step'])"
  done
done
