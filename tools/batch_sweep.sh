#!/bin/bash
# Frames per step x extraction launches per step, pipelined bench, one line each.
cd $GRAFT_REPO_ROOT
for a in "--batch 64 --split 2" "--batch 96 --split 3" "--batch 128 --split 2" "--batch 128 --split 4" "--batch 192 --split 3" "--batch 256 --split 4" "--batch 64 --split 2"; do
  timeout -k 10 120 python3 bench.py --steps 60 --warmup 10 --cpu-sample 0 $a > /tmp/sw.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('/tmp/sw.log').read().strip().splitlines()[-1]);print('$a', d['value'], d['ms_per_step'])"
done
