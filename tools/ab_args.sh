#!/bin/bash
# Interleaved A/B of bench.py argument sets, R rounds: prints value per run.
# Usage: R=3 tools/ab_args.sh "" "--split 1" ...
cd "$GRAFT_REPO_ROOT"
for r in $(seq ${R:-3}); do
  for a in "$@"; do
    timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream $a > /tmp/ab.log 2>&1 || { tail -5 /tmp/ab.log; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.log').read().strip().splitlines()[-1]);print('[$a]',d['value'],d['ms_per_step'])"
  done
done
