#!/bin/bash
# Interleaved pipelined-bench A/B of environment settings (tuning knobs), R rounds.
# Usage: R=2 tools/ab_env.sh "" "ORBX_EXTRACT_ORDER=pfbqo" ...
cd "$GRAFT_REPO_ROOT"
for r in $(seq ${R:-2}); do
  for e in "$@"; do
    env $e timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > /tmp/abe.log 2>&1 || { tail -5 /tmp/abe.log; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/abe.log').read().strip().splitlines()[-1]);s=d['stage_ms_per_batch'];print('[$e]',d['value'],'init',s['search_init'],'top2',s['hamming_top2'])"
  done
done
