#!/bin/bash
# Interleaved C3 / C3+BoW A/B of bench.py argument sets, R rounds (tools/ab_bow_env.sh without --bow-match)
cd "$GRAFT_REPO_ROOT"
settings=("$@")
for r in $(seq ${R:-2}); do
  for a in "${settings[@]}"; do
    timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream $a > /tmp/ab.log 2>&1 || { tail -5 /tmp/ab.log; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.log').read().strip().splitlines()[-1]);s=d['stage_ms_per_batch'];print('[$a]',d['value'],{k:s[k] for k in ('hamming_top2','search_init','bow_match') if k in s})"
  done
done
