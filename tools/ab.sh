#!/bin/bash
# Interleaved C3 A/B of (env, bench args) settings, R rounds.
# Usage: R=3 tools/ab_argenv.sh "" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8 --split 3" ...
cd "$GRAFT_REPO_ROOT"
settings=("$@")
for r in $(seq ${R:-2}); do
  for a in "${settings[@]}"; do
    envs=(); args=()
    for t in $a; do case $t in --*) args+=("$t");; *=*) envs+=("$t");; *) args+=("$t");; esac; done
    env "${envs[@]}" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream "${args[@]}" > /tmp/ab.log 2>&1 || { tail -5 /tmp/ab.log; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.log').read().strip().splitlines()[-1]);print('[$a]',d['value'],d['ms_per_step'])"
  done
done
