#!/bin/bash
# Interleaved C3 + BoW A/B of (variant, env) settings, R rounds.
# Usage: R=3 tools/ab_bow_env.sh "base" "vocold" "base ORBX_VOC_GL=4" "base --match-order top2-first" ...
cd "$GRAFT_REPO_ROOT"
settings=("$@")
for r in $(seq ${R:-2}); do
  for a in "${settings[@]}"; do
    set -- $a
    v=$1; shift
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    envs=(); args=()
    for t in "$@"; do case $t in --*) args+=("$t");; *=*) envs+=("$t");; *) args+=("$t");; esac; done
    env "${envs[@]}" timeout -k 10 200 python3 bench.py "${args[@]}" --allow-diag --bow-match --steps 50 --warmup 10 --cpu-sample 0 --no-latency --no-host-stream > /tmp/vb.log 2>&1 || { tail -5 /tmp/vb.log; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/vb.log').read().strip().splitlines()[-1]);s=d['stage_ms_per_batch'];print('[$a]',d['value'],'bow_match',s['bow_match'],'bow_transform',s['bow_transform'])"
  done
done
