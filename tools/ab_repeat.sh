#!/bin/bash
# Interleaved A/B of the pipelined bench: variants in turn, N rounds, mean per variant.
# Usage: tools/ab_repeat.sh N base v1 ...
cd "$GRAFT_REPO_ROOT"
N=$1; shift
for r in $(seq $N); do
  for v in "$@"; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 120 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 > /tmp/ab.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('/tmp/ab.log').read().strip().splitlines()[-1]);print('$v', d['value'])" | tee -a /tmp/ab_all.txt
  done
done
python3 - <<PY
import collections
d=collections.defaultdict(list)
for l in open('/tmp/ab_all.txt'):
    k,v=l.split(); d[k].append(float(v))
for k,v in d.items(): print('MEAN', k, round(sum(v)/len(v),1), 'n', len(v))
PY
