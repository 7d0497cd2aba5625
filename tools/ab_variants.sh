#!/bin/bash
# Interleaved pipelined-bench A/B of liborbx variants (tools/variant.sh), two
# rounds. Usage: tools/ab_variants.sh base v1 v2 ...
cd "$GRAFT_REPO_ROOT"
for r in $(seq ${R:-2}); do
  for v in "$@"; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > /tmp/vb.log 2>&1 || { tail -5 /tmp/vb.log; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/vb.log').read().strip().splitlines()[-1]);print('$v',d['value'],d['stage_ms_per_batch'])"
  done
done
