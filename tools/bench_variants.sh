#!/bin/bash
# A/B of liborbx variants (tools/variant.sh) in the real pipelined bench plus
# the Hamming parity tests. Usage: tools/bench_variants.sh base a b ...
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  t=$(timeout -k 10 200 python -u -m pytest tests/test_gpu_match.py -x -q -k hamming --timeout 120 --timeout-method thread 2>&1 | tail -n 1)
  echo -n "$v [$t] top2-alone: "
  WHICH=top2 timeout -k 10 60 python3 tools/init_timing.py 64 | grep -o "ms_per_call=[0-9.]*" || exit 1
  timeout -k 10 120 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 > /tmp/bv.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('/tmp/bv.log').read().strip().splitlines()[-1]);print('   bench',d['value'],d['ms_per_step'],'ham',d['stage_ms_per_batch']['hamming_top2'])"
done
