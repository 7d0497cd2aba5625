#!/bin/bash
# search_init shape A/B: matcher parity per variant, then interleaved pipelined lines.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/iab; mkdir -p $O
for v in "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "$v parity FAILED"; tail -n 30 $O/tests_$v.log; exit 1; }
  echo "$v parity: $(tail -n 1 $O/tests_$v.log)"
done
unset ORBX_LIB_VARIANT
for rep in 1 2 3; do
  for v in "$@"; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench_${v}_$rep.log 2>&1
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]);s=d['stage_ms_per_batch'];print('$v rep $rep VALUE',d['value'],'top2',s['hamming_top2'],'init',s['search_init'])"
  done
done
