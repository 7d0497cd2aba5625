#!/bin/bash
# Variants: extraction parity each, then interleaved pipelined lines (3 rounds).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/vp; mkdir -p $O
for v in "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "$v parity FAILED"; tail -n 30 $O/tests_$v.log; exit 1; }
  echo "$v parity: $(tail -n 1 $O/tests_$v.log)"
done
unset ORBX_LIB_VARIANT
tools/variant_serial.sh vp "$@" | grep -E "==|blur|pyr|fast|orient"
for rep in 1 2 3; do
  for v in "$@"; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench_${v}_$rep.log 2>&1
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]);print('$v rep $rep VALUE',d['value'],d['stage_ms_per_batch'])"
  done
done
