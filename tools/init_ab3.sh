#!/bin/bash
# search_init prep workgroup sizes against the default: parity of the
# matcher tests, then three interleaved pipelined C3 lines each.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/iab3; mkdir -p $O
for v in "$@"; do
  ORBX_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc: $(tail -n 1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit 1
done
for rep in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]);print('$v rep $rep VALUE',d['value'],d['stage_ms_per_batch'])"
  done
done
