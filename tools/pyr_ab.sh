#!/bin/bash
# Pyramid A/B: parity (extraction + yaml configs), planned bands and resident
# workgroups per CU, serial rocprof averages, interleaved pipelined lines.
# Usage: tools/pyr_ab.sh variant...   (variants from tools/variant.sh)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pyab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests_base.log 2>&1 || { echo "base parity FAILED"; tail -n 30 $O/tests_base.log; exit 1; }
echo "base parity: $(tail -n 1 $O/tests_base.log)"
for v in base "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  ORBX_PYR_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 > $O/prof_$v.log 2>&1 || { echo "$v prof failed"; tail -5 $O/prof_$v.log; exit 1; }
  grep -E "^pyr plan|^pyr_band" $O/prof_$v.log | sort | uniq | head -20 | sed "s/^/$v /"
done
unset ORBX_LIB_VARIANT
tools/variant_serial.sh pyab base "$@"
for rep in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench_${v}_$rep.log 2>&1
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]);print('$v rep $rep VALUE',d['value'],d['stage_ms_per_batch'])"
  done
done
