#!/bin/bash
# extraction-kernel A/B (FAST counters): parity, serial times, LDS conflict counters, pipelined lines.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fab; mkdir -p $O
for v in base "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "$v parity FAILED"; tail -n 30 $O/tests_$v.log; exit 1; }
  echo "$v parity: $(tail -n 1 $O/tests_$v.log)"
  bash tools/pmc_sq.sh gpurun_out/fab/sq_$v --allow-diag > $O/sq_$v.log 2>&1 || { echo "sq $v failed"; tail $O/sq_$v.log; exit 1; }
  grep -A16 "fast_cells" $O/sq_$v/summary.txt | grep -E "BANK|IDX_ACTIVE|INSTS_VALU|INSTS_SALU|WAVE_CYCLES" | sed "s/^/$v /"
done
unset ORBX_LIB_VARIANT
tools/variant_serial.sh fab base "$@"
for rep in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench_${v}_$rep.log 2>&1
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]);print('$v rep $rep VALUE',d['value'],d['stage_ms_per_batch'])"
  done
done
