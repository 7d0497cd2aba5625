#!/bin/bash
# Variant A/B in one GPU call: base parity (extraction + yaml configs), each
# variant's extraction parity (a failing variant is reported and dropped, a
# crash / timeout ends the script), serial rocprof averages, interleaved
# pipelined lines.   Usage: tools/var_ab.sh TAG variant...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
stop() { echo "$1 exited $2: stopping"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests_base.log 2>&1
rc=$?; echo "base parity rc=$rc: $(tail -n 1 $O/tests_base.log)"; [ $rc -ne 0 ] && { tail -n 40 $O/tests_base.log; exit 1; }
ORBX_PYR_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 > $O/pyrprof.log 2>&1 || stop pyrprof $?
grep -E "^pyr plan|^pyr_band" $O/pyrprof.log | sort | uniq -c | head -20
ok=""
for v in "$@"; do
  ORBX_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc: $(tail -n 1 $O/tests_$v.log)"
  case $rc in 0) ok="$ok $v";; 1) grep -m3 -E "^E  " $O/tests_$v.log;; *) stop $v $rc;; esac
done
tools/variant_serial.sh $TAG base $ok || exit 1
for rep in 1 2; do
  for v in base $ok; do
    if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > $O/bench_${v}_$rep.log 2>&1 || stop bench_$v $?
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]);print('$v rep $rep VALUE',d['value'],d['stage_ms_per_batch'])"
  done
done
