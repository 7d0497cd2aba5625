#!/bin/bash
# A/B of liborbx variants: extraction parity tests, serial kernel averages,
# pipelined bench. Usage: tools/bench_variants_ext.sh base v1 v2 ...
cd "$GRAFT_REPO_ROOT"
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  t=$(timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -n 1)
  echo "$v [$t]"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bv_$v -o run -- python3 bench.py --allow-diag --serial --steps 20 --warmup 5 --cpu-sample 0 > /tmp/bvs.log 2>&1 || exit 1
  python3 tools/stats_brief.py gpurun_out/bv_$v/run_kernel_stats.csv | grep -E "fast|pyr|blur|orient|quad"
  timeout -k 10 120 python3 bench.py --allow-diag --steps 100 --warmup 20 --cpu-sample 0 > /tmp/bv.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('/tmp/bv.log').read().strip().splitlines()[-1]);print('   bench',d['value'],d['ms_per_step'])"
done
