#!/bin/bash
# A/B sweep of library variants on the GPU box: parity of the extraction
# tests, then serial and pipelined bench lines per variant.
#   tools/variant_sweep.sh base name1 name2 ...   ("base" = the normal build)
set -e
mkdir -p gpurun_out/var
for v in "$@"; do
  if [ "$v" = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py > gpurun_out/var/$v.test.log 2>&1
  timeout -k 10 120 python bench.py --allow-diag --serial --steps 30 --warmup 5 --cpu-sample 0 > gpurun_out/var/$v.serial.json
  timeout -k 10 120 python bench.py --allow-diag --cpu-sample 0 > gpurun_out/var/$v.b1.json
  timeout -k 10 120 python bench.py --allow-diag --cpu-sample 0 > gpurun_out/var/$v.b2.json
done
