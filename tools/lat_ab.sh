#!/bin/bash
# Latency A/B of the shim driver's latency mode (tools/shim_prof.sh) over
# environment settings, after the per-frame parity tests. Usage:
#   OUT=gpurun_out/x bash tools/lat_ab.sh "" "ORBX_BLUR_FORK=1" "ORBX_STAGE_THREAD=0" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/latab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dropin.py tests/test_shim.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
i=0
for v in "$@"; do
  i=$((i + 1))
  env $v ORBX_STEREO_PROF=1 bash tools/shim_prof.sh > $O/v$i.log 2>&1 || { echo "variant '$v' failed"; tail -5 $O/v$i.log; exit 1; }
  echo "== '$v'"
  grep -h "stereo_frame host" $O/v$i.log | head -3
  grep -o '"orbx_extract_ms": {[^}]*}\|"operator_ms": {[^}]*}\|"stereo_frame[a-z_]*": {[^}]*}' $O/v$i.log
done
