#!/bin/bash
# Single-frame latency check (round 6): parity tests of the per-frame path,
# stage times, the device timeline of orbx_extract calls (rocprofv3 kernel +
# copy trace, tools/single_timeline.py) and the shim's latency mode with its
# host phases. Usage: OUT=gpurun_out/x [TESTS="..."] bash tools/lat_check.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/latcheck}
mkdir -p $O
T=${TESTS:-tests/test_gpu_dropin.py tests/test_gpu_extract.py tests/test_shim.py}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ORBX_TIMING=1 timeout -k 10 100 python3 tools/single_stages.py > $O/stages.txt 2>&1 || exit 1
cat $O/stages.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/latency_prof.py 300 > $O/prof.log 2>&1 || exit 1
python3 tools/single_timeline.py $O/prof/run_kernel_trace.csv $O/prof/run_memory_copy_trace.csv | tee $O/timeline.txt
bash tools/shim_prof.sh > $O/shim.log 2>&1 || exit 1
grep -h "host phases\|orbx_extract_ms" $O/shim.log | cut -c1-400
