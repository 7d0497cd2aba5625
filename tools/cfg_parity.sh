#!/bin/bash
# GPU parity at the reference's shipped yaml settings (tests/test_gpu_configs.py,
# the kitti14 / intcatch1080 timed pipelines), then the KITTI14 single-frame
# case under a kernel trace so the >8-level kernel instantiations are on record.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cfg; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py "tests/test_gpu_pipeline.py::test_timed_pipeline_matches_oracle" tests/test_shim.py tests/test_gpu_match.py tests/test_gpu_extract.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -n 60 $O/tests.log; exit 1; }
tail -n 3 $O/tests.log
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -m pytest "tests/test_gpu_configs.py::test_yaml_batch_parity[KITTI14]" -x -q > $O/trace.log 2>&1
cut -d, -f1-4 $O/trace/run_kernel_stats.csv
