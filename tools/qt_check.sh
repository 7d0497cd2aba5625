set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=r5h NO_SHIM=1 TESTS="tests/test_gpu_extract.py tests/test_gpu_configs.py tests/test_gpu_runtime.py" bash tools/gpu_check.sh || exit 1
BENCH_ARGS="--config intcatch1080" OUT=r5h_ic NO_SHIM=1 bash tools/gpu_check.sh || exit 1
bash tools/qt_prof.sh || exit 1
ORBX_QT_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 --config intcatch1080 2>&1 | grep "^quadtree" | tail -3
