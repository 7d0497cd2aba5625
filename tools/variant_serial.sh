#!/bin/bash
# Per-kernel serial timings (rocprofv3 --stats, every kernel alone on the chip)
# of liborbx variants built by tools/variant.sh.
# Usage: tools/variant_serial.sh TAG base v1 v2 ...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  OUT=gpurun_out/vs_${TAG}_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --allow-diag --serial --steps 20 --warmup 3 --cpu-sample 0 --no-latency --no-host-stream > $OUT.log 2>&1 || { echo "$v failed"; tail -5 $OUT.log; exit 1; }
  echo "== $v"
  python3 tools/stats_brief.py $OUT/run_kernel_stats.csv | grep -v rocclr
done
