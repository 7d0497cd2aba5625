#!/bin/bash
# KITTI14 regression check (round 6): the line with the legacy quadtree rounds,
# and serial per-kernel stats of the current library and of the round-5 one.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k14; mkdir -p $O
R=1 bash tools/ab.sh "--allow-diag --config kitti14" "ORBX_QT_SORTED=0 --allow-diag --config kitti14" || exit 1
for v in cur r05; do
  if [ $v = r05 ]; then export ORBX_LIB_VARIANT=r05; else unset ORBX_LIB_VARIANT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --allow-diag --serial --config kitti14 --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream > $O/$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/stats_brief.py $O/$v/run_kernel_stats.csv
done
