#!/bin/bash
# KITTI14 pipelined A/B (round 6): lines and pipelined rocprof stats with the
# sorted-key quadtree path and with the legacy rounds, plus LDS budgets.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k14p; mkdir -p $O
for c in kitti kitti14; do ORBX_PLAN_INFO=1 timeout -k 10 120 python3 bench.py --allow-diag --config $c --steps 2 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream 2>&1 | grep "^plan" | sort -u; done
R=1 bash tools/ab.sh "--allow-diag --config kitti14" "ORBX_QT_SORTED=0 --allow-diag --config kitti14" "ORBX_QT_LDS_KB=64 --allow-diag --config kitti14" "ORBX_QT_SORTED=0 --allow-diag" "--allow-diag" || exit 1
for v in sorted legacy; do
  if [ $v = legacy ]; then export ORBX_QT_SORTED=0; else unset ORBX_QT_SORTED; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --allow-diag --config kitti14 --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream > $O/$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/stats_brief.py $O/$v/run_kernel_stats.csv
done
