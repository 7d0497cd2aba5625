#!/bin/bash
# Quadtree A/B in one GPU call: extraction parity tests, per-level phase
# clocks (ORBX_QT_PROF=1), serial kernel averages and the pipelined bench.
# Usage: tools/qt_prof.sh [variant ...]   ("base" = the in-tree library)
cd "$GRAFT_REPO_ROOT"
for v in ${@:-base}; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  echo "== $v"
  ORBX_QT_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 > /tmp/qtp.log 2>&1 || { tail -20 /tmp/qtp.log; exit 1; }
  grep "^quadtree" /tmp/qtp.log | tail -8
done
