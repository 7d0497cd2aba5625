#!/bin/bash
# FAST phase clocks (ORBX_FAST_PROF=1) of liborbx variants. Usage: tools/fast_prof.sh base v1 ...
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  echo "== $v"
  ORBX_FAST_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 > /tmp/fp.log 2>&1 || { tail -5 /tmp/fp.log; exit 1; }
  grep "^fast" /tmp/fp.log | tail -2
done
