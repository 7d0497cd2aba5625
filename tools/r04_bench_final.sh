#!/bin/bash
# The default bench line after the counter files (sq_valu.json,
# pmc_traffic.json) of the same commit are in profiles/, then variant A/Bs.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ev4c
timeout -k 10 400 python3 bench.py > gpurun_out/ev4c/bench_default.log 2>&1 || { tail -5 gpurun_out/ev4c/bench_default.log; exit 1; }
tail -n 1 gpurun_out/ev4c/bench_default.log | cut -c1-200
[ $# -gt 0 ] && bash tools/var_ab.sh "$@"
exit 0
