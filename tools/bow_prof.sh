#!/bin/bash
# SearchByBoW batch per-variant: serial kernel average and the per-workgroup
# phase report (ORBX_BOW_PROF=1). Usage: tools/bow_prof.sh base v1 ...
cd "$GRAFT_REPO_ROOT"
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  echo "== $v"
  OUT=gpurun_out/bp_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --allow-diag --bow-match --serial --steps 10 --warmup 2 --cpu-sample 0 --no-latency --no-host-stream > $OUT.log 2>&1 || { tail -3 $OUT.log; exit 1; }
  python3 tools/stats_brief.py $OUT/run_kernel_stats.csv | grep bow
  ORBX_BOW_PROF=1 timeout -k 10 100 python3 bench.py --allow-diag --bow-match --serial --steps 1 --warmup 1 --cpu-sample 0 --no-latency --no-host-stream --pool 64 2>&1 | grep "^bow" | head -4
done
