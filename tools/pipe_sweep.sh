set -e
cd $GRAFT_REPO_ROOT
for a in "" "--no-match" "--priority" "--carry ext" "--split 4" "--no-match --split 4" "--no-match --split 1"; do
  echo "== $a" >> gpurun_out/pipe_sweep.log
  timeout -k 10 120 python3 bench.py --steps 40 --warmup 10 --cpu-sample 0 $a >> gpurun_out/pipe_sweep.log 2>&1
done
