set -e
cd $GRAFT_REPO_ROOT
for a in "--batch 64 --split 2" "--batch 64 --split 1" "--batch 128 --split 2" "--batch 128 --split 4" "--batch 256 --split 4" "--batch 64 --split 2 --serial"; do
  echo "== $a" >> gpurun_out/sweep.log
  timeout -k 10 120 python3 bench.py --steps 40 --warmup 10 --cpu-sample 0 $a >> gpurun_out/sweep.log 2>&1
done
