set -e
mkdir -p gpurun_out
for i in 0 1 2 3 4; do
  ORBX_PYR_PLAN=$i timeout -k 10 120 python bench.py --cpu-sample 0 > gpurun_out/plan$i.json
  ORBX_PYR_PLAN=$i timeout -k 10 120 python bench.py --serial --steps 30 --warmup 5 --cpu-sample 0 > gpurun_out/splan$i.json
done
