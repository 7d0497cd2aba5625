#!/bin/bash
# Copy the round-4 evidence of tools/r04_evidence_a.sh / _b.sh (gpurun_out/)
# into profiles/ under r04_* names, and refresh the counter files bench.py
# reads (profiles/pmc_traffic.json, profiles/sq_valu.json).
set -e
cd "$(dirname "$0")/.."
A=gpurun_out/ev4; B=gpurun_out/ev4b; P=profiles; R=gpurun_out/prof_r04
last() { tail -n 1 "$1"; }
echo "$(cat .git_rev) ($(date -u +%Y-%m-%d))" > $P/r04_rev.txt
grep -E "PASSED|FAILED|SKIPPED|passed|failed" $A/gpu_tests.log > $P/r04_gpu_tests.txt
cp $A/smoke.log $P/r04_smoke.txt
last $A/bench_default.log > $P/r04_bench.json
# the line re-run after the counter files of this commit are in place (tools/r04_bench_final.sh)
[ -f gpurun_out/ev4c/bench_default.log ] && last gpurun_out/ev4c/bench_default.log > $P/r04_bench.json
cp $R/stats/run_kernel_stats.csv $P/r04_kernel_stats.csv
grep '^{' $R/stats.log | tail -n 1 > $P/r04_bench_profiled.json
cp $R/pmc_traffic.json $P/r04_pmc_traffic.json; cp $R/pmc_traffic.json $P/pmc_traffic.json
cp $R/traffic.txt $P/r04_traffic.txt
cp $A/serial/run_kernel_stats.csv $P/r04_serial_kernel_stats.csv
[ -d $B/sq ] || { echo "part B not collected yet"; ls $P/r04_* | wc -l; exit 0; }
cp $B/sq/summary.txt $P/r04_sq_counters_serial.txt
cp $B/sq_valu.json $P/sq_valu.json
cp $B/fast_phases.txt $P/r04_fast_phases.txt
cp $B/init_phases.txt $P/r04_init_phases.txt
cp $B/h2d.json $P/r04_h2d_link.json
for c in c2 c4 c5 bowmatch bowmatch_serial kitti14 intcatch1080; do
  last $B/$c.log > $P/r04_${c}_bench.json
  cp $B/$c/run_kernel_stats.csv $P/r04_${c}_kernel_stats.csv
done
ls $P/r04_* | wc -l
