#!/bin/bash
# Copy a round's evidence of tools/evidence_a.sh / _b.sh (gpurun_out/) into
# profiles/ under rNN_* names (ROUND=rNN, default r05), and refresh the
# counter files bench.py reads (profiles/pmc_traffic.json, profiles/sq_valu.json).
set -e
cd "$(dirname "$0")/.."
N=${ROUND:-r05}
A=gpurun_out/ev_${N}a; B=gpurun_out/ev_${N}b; C=gpurun_out/ev_${N}c; P=profiles; R=gpurun_out/prof_$N
last() { tail -n 1 "$1"; }
echo "$(cat .git_rev) ($(date -u +%Y-%m-%d))" > $P/${N}_rev.txt
grep -E "PASSED|FAILED|SKIPPED|passed|failed" $A/gpu_tests.log > $P/${N}_gpu_tests.txt
cp $A/smoke.log $P/${N}_smoke.txt
last $A/bench_default.log > $P/${N}_bench.json
# the line re-run after the counter files of this commit are in place (evidence_b.sh's last step)
[ -f $C/bench_default.log ] && last $C/bench_default.log > $P/${N}_bench.json
cp $R/stats/run_kernel_stats.csv $P/${N}_kernel_stats.csv
grep '^{' $R/stats.log | tail -n 1 > $P/${N}_bench_profiled.json
cp $R/pmc_traffic.json $P/${N}_pmc_traffic.json; cp $R/pmc_traffic.json $P/pmc_traffic.json
cp $R/traffic.txt $P/${N}_traffic.txt
cp $A/serial/run_kernel_stats.csv $P/${N}_serial_kernel_stats.csv
[ -d $B/sq ] || { echo "part B not collected yet"; ls $P/${N}_* | wc -l; exit 0; }
cp $B/sq/summary.txt $P/${N}_sq_counters_serial.txt
cp $B/sq_valu.json $P/sq_valu.json
cp $B/fast_phases.txt $P/${N}_fast_phases.txt
cp $B/init_phases.txt $P/${N}_init_phases.txt
cp $B/h2d.json $P/${N}_h2d_link.json
cp $B/intcatch1080_serial/run_kernel_stats.csv $P/${N}_intcatch1080_serial_kernel_stats.csv
cp $B/qt_phases.txt $P/${N}_qt_phases.txt
for c in c2 c4 c5 bowmatch bowmatch_serial kitti14 intcatch1080; do
  last $B/$c.log > $P/${N}_${c}_bench.json
  cp $B/$c/run_kernel_stats.csv $P/${N}_${c}_kernel_stats.csv
done
ls $P/${N}_* | wc -l
