#!/bin/bash
# A round's evidence, part A (ROUND=rNN, default r05) (one GPU call): the GPU suite, smoke(), the default
# bench line, pipelined rocprofv3 stats + FETCH_SIZE / WRITE_SIZE passes,
# serial stats. Stops at the first failing step.
set -e
cd "$GRAFT_REPO_ROOT"
R=${ROUND:-r05}
O=gpurun_out/ev_${R}a; mkdir -p $O
git_rev=$(cat .git_rev 2>/dev/null || echo unknown); echo "rev $git_rev"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -n 40 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.log 2>&1
tail -n 1 $O/bench_default.log | cut -c1-300
bash tools/profile_round.sh $R --steps 30 --warmup 5 > $O/prof_main.txt 2>&1
cd /tmp; export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- python3 bench.py --serial --steps 30 --warmup 5 --cpu-sample 0 --no-latency --no-host-stream > $O/serial.log 2>&1
python3 tools/stats_brief.py $O/serial/run_kernel_stats.csv
echo all-done
