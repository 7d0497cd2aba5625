set -e
bash tools/profile_round.sh main --steps 30 --warmup 5 > gpurun_out/prof_main.txt 2>&1
cd /tmp; export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_extra
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_extra/stereo -o run -- python3 bench.py --config stereo --steps 30 --warmup 5 --cpu-sample 0 > gpurun_out/prof_extra/stereo.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_extra/bow -o run -- python3 bench.py --bow --serial --steps 30 --warmup 5 --cpu-sample 0 > gpurun_out/prof_extra/bow.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_extra/proj -o run -- python3 tools/proj_timing.py 64 > gpurun_out/prof_extra/proj.log 2>&1
echo all done
