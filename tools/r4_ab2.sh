#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/init4; mkdir -p $O
ORBX_INIT_PROF=1 timeout -k 10 120 python3 tools/init_timing.py 64 > $O/prof.log 2>&1
tail -n 3 $O/prof.log
tools/variant_serial.sh r4b base serarcs
tools/host_ab.sh
