#!/bin/bash
# Host-streamed leg A/B: upload mode, copy-kernel size, stream priority.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/host; mkdir -p $O
run() {  # name, args
  n=$1; shift
  timeout -k 10 150 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-latency --host-steps 40 "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]);h=d['host_stream'];print('$n',h['value'],h['h2d_gb_per_s'],h.get('h2d_frac_of_link_peak'),h['link']['h2d_peak_GBps'],'issue',h['host_issue_ms_per_step'],'ms',h['ms_per_step'])"
}
run kernel_prio_s1 --h2d-mode kernel --h2d-priority --h2d-split 1
run kernel_s1 --h2d-mode kernel --h2d-split 1
run kernel_prio_s1_64 --h2d-mode kernel --h2d-priority --h2d-split 1 --h2d-kernel-wgs 64
run kernel_prio_s1_256 --h2d-mode kernel --h2d-priority --h2d-split 1 --h2d-kernel-wgs 256
run kernel_prio_s1_512 --h2d-mode kernel --h2d-priority --h2d-split 1 --h2d-kernel-wgs 512
run dma_s1 --h2d-split 1
run dma_prio_s1 --h2d-priority --h2d-split 1
run kernel_prio_s1_b128 --h2d-mode kernel --h2d-priority --h2d-split 1 --batch 128 --pool 640
