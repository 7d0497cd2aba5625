#!/bin/bash
# The shim driver's latency mode with orbx_extract's host phases
# (ORBX_EXTRACT_PROF=1: staging copy / issue / wait / copy-out, printed per
# extractor at destruction). Usage: tools/shim_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/shimprof
timeout -k 10 200 python3 -c "
import numpy as np
from orb_slam_cuda_amd.synth import SynthSequence, stereo_pair
f = SynthSequence(1, 1241, 376).frames(32)
p = [stereo_pair(1000 + i, 1241, 376) for i in range(32)]
np.ascontiguousarray(f).tofile('gpurun_out/shimprof/mono.u8')
np.ascontiguousarray(np.stack([a for a, b in p])).tofile('gpurun_out/shimprof/l.u8')
np.ascontiguousarray(np.stack([b for a, b in p])).tofile('gpurun_out/shimprof/r.u8')
" || exit 1
ORBX_EXTRACT_PROF=1 timeout -k 10 200 shim/build/orbx_shim_driver --latency gpurun_out/shimprof/mono.u8 \
  gpurun_out/shimprof/l.u8 gpurun_out/shimprof/r.u8 32 1241 376 200 20
