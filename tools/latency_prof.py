"""Single-frame orbx_extract calls (the latency API Tracking uses) for a
rocprofv3 kernel trace: per-kernel durations of one 1241x376 frame.
Usage: rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/latency_prof.py [calls]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import orb_slam_cuda_amd as pkg  # noqa: E402
from orb_slam_cuda_amd.synth import SynthSequence  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
W, H = 1241, 376
frames = SynthSequence(1, W, H).frames(16)
ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
ts = []
for i in range(n + 20):
    t0 = time.perf_counter()
    kps, desc = ext(frames[i % len(frames)])
    if i >= 20:
        ts.append(time.perf_counter() - t0)
print(f"orbx_extract via ORBextractor.__call__: median {np.median(ts) * 1e3:.4f} ms over {n} calls, "
      f"{len(kps)} keypoints")
