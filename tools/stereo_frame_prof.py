"""Stereo Frame calls for a rocprofv3 trace: ExtractStereo (orbm_stereo_frame,
one device round trip) on KITTI-sized pairs, then the reference-structured
sequence (two extractor calls, ComputeStereoMatchesLast), host medians printed.
Usage: rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/stereo_frame_prof.py [calls]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import orb_slam_cuda_amd as pkg  # noqa: E402
from orb_slam_cuda_amd.synth import stereo_pair  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
W, H = 1241, 376
pairs = [stereo_pair(1000 + i, W, H) for i in range(8)]
eL = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
eR = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
m = pkg.ORBmatcher(max_kps=4096)
mb, mbf = 0.54, 0.54 * 718.856
ts = []
for i in range(n + 20):
    L, R = pairs[i % len(pairs)]
    t0 = time.perf_counter()
    pkg.ExtractStereo(eL, eR, L, R, m, mb, mbf)
    if i >= 20:
        ts.append(time.perf_counter() - t0)
print(f"ExtractStereo: median {np.median(ts) * 1e3:.4f} ms over {n} calls (Python, ctypes + numpy copies included)")
