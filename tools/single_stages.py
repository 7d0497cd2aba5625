"""Device time per extraction stage of single-frame orbx_extract calls
(ORBX_TIMING=1: stage events, plain stream operations instead of the graph).
Usage: ORBX_TIMING=1 python3 tools/single_stages.py [W H NFEAT NLEVELS]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import orb_slam_cuda_amd as pkg  # noqa: E402
from orb_slam_cuda_amd.synth import SynthSequence  # noqa: E402

W, H, NF, NL = (int(a) for a in (sys.argv[1:5] if len(sys.argv) >= 5 else (1241, 376, 2000, 8)))
assert os.environ.get("ORBX_TIMING") == "1", "run with ORBX_TIMING=1"
frames = SynthSequence(3, W, H).frames(8)
ext = pkg.ORBextractor(NF, 1.2, NL, 20, 7, W, H)
rows = []
for i in range(120):
    ext(frames[i % len(frames)])
    if i >= 20:
        rows.append(ext.stage_times())
names = list(rows[0])
med = {k: float(np.median([r[k] for r in rows])) * 1e3 for k in names}
print(f"{W}x{H} nF {NF} L {NL}: single-frame stage medians (us):",
      ", ".join(f"{k} {v:.1f}" for k, v in med.items()), f"| sum {sum(med.values()):.1f}")
