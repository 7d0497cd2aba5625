"""Device time of the band pyramid per plan (ORBX_PYR_PLAN forced per launch)
for a batch of B resident frames, from the extractor's stage events
(ORBX_TIMING=1). Prints the plan table (ORBX_PYR_PROF=1) on stderr first.
ORBX_PYR_KEEP="nb:nct,..." plans exactly those tilings.
Usage: ORBX_TIMING=1 [ORBX_PYR_KEEP=...] python3 tools/pyr_plans.py [B W H NLEVELS]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import orb_slam_cuda_amd as pkg  # noqa: E402
from orb_slam_cuda_amd import _lib  # noqa: E402
from orb_slam_cuda_amd.synth import SynthSequence  # noqa: E402

B, W, H, NL = (int(a) for a in (sys.argv[1:5] if len(sys.argv) >= 5 else (32, 1241, 376, 8)))
assert os.environ.get("ORBX_TIMING") == "1", "run with ORBX_TIMING=1"
pitch = (W + 63) & ~63
frames = SynthSequence(5, W, H).frames(B)
img = np.zeros((B, H, pitch), np.uint8)
img[:, :, :W] = frames
d = _lib.DeviceArray(img.nbytes)
d.upload(img)
ext = pkg.ORBextractor(2000, 1.2, NL, 20, 7, W, H, max_batch=B)
cap = ext.frame_capacity
dk, dd, dc = _lib.DeviceArray(B * cap * 28), _lib.DeviceArray(B * cap * 32), _lib.DeviceArray(B * 4)
# the plan table, from a child process with ORBX_PYR_PROF=1 (profiling in
# this process would add a sync and a copy to every launch)
import re  # noqa: E402
import subprocess  # noqa: E402
code = ("import sys; sys.path.insert(0, %r); import orb_slam_cuda_amd as pkg; "
        "pkg.ORBextractor(2000, 1.2, %d, 20, 7, %d, %d, max_batch=%d)") % (
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), NL, W, H, B)
env = dict(os.environ, ORBX_PYR_PROF="1")
env.pop("ORBX_TIMING", None)
out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True).stderr
names = {int(m.group(1)): f"{m.group(2)}:{m.group(3)}" for m in
         re.finditer(r"pyr plan (\d+): (\d+) bands x (\d+) column tiles", out)}
res = []
for plan in list(range(8)) + [-1]:
    if plan >= 0:
        os.environ["ORBX_PYR_PLAN"] = str(plan)
    else:
        os.environ.pop("ORBX_PYR_PLAN", None)
    t = []
    for i in range(25):
        ext.extract_batch_device(d.ptr, B, H * pitch, pitch, dk.ptr, dd.ptr, dc.ptr)
        if i >= 5:
            t.append(ext.stage_times()["Pyramid/Resize"])
    res.append((plan, float(np.median(t)) * 1e3))
lab = lambda p: names.get(p, "pick" if p < 0 else f"{p}(none)")
print(f"B {B} {W}x{H} L {NL}: pyramid us per plan:", ", ".join(f"{lab(p)}: {v:.1f}" for p, v in res))
