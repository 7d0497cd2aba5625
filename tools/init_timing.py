"""Times orbm_search_for_initialization_batch (and orbm_hamming_top2) alone on a
resident batch of 64 (t, t-1) pairs of extracted frames (tuning aid; per-kernel
times: run it under rocprofv3 --kernel-trace --stats)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import orb_slam_cuda_amd as pkg  # noqa: E402
from orb_slam_cuda_amd import _lib  # noqa: E402
from orb_slam_cuda_amd.synth import SynthSequence  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 1241, 376
frames = np.ascontiguousarray(SynthSequence(3, W, H).frames(B + 1))
ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=B + 1)
cap = ext.frame_capacity
d_in = _lib.DeviceArray(frames.nbytes)
d_in.upload(frames)
d_kp, d_desc, d_n = _lib.DeviceArray((B + 1) * cap * 28), _lib.DeviceArray((B + 1) * cap * 32), _lib.DeviceArray(4 * (B + 1))
s = _lib.Stream()
ext.extract_batch_device(d_in.ptr, B + 1, H * W, W, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
m = pkg.ORBmatcher(0.9, True, max_pairs=B, max_kps=cap)
d_m12, d_nm = _lib.DeviceArray(B * cap * 4), _lib.DeviceArray(4 * B)
d_bi, d_bd, d_sd = (_lib.DeviceArray(B * cap * 4) for _ in range(3))
L = _lib.lib()
v = C.c_void_p
bounds = _lib.GridBounds(0.0, float(W), 0.0, float(H))
which = os.environ.get("WHICH", "init")


def run():
    if which == "init":
        _lib.check(L.orbm_search_for_initialization_batch(
            m.handle, v(d_kp.ptr), v(d_desc.ptr), v(d_n.ptr), v(d_kp.ptr + cap * 28), v(d_desc.ptr + cap * 32),
            v(d_n.ptr + 4), cap, B, bounds, None, 100, C.c_float(0.9), 1, v(d_m12.ptr), v(d_nm.ptr), s.s),
            matcher=True)
    else:
        _lib.check(L.orbm_hamming_top2(m.handle, v(d_desc.ptr + cap * 32), cap * 32, v(d_n.ptr + 4), cap,
                                       v(d_desc.ptr), cap * 32, v(d_n.ptr), B, v(d_bi.ptr), v(d_bd.ptr),
                                       v(d_sd.ptr), s.s), matcher=True)


for _ in range(3):
    run()
e0, e1 = _lib.Event(), _lib.Event()
N = 20
e0.record(s)
for _ in range(N):
    run()
e1.record(s)
s.synchronize()
print(f"{which} cap={cap} pairs={B} ms_per_call={e0.elapsed_ms(e1) / N:.4f} "
      f"matches_mean={d_nm.download(B, np.int32).mean():.1f}")
