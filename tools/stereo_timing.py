"""Times orbm_compute_stereo_matches_batch alone on a resident batch (tuning aid).
Usage: python tools/stereo_timing.py [pairs]; env ORBX_STEREO_GROUPS / ORBX_STEREO_STOP."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import orb_slam_cuda_amd as pkg  # noqa: E402
from orb_slam_cuda_amd import _lib  # noqa: E402
from orb_slam_cuda_amd.synth import stereo_pair  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 1241, 376
pairs = [stereo_pair(100 + i, W, H) for i in range(P)]
frames = np.ascontiguousarray(np.stack([p[0] for p in pairs] + [p[1] for p in pairs]))
ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=2 * P)
cap = ext.frame_capacity
d_in = _lib.DeviceArray(frames.nbytes)
d_in.upload(frames)
d_kp, d_desc, d_n = (_lib.DeviceArray(2 * P * cap * 28), _lib.DeviceArray(2 * P * cap * 32), _lib.DeviceArray(8 * P))
s = _lib.Stream()
ext.extract_batch_device(d_in.ptr, 2 * P, H * W, W, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
m = pkg.ORBmatcher(max_pairs=P, max_kps=cap)
d_u, d_d, d_k = _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * 4)
kpb, db = P * cap * 28, P * cap * 32
L = _lib.lib()


def run():
    _lib.check(L.orbm_compute_stereo_matches_batch(
        m.handle, ext.handle, 0, ext.handle, P, C.c_void_p(d_kp.ptr), C.c_void_p(d_desc.ptr), C.c_void_p(d_n.ptr),
        C.c_void_p(d_kp.ptr + kpb), C.c_void_p(d_desc.ptr + db), C.c_void_p(d_n.ptr + 4 * P), cap, P,
        C.c_float(0.54), C.c_float(0.54 * 718.856), C.c_void_p(d_u.ptr), C.c_void_p(d_d.ptr), C.c_void_p(d_k.ptr),
        s.s), matcher=True)


for _ in range(5):
    run()
e0, e1 = _lib.Event(), _lib.Event()
N = 50
e0.record(s)
for _ in range(N):
    run()
e1.record(s)
s.synchronize()
print(f"groups={os.environ.get('ORBX_STEREO_GROUPS', 'auto')} stop={os.environ.get('ORBX_STEREO_STOP', '0')} "
      f"ms_per_call={e0.elapsed_ms(e1) / N:.4f} kept_mean={d_k.download(P, np.int32).mean():.1f}")
