"""Times orbm_search_by_projection_batch on resident synthetic tracking cases
(tests/projcase.py: 2000 keypoints, 3000 projected map points per frame).
Usage: python tools/proj_timing.py [frames]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import orb_slam_cuda_amd as pkg  # noqa: E402
from oracle import oracle as O  # noqa: E402  (test-data generation only)
from orb_slam_cuda_amd import _lib  # noqa: E402
from projcase import projection_case  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
K, M = 2100, 3000
base = [projection_case(O, 100 + i, nmp=M, stereo=bool(i % 2)) for i in range(min(B, 8))]
kp = np.zeros((B, K), pkg.KP_DTYPE); ds = np.zeros((B, K, 32), np.uint8); ur = np.full((B, K), -1, np.float32)
bl = np.zeros((B, K), np.uint8); mp = np.zeros((B, M), _lib.MAP_POINT_PROJ_DTYPE); md = np.zeros((B, M, 32), np.uint8)
n = np.zeros(B, np.int32); nmp = np.zeros(B, np.int32)
for i in range(B):
    k, d, u, bounds, scale, b, p, q = base[i % len(base)]
    n[i], nmp[i] = len(k), len(p)
    kp[i, :n[i]] = k; ds[i, :n[i]] = d; bl[i, :n[i]] = b
    if u is not None:
        ur[i, :n[i]] = u
    mp[i, :nmp[i]] = p.view(_lib.MAP_POINT_PROJ_DTYPE); md[i, :nmp[i]] = q
dev = {}
for name, a in dict(kp=kp, ds=ds, ur=ur, bl=bl, mp=mp, md=md, n=n, nmp=nmp).items():
    dev[name] = _lib.DeviceArray(a.nbytes)
    dev[name].upload(np.ascontiguousarray(a))
d_out, d_nm = _lib.DeviceArray(B * K * 4), _lib.DeviceArray(4 * B)
m = pkg.ORBmatcher(0.8, True, max_pairs=B, max_kps=K)
sc = np.ascontiguousarray(base[0][4], np.float32)
s = _lib.Stream()
v = lambda a: C.c_void_p(a.ptr)


def run():
    _lib.check(_lib.lib().orbm_search_by_projection_batch(
        m.handle, v(dev["kp"]), v(dev["ds"]), v(dev["n"]), K, v(dev["ur"]), _lib.GridBounds(*base[0][3]),
        sc.ctypes.data_as(C.c_void_p), len(sc), v(dev["bl"]), v(dev["mp"]), v(dev["md"]), v(dev["nmp"]), M, B,
        C.c_float(3.0), C.c_float(0.8), v(d_out), v(d_nm), s.s), matcher=True)


for _ in range(3):
    run()
e0, e1 = _lib.Event(), _lib.Event()
N = 20
e0.record(s)
for _ in range(N):
    run()
e1.record(s)
s.synchronize()
print(f"frames={B} map_points={M} ms_per_call={e0.elapsed_ms(e1) / N:.4f} "
      f"matches_mean={d_nm.download(B, np.int32).mean():.1f}")
