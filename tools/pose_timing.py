"""Times orbm_search_by_projection_pose_batch on resident synthetic cases
(tests/posecase.py: ~2000 keypoints per frame; LAST_FRAME: one record per
last-frame keypoint, KEYFRAME / SIM3: map points of a keyframe / loop set).
Usage: python tools/pose_timing.py [frames] [mode: last|kf|sim3] [points]"""
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
import posecase as pc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
mode = sys.argv[2] if len(sys.argv) > 2 else "last"
M = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
K = 2100
MODE = {"last": _lib.ORBM_PROJ_LAST_FRAME, "kf": _lib.ORBM_PROJ_KEYFRAME, "sim3": _lib.ORBM_PROJ_SIM3}[mode]
if mode == "last":
    base = [pc.last_frame_case(O, 100 + i, nmp=M, stereo=bool(i % 2), motion=["none", "forward"][i % 2])
            for i in range(min(B, 8))]
elif mode == "kf":
    base = [pc.keyframe_case(O, 100 + i, nmp=M) for i in range(min(B, 8))]
else:
    base = [pc.sim3_case(O, 100 + i, nmp=M) for i in range(min(B, 8))]
kp = np.zeros((B, K), pkg.KP_DTYPE); ds = np.zeros((B, K, 32), np.uint8); ur = np.full((B, K), -1, np.float32)
bl = np.zeros((B, K), np.uint8); mp = np.zeros((B, M), _lib.MAP_POINT_WORLD_DTYPE); md = np.zeros((B, M, 32), np.uint8)
n = np.zeros(B, np.int32); nmp = np.zeros(B, np.int32)
poses = (_lib.OrbmPose * B)()
for i in range(B):
    c = base[i % len(base)]
    n[i], nmp[i] = len(c["kps"]), len(c["mps"])
    kp[i, :n[i]] = c["kps"]; ds[i, :n[i]] = c["desc"]
    blk = c.get("blocked", c.get("has_mp"))
    if blk is None:
        blk = (c["matched"] >= 0).astype(np.uint8)
    bl[i, :n[i]] = blk
    if c.get("uright") is not None:
        ur[i, :n[i]] = c["uright"]
    mp[i, :nmp[i]] = c["mps"].view(_lib.MAP_POINT_WORLD_DTYPE); md[i, :nmp[i]] = c["mpdesc"]
    cam = _lib.camera(c["cam"].fx, c["cam"].fy, c["cam"].cx, c["cam"].cy, c["cam"].mb, c["cam"].mbf,
                      np.array(list(c["cam"].Tcw), np.float32))
    Tlw = np.ascontiguousarray(c["Tlw"], np.float32) if mode == "last" else None
    _lib.check(_lib.lib().orbm_prepare_pose(MODE, C.byref(cam), None if Tlw is None else Tlw.ctypes.data_as(C.c_void_p),
                                            int(c.get("mono", 0)), C.byref(poses[i])), matcher=True)
pz = np.frombuffer(bytes(poses), np.uint8)
dev = {}
for name, a in dict(kp=kp, ds=ds, ur=ur, bl=bl, mp=mp, md=md, n=n, nmp=nmp, pz=pz).items():
    dev[name] = _lib.DeviceArray(a.nbytes)
    dev[name].upload(np.ascontiguousarray(a))
d_out, d_nm = _lib.DeviceArray(B * K * 4), _lib.DeviceArray(4 * B)
m = pkg.ORBmatcher(0.8, True, max_pairs=B, max_kps=K)
sc = np.ascontiguousarray(base[0]["scale"], np.float32)
s = _lib.Stream()
v = lambda a: C.c_void_p(a.ptr)
th, dist_th = {"last": (7.0, 100), "kf": (10.0, 100), "sim3": (10.0, 50)}[mode]


def run():
    _lib.check(_lib.lib().orbm_search_by_projection_pose_batch(
        m.handle, MODE, v(dev["kp"]), v(dev["ds"]), v(dev["n"]), K, v(dev["ur"]) if mode == "last" else None,
        _lib.GridBounds(*base[0]["bounds"]), sc.ctypes.data_as(C.c_void_p), len(sc), C.c_float(1.2), v(dev["bl"]),
        v(dev["pz"]), v(dev["mp"]), v(dev["md"]), v(dev["nmp"]), M, B, C.c_float(th), dist_th, 1, None, v(d_out),
        v(d_nm), s.s), matcher=True)


for _ in range(3):
    run()
e0, e1 = _lib.Event(), _lib.Event()
N = 20
e0.record(s)
for _ in range(N):
    run()
e1.record(s)
s.synchronize()
print(f"mode={mode} frames={B} points={M} ms_per_call={e0.elapsed_ms(e1) / N:.4f} "
      f"matches_mean={d_nm.download(B, np.int32).mean():.1f}", flush=True)
