"""GPU parity of the pose-projection SearchByProjection overloads (liborbx.so,
orbx_project_pose.hip) against the CPU oracle (itself cross-checked against
tests/refpy.py in test_oracle.py):
  * SearchByProjection(CurrentFrame, LastFrame, th, bMono)   src/ORBmatcher.cc:1328-1470
  * SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)  :1472-1599
  * SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)     :290-403
Assignments (including the order-dependent blocking and the rotation check's
clearing, -2) and match counts must be identical."""
import ctypes as C

import numpy as np
import pytest

from posecase import keyframe_case, last_frame_case, sim3_case

pytestmark = pytest.mark.gpu


def _v(a):
    return None if a is None else np.ascontiguousarray(a).ctypes.data_as(C.c_void_p)


def _cam(c):
    from orb_slam_cuda_amd import _lib
    return _lib.camera(c.fx, c.fy, c.cx, c.cy, c.mb, c.mbf, np.array(list(c.Tcw), np.float32))


def gpu_last_frame(pkg, m, c, th, check_ori=True):
    from orb_slam_cuda_amd import _lib
    kps, d, ur = c["kps"], c["desc"], c["uright"]
    sc = np.ascontiguousarray(c["scale"], np.float32)
    out = np.full(max(len(kps), 1), -7, np.int32)
    nm = C.c_int(-1)
    cam = _cam(c["cam"])
    _lib.check(_lib.lib().orbm_search_by_projection_last_frame(
        m.handle, _v(kps), _v(d), len(kps), _v(ur), _lib.GridBounds(*c["bounds"]), _v(sc), len(sc),
        _v(c["blocked"].astype(np.uint8)), C.byref(cam), _v(np.ascontiguousarray(c["Tlw"], np.float32)),
        _v(c["mps"]), _v(c["mpdesc"]), len(c["mps"]), C.c_float(th), int(c["mono"]), int(check_ori), _v(out),
        C.byref(nm)), matcher=True)
    return out[:len(kps)], nm.value


@pytest.mark.parametrize("seed,motion,stereo,th,nmp", [(1, "none", False, 7.0, 2000), (2, "forward", True, 7.0, 2000),
                                                       (3, "backward", True, 15.0, 2500), (4, "none", True, 7.0, 9000),
                                                       (5, "forward", False, 7.0, 0)])
def test_last_frame_parity(pkg, O, seed, motion, stereo, th, nmp):
    c = last_frame_case(O, seed, nmp=nmp, stereo=stereo, motion=motion)
    m = pkg.ORBmatcher(0.9, True, max_kps=4096)
    out, nm = gpu_last_frame(pkg, m, c, th)
    eout, enm = O.search_by_projection_last_frame(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"],
                                                  c["blocked"], c["cam"], c["Tlw"], c["mps"], c["mpdesc"], th,
                                                  c["mono"])
    assert nm == enm and np.array_equal(out, eout)
    if nmp:
        assert nm > 300


def test_last_frame_no_rotation_and_sequential_fallback(pkg, O, monkeypatch):
    c = last_frame_case(O, 6, stereo=True, motion="none")
    m = pkg.ORBmatcher(0.9, False, max_kps=4096)
    out, nm = gpu_last_frame(pkg, m, c, 7.0, check_ori=False)
    eout, enm = O.search_by_projection_last_frame(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"],
                                                  c["blocked"], c["cam"], c["Tlw"], c["mps"], c["mpdesc"], 7.0,
                                                  c["mono"], False)
    assert nm == enm and np.array_equal(out, eout)
    monkeypatch.setenv("ORBX_PROJ_ROUNDS", "1")
    out, nm = gpu_last_frame(pkg, m, c, 7.0)
    eout, enm = O.search_by_projection_last_frame(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"],
                                                  c["blocked"], c["cam"], c["Tlw"], c["mps"], c["mpdesc"], 7.0,
                                                  c["mono"])
    assert nm == enm and np.array_equal(out, eout)


@pytest.mark.parametrize("seed,th,orb_dist,nmp", [(1, 10.0, 100, 2000), (2, 3.0, 64, 3000), (3, 5.0, 50, 12000)])
def test_keyframe_parity(pkg, O, seed, th, orb_dist, nmp):
    from orb_slam_cuda_amd import _lib
    c = keyframe_case(O, seed, nmp=nmp)
    m = pkg.ORBmatcher(0.75, True, max_kps=4096)
    kps = c["kps"]
    sc = np.ascontiguousarray(c["scale"], np.float32)
    out = np.full(len(kps), -7, np.int32)
    nm = C.c_int(-1)
    cam = _cam(c["cam"])
    _lib.check(_lib.lib().orbm_search_by_projection_keyframe(
        m.handle, _v(kps), _v(c["desc"]), len(kps), _lib.GridBounds(*c["bounds"]), _v(sc), len(sc), C.c_float(1.2),
        _v(c["has_mp"]), C.byref(cam), _v(c["mps"]), _v(c["mpdesc"]), len(c["mps"]), C.c_float(th), orb_dist, 1,
        _v(out), C.byref(nm)), matcher=True)
    eout, enm = O.search_by_projection_keyframe(kps, c["desc"], c["bounds"], c["scale"], 1.2, c["has_mp"], c["cam"],
                                                c["mps"], c["mpdesc"], th, orb_dist)
    assert nm.value == enm and np.array_equal(out, eout)
    assert enm > 300


@pytest.mark.parametrize("seed,th,s,nmp", [(1, 10, 1.3, 3000), (2, 5, 0.7, 3000), (3, 10, 2.0, 20000)])
def test_sim3_parity(pkg, O, seed, th, s, nmp):
    from orb_slam_cuda_amd import _lib
    c = sim3_case(O, seed, nmp=nmp, s=s)
    m = pkg.ORBmatcher(0.75, True, max_kps=4096)
    kps = c["kps"]
    sc = np.ascontiguousarray(c["scale"], np.float32)
    out = np.full(len(kps), -7, np.int32)
    nm = C.c_int(-1)
    cam = _cam(c["cam"])
    _lib.check(_lib.lib().orbm_search_by_projection_sim3(
        m.handle, _v(kps), _v(c["desc"]), len(kps), _lib.GridBounds(*c["bounds"]), _v(sc), len(sc), C.c_float(1.2),
        C.byref(cam), _v(c["mps"]), _v(c["mpdesc"]), len(c["mps"]), th, _v(c["matched"]), _v(out), C.byref(nm)),
        matcher=True)
    eout, enm = O.search_by_projection_sim3(kps, c["desc"], c["bounds"], c["scale"], 1.2, c["cam"], c["mps"],
                                            c["mpdesc"], th, c["matched"])
    assert nm.value == enm and np.array_equal(out, eout)
    assert enm > 300


def test_mirror_objects_last_frame_keyframe_sim3(pkg, O):
    """The Python mirror (Frame / KeyFrame / MapPoints, the reference's overload signatures)
    gives the same pointers as the oracle on the same data."""
    from orb_slam_cuda_amd import _lib
    c = last_frame_case(O, 8, stereo=True, motion="forward")
    M = len(c["mps"])
    table = pkg.MapPoints(pos=c["mps"]["pos"], descriptors=c["mpdesc"], nobs=c["mps"]["obs_positive"].astype(int))
    # LastFrame: keypoint i holds map point i (valid ones), outliers where !valid
    lk = np.zeros(M, pkg.KP_DTYPE)
    lk["angle"], lk["octave"] = c["mps"]["angle"], c["mps"]["octave"]
    Last = pkg.Frame(lk, np.zeros((M, 32), np.uint8), mvpMapPoints=np.arange(M), mvbOutlier=~c["mps"]["valid"].astype(bool),
                     mTcw=c["Tlw"])
    # CurrentFrame: blocked keypoints hold a point with observations (index 0 has nobs > 0 or not: pick one that has)
    holder = int(np.nonzero(c["mps"]["obs_positive"])[0][0])
    cur_mp = np.where(c["blocked"] == 1, holder, -1)
    sc = np.ascontiguousarray(c["scale"], np.float32)
    cam = c["cam"]
    Cur = pkg.Frame(c["kps"], c["desc"], *c["bounds"], mvuRight=c["uright"], mb=cam.mb, mbf=cam.mbf,
                    mvScaleFactors=sc, mvpMapPoints=cur_mp.copy(), fx=cam.fx, fy=cam.fy, cx=cam.cx, cy=cam.cy,
                    mTcw=np.array(list(cam.Tcw), np.float32).reshape(3, 4), mpMap=table)
    m = pkg.ORBmatcher(0.9, True, max_kps=4096)
    nm = m.SearchByProjection(Cur, Last, 7.0, c["mono"])
    eout, enm = O.search_by_projection_last_frame(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"],
                                                  c["blocked"], c["cam"], c["Tlw"], c["mps"], c["mpdesc"], 7.0,
                                                  c["mono"])
    want = cur_mp.copy()
    want[eout >= 0] = eout[eout >= 0]
    want[eout == -2] = -1
    assert nm == enm and np.array_equal(Cur.mvpMapPoints, want)
    # Sim3 through the mirror: vpMatched updated in place
    s3 = sim3_case(O, 9, nmp=2500)
    tab = pkg.MapPoints(pos=s3["mps"]["pos"], descriptors=s3["mpdesc"], normal=s3["mps"]["normal"],
                        min_distance=s3["mps"]["min_distance"], max_distance=s3["mps"]["max_distance"],
                        bad=~s3["mps"]["valid"].astype(bool))
    kf = pkg.KeyFrame(s3["kps"], s3["desc"], np.full(len(s3["kps"]), -1), mnMinX=0.0, mnMaxX=1241.0, mnMinY=0.0,
                      mnMaxY=376.0, fx=s3["cam"].fx, fy=s3["cam"].fy, cx=s3["cam"].cx, cy=s3["cam"].cy,
                      mvScaleFactors=np.ascontiguousarray(s3["scale"], np.float32), mpMap=tab)
    vpMatched = [-1] * len(s3["kps"])
    nm = m.SearchByProjection(kf, np.array(list(s3["cam"].Tcw), np.float32).reshape(3, 4), list(range(2500)),
                              vpMatched, 10)
    eout, enm = O.search_by_projection_sim3(s3["kps"], s3["desc"], s3["bounds"], s3["scale"], 1.2, s3["cam"],
                                            s3["mps"], s3["mpdesc"], 10, None)
    assert nm == enm and np.array_equal(np.array(vpMatched), eout)
    assert _lib.ORBM_PROJ_SIM3 == 3


def test_pose_batch_mixed_frames(pkg, O):
    """orbm_search_by_projection_pose_batch: 4 motion-model frames of different sizes in one launch."""
    from orb_slam_cuda_amd import _lib
    B, K, M = 4, 2100, 4000
    cases = [last_frame_case(O, 30 + i, nmp=2000 + 500 * i, stereo=True, motion=["none", "forward", "backward",
                                                                                 "none"][i]) for i in range(B)]
    kp = np.zeros((B, K), pkg.KP_DTYPE); ds = np.zeros((B, K, 32), np.uint8); ur = np.full((B, K), -1, np.float32)
    bl = np.zeros((B, K), np.uint8); mp = np.zeros((B, M), _lib.MAP_POINT_WORLD_DTYPE); md = np.zeros((B, M, 32), np.uint8)
    n = np.zeros(B, np.int32); nmp = np.zeros(B, np.int32)
    poses = (_lib.OrbmPose * B)()
    for i, c in enumerate(cases):
        n[i], nmp[i] = len(c["kps"]), len(c["mps"])
        kp[i, :n[i]] = c["kps"]; ds[i, :n[i]] = c["desc"]; bl[i, :n[i]] = c["blocked"]; ur[i, :n[i]] = c["uright"]
        mp[i, :nmp[i]] = c["mps"].view(_lib.MAP_POINT_WORLD_DTYPE); md[i, :nmp[i]] = c["mpdesc"]
        cam = _cam(c["cam"])
        _lib.check(_lib.lib().orbm_prepare_pose(_lib.ORBM_PROJ_LAST_FRAME, C.byref(cam), _v(c["Tlw"]), int(c["mono"]),
                                                C.byref(poses[i])), matcher=True)
    pz = np.frombuffer(bytes(poses), np.uint8)
    dev = {}
    for name, a in dict(kp=kp, ds=ds, ur=ur, bl=bl, mp=mp, md=md, n=n, nmp=nmp, pz=pz).items():
        dev[name] = _lib.DeviceArray(a.nbytes)
        dev[name].upload(np.ascontiguousarray(a))
    d_out, d_nm = _lib.DeviceArray(B * K * 4), _lib.DeviceArray(4 * B)
    m = pkg.ORBmatcher(0.9, True, max_pairs=B, max_kps=K)
    sc = np.ascontiguousarray(cases[0]["scale"], np.float32)
    s = _lib.Stream()
    v = lambda a: C.c_void_p(a.ptr)
    _lib.check(_lib.lib().orbm_search_by_projection_pose_batch(
        m.handle, _lib.ORBM_PROJ_LAST_FRAME, v(dev["kp"]), v(dev["ds"]), v(dev["n"]), K, v(dev["ur"]),
        _lib.GridBounds(*cases[0]["bounds"]), _v(sc), len(sc), C.c_float(1.2), v(dev["bl"]), v(dev["pz"]),
        v(dev["mp"]), v(dev["md"]), v(dev["nmp"]), M, B, C.c_float(7.0), 100, 1, None, v(d_out), v(d_nm), s.s),
        matcher=True)
    s.synchronize()
    out = d_out.download(B * K, np.int32).reshape(B, K)
    nm = d_nm.download(B, np.int32)
    for i, c in enumerate(cases):
        eout, enm = O.search_by_projection_last_frame(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"],
                                                      c["blocked"], c["cam"], c["Tlw"], c["mps"], c["mpdesc"], 7.0,
                                                      c["mono"])
        assert nm[i] == enm and np.array_equal(out[i, :n[i]], eout)
