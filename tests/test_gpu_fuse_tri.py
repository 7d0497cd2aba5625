"""GPU parity of Fuse (both overloads, matching part), SearchBySim3 and
SearchForTriangulation (liborbx.so: orbx_project_pose.hip modes FUSE /
FUSE_SIM3 / SIM3_MATCH, orbx_triangulate.hip) against the CPU oracle (itself
cross-checked against tests/refpy.py in test_oracle.py)."""
import ctypes as C

import numpy as np
import pytest

from posecase import fuse_case, sim3_case, sim3_match_case, triangulation_case

pytestmark = pytest.mark.gpu


def _v(a):
    return None if a is None else np.ascontiguousarray(a).ctypes.data_as(C.c_void_p)


def _cam(c):
    from orb_slam_cuda_amd import _lib
    return _lib.camera(c.fx, c.fy, c.cx, c.cy, c.mb, c.mbf, np.array(list(c.Tcw), np.float32))


@pytest.mark.parametrize("seed,stereo,th,nmp", [(1, True, 3.0, 3000), (2, False, 3.0, 3000), (3, True, 5.0, 15000)])
def test_fuse_parity(pkg, O, seed, stereo, th, nmp):
    from orb_slam_cuda_amd import _lib
    c = fuse_case(O, seed, nmp=nmp, stereo=stereo)
    m = pkg.ORBmatcher(0.6, True, max_kps=4096)
    sc = np.ascontiguousarray(c["scale"], np.float32)
    isg = np.ascontiguousarray(c["inv_sigma2"], np.float32)
    out = np.full(nmp, -7, np.int32)
    nf = C.c_int(-1)
    cam = _cam(c["cam"])
    _lib.check(_lib.lib().orbm_fuse(m.handle, _v(c["kps"]), _v(c["desc"]), len(c["kps"]), _v(c["uright"]),
                                    _lib.GridBounds(*c["bounds"]), _v(sc), _v(isg), len(sc), C.c_float(1.2),
                                    C.byref(cam), _v(c["mps"]), _v(c["mpdesc"]), nmp, C.c_float(th), _v(out),
                                    C.byref(nf)), matcher=True)
    eout, enf = O.fuse(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"], c["inv_sigma2"], 1.2, c["cam"],
                       c["mps"], c["mpdesc"], th)
    assert nf.value == enf and np.array_equal(out, eout) and enf > 500


@pytest.mark.parametrize("seed,th,s", [(1, 4.0, 1.3), (2, 4.0, 0.6)])
def test_fuse_sim3_parity(pkg, O, seed, th, s):
    from orb_slam_cuda_amd import _lib
    c = sim3_case(O, seed, nmp=4000, s=s)
    m = pkg.ORBmatcher(0.6, True, max_kps=4096)
    sc = np.ascontiguousarray(c["scale"], np.float32)
    out = np.full(4000, -7, np.int32)
    nf = C.c_int(-1)
    cam = _cam(c["cam"])
    _lib.check(_lib.lib().orbm_fuse_sim3(m.handle, _v(c["kps"]), _v(c["desc"]), len(c["kps"]),
                                         _lib.GridBounds(*c["bounds"]), _v(sc), len(sc), C.c_float(1.2), C.byref(cam),
                                         _v(c["mps"]), _v(c["mpdesc"]), 4000, C.c_float(th), _v(out), C.byref(nf)),
               matcher=True)
    eout, enf = O.fuse_sim3(c["kps"], c["desc"], c["bounds"], c["scale"], 1.2, c["cam"], c["mps"], c["mpdesc"], th)
    assert nf.value == enf and np.array_equal(out, eout) and enf > 500


@pytest.mark.parametrize("seed,s12,th", [(1, 1.0, 7.5), (2, 1.08, 7.5), (3, 1.0, 15.0)])
def test_search_by_sim3_parity(pkg, O, seed, s12, th):
    from orb_slam_cuda_amd import _lib
    kf1, kf2, cam1, s, R, t = sim3_match_case(O, seed, s12=s12)
    m = pkg.ORBmatcher(0.75, True, max_kps=4096)
    sc = np.ascontiguousarray(kf1["scale"], np.float32)
    out = np.full(len(kf1["kps"]), -7, np.int32)
    nf = C.c_int(-1)
    cam = _cam(cam1)
    _lib.check(_lib.lib().orbm_search_by_sim3(
        m.handle, _v(kf1["kps"]), _v(kf1["desc"]), len(kf1["kps"]), _lib.GridBounds(*kf1["bounds"]), _v(kf1["Tcw"]),
        _v(kf1["mps"]), _v(kf1["mpdesc"]), _v(kf2["kps"]), _v(kf2["desc"]), len(kf2["kps"]),
        _lib.GridBounds(*kf2["bounds"]), _v(kf2["Tcw"]), _v(kf2["mps"]), _v(kf2["mpdesc"]), _v(sc), len(sc),
        C.c_float(1.2), C.byref(cam), C.c_float(s), _v(R), _v(t), C.c_float(th), _v(out), C.byref(nf)), matcher=True)
    e1, enf, _, _ = O.search_by_sim3(kf1, kf2, cam1, s, R, t, th)
    assert nf.value == enf and np.array_equal(out, e1)
    if s12 == 1.0:
        assert enf > 300


def _tri_call(pkg, m, kf1, kf2, cw1, T2w, cam2, sig2, F12, only_stereo, check_ori):
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.matcher import _fvc
    out = np.full(len(kf1["kps"]), -7, np.int32)
    nm = C.c_int(-1)
    sc2 = np.ascontiguousarray(kf2["scale"], np.float32)
    _lib.check(_lib.lib().orbm_search_for_triangulation(
        m.handle, _v(kf1["kps"]), _v(kf1["desc"]), _v(kf1["uright"]), _v(kf1["has_mp"]), len(kf1["kps"]),
        _fvc(kf1["fv"]), _v(kf2["kps"]), _v(kf2["desc"]), _v(kf2["uright"]), _v(kf2["has_mp"]), len(kf2["kps"]),
        _fvc(kf2["fv"]), _v(cw1), _v(T2w), _v(cam2), _v(sc2), _v(np.asarray(sig2, np.float32)), len(sc2), _v(F12),
        int(only_stereo), int(check_ori), _v(out), C.byref(nm)), matcher=True)
    return out, nm.value


@pytest.mark.parametrize("seed,only_stereo,check_ori", [(1, False, True), (2, True, True), (3, False, False),
                                                        (4, False, True)])
def test_search_for_triangulation_parity(pkg, O, seed, only_stereo, check_ori):
    kf1, kf2, cw1, T2w, cam2, sig2, F12 = triangulation_case(O, seed)
    m = pkg.ORBmatcher(0.6, check_ori, max_kps=4096)
    out, nm = _tri_call(pkg, m, kf1, kf2, cw1, T2w, cam2, sig2, F12, only_stereo, check_ori)
    e, enm = O.search_for_triangulation(kf1, kf2, cw1, T2w, cam2, sig2, F12, only_stereo, check_ori)
    assert nm == enm and np.array_equal(out, e)
    assert enm > (50 if only_stereo else 300)


def test_search_for_triangulation_empty(pkg, O):
    kf1, kf2, cw1, T2w, cam2, sig2, F12 = triangulation_case(O, 5)
    kf2 = dict(kf2, fv=(np.zeros(0, np.uint32), np.zeros(1, np.int32), np.zeros(0, np.int32)))
    m = pkg.ORBmatcher(0.6, True, max_kps=4096)
    out, nm = _tri_call(pkg, m, kf1, kf2, cw1, T2w, cam2, sig2, F12, False, True)
    assert nm == 0 and (out == -1).all()


def test_search_for_triangulation_batch_shared_kf1(pkg, O):
    """One new keyframe against 6 neighbours in one launch (kp_pitch1 = node_pitch1 = 0)."""
    from orb_slam_cuda_amd import _lib
    base = triangulation_case(O, 10)
    kf1 = base[0]
    P, K, NP = 6, 2400, 128
    cases = [base] + [triangulation_case(O, 10, stereo_frac=0.3 + 0.05 * i) for i in range(1, P)]
    # same KF1 keypoints in every case; the stereo masks differ with stereo_frac
    k2 = np.zeros((P, K), pkg.KP_DTYPE); d2 = np.zeros((P, K, 32), np.uint8); u2 = np.full((P, K), -1, np.float32)
    h2 = np.zeros((P, K), np.uint8); n2 = np.zeros(P, np.int32); nd2 = np.zeros((P, NP), np.uint32)
    of2 = np.zeros((P, NP + 1), np.int32); ix2 = np.zeros((P, K), np.int32); nn2 = np.zeros(P, np.int32)
    tp = (_lib.OrbmTriPair * P)()
    for p, (a, b, cw1, T2w, cam2, sig2, F12) in enumerate(cases):
        assert np.array_equal(a["kps"].view(np.uint8), kf1["kps"].view(np.uint8))
        n = len(b["kps"]); n2[p] = n
        k2[p, :n] = b["kps"]; d2[p, :n] = b["desc"]; u2[p, :n] = b["uright"]; h2[p, :n] = b["has_mp"]
        nodes, off, idx = b["fv"]
        nn2[p] = len(nodes); nd2[p, :len(nodes)] = nodes; of2[p, :len(off)] = off; ix2[p, :len(idx)] = idx
        _lib.check(_lib.lib().orbm_prepare_triangulation(_v(cw1), _v(T2w), _v(cam2), _v(F12), C.byref(tp[p])),
                   matcher=True)
    nodes1, off1, idx1 = kf1["fv"]
    host = dict(k1=kf1["kps"], d1=kf1["desc"], u1=kf1["uright"], h1=kf1["has_mp"],
                n1=np.array([len(kf1["kps"])], np.int32), nd1=nodes1, of1=off1, ix1=idx1,
                nn1=np.array([len(nodes1)], np.int32), k2=k2, d2=d2, u2=u2, h2=h2, n2=n2, nd2=nd2, of2=of2, ix2=ix2,
                nn2=nn2, tp=np.frombuffer(bytes(tp), np.uint8))
    dev = {}
    for name, a in host.items():
        dev[name] = _lib.DeviceArray(a.nbytes)
        dev[name].upload(np.ascontiguousarray(a))
    v = lambda k: C.c_void_p(dev[k].ptr)
    OUTP = 2048
    d_out, d_nm = _lib.DeviceArray(P * OUTP * 4), _lib.DeviceArray(4 * P)
    m = pkg.ORBmatcher(0.6, True, max_kps=4096)
    sc2 = np.ascontiguousarray(base[1]["scale"], np.float32)
    sg2 = np.ascontiguousarray(base[5], np.float32)
    s = _lib.Stream()
    _lib.check(_lib.lib().orbm_search_for_triangulation_batch(
        m.handle, v("k1"), v("d1"), v("u1"), v("h1"), v("n1"), v("nd1"), v("of1"), v("ix1"), v("nn1"), 0, 0,
        v("k2"), v("d2"), v("u2"), v("h2"), v("n2"), v("nd2"), v("of2"), v("ix2"), v("nn2"), K, NP, v("tp"),
        _v(sc2), _v(sg2), len(sc2), P, 0, 1, C.c_void_p(d_out.ptr), OUTP, C.c_void_p(d_nm.ptr), s.s), matcher=True)
    s.synchronize()
    out = d_out.download(P * OUTP, np.int32).reshape(P, OUTP)
    nm = d_nm.download(P, np.int32)
    n1 = len(kf1["kps"])
    for p, (a, b, cw1, T2w, cam2, sig2, F12) in enumerate(cases):
        e, enm = O.search_for_triangulation(kf1, b, cw1, T2w, cam2, sig2, F12, False, True)  # the shared KF1
        assert nm[p] == enm and np.array_equal(out[p, :n1], e)


def test_mirror_fuse_and_triangulation(pkg, O):
    """The Python mirror (KeyFrame / MapPoints, reference signatures) on the same data."""
    c = fuse_case(O, 11, nmp=2500)
    mp = c["mps"]
    table = pkg.MapPoints(pos=mp["pos"], descriptors=c["mpdesc"], normal=mp["normal"], min_distance=mp["min_distance"],
                          max_distance=mp["max_distance"], bad=~mp["valid"].astype(bool))
    cam = c["cam"]
    n = len(c["kps"])
    kf = pkg.KeyFrame(c["kps"], c["desc"], np.full(n, -1, np.int64), mnMinX=0.0, mnMaxX=1241.0, mnMinY=0.0,
                      mnMaxY=376.0, fx=cam.fx, fy=cam.fy, cx=cam.cx, cy=cam.cy,
                      mvScaleFactors=np.ascontiguousarray(c["scale"], np.float32), mpMap=table,
                      mTcw=np.array(list(cam.Tcw), np.float32).reshape(3, 4), mvuRight=c["uright"], mbf=cam.mbf,
                      mvInvLevelSigma2=np.ascontiguousarray(c["inv_sigma2"], np.float32))
    m = pkg.ORBmatcher(0.6, True, max_kps=4096)
    nf = m.Fuse(kf, np.arange(2500), 3.0)
    eout, enf = O.fuse(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"], c["inv_sigma2"], 1.2, cam, mp,
                       c["mpdesc"], 3.0)
    assert nf == enf and np.array_equal(m.last_fuse, eout)
    # first point to reach an empty keypoint is added there; later ones become replacements
    first = {}
    for i in np.nonzero(eout >= 0)[0]:
        first.setdefault(int(eout[i]), int(i))
    for idx, i in first.items():
        assert kf.mvpMapPoints[idx] == i
    kf1, kf2, cw1, T2w, cam2, sig2, F12 = triangulation_case(O, 12)

    def mk(k, T):
        nodes, off, idx = k["fv"]
        fv = {int(nd): idx[off[j]:off[j + 1]].tolist() for j, nd in enumerate(nodes)}
        return pkg.KeyFrame(k["kps"], k["desc"], np.where(k["has_mp"] == 1, 0, -1), fv, fx=cam2[0], fy=cam2[1],
                            cx=cam2[2], cy=cam2[3], mvScaleFactors=np.ascontiguousarray(kf2["scale"], np.float32),
                            mTcw=T, mvuRight=k["uright"], mvLevelSigma2=np.ascontiguousarray(sig2, np.float32))
    T1 = np.eye(4, dtype=np.float32)[:3].copy()
    T1[:, 3] = -cw1  # identity rotation with camera centre cw1
    K1, K2 = mk(kf1, T1), mk(kf2, T2w)
    pairs = []
    nm = m.SearchForTriangulation(K1, K2, F12, pairs, False)
    e, enm = O.search_for_triangulation(kf1, kf2, K1.GetCameraCenter(), T2w, cam2, sig2, F12, False, True)
    assert nm == enm and pairs == [(int(i), int(j)) for i, j in enumerate(e) if j >= 0]
