"""GPU parity of ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)
(liborbx.so, orbx_project.hip) against the CPU oracle (itself cross-checked
against tests/refpy.py). The keypoint -> map point assignment and the match
count must be identical, including the sequential blocking among map points."""
import ctypes as C
import os

import numpy as np
import pytest

from projcase import projection_case

pytestmark = pytest.mark.gpu


def _frame(pkg, kps, desc, ur, bounds, scale):
    F = pkg.Frame(kps, desc, *bounds)
    F.mvuRight = ur
    F.mvScaleFactors = np.asarray(scale, np.float32)
    return F


@pytest.mark.parametrize("seed,th,ratio,stereo,nmp", [(1, 1.0, 0.8, False, 3000), (2, 3.0, 0.9, True, 3000),
                                                      (3, 1.5, 0.6, False, 6000), (4, 5.0, 0.75, True, 8192),
                                                      (5, 1.0, 1.0, False, 0)])
def test_search_by_projection_parity(pkg, O, seed, th, ratio, stereo, nmp):
    kps, desc, ur, bounds, scale, blocked, mps, mpd = projection_case(O, seed, nmp=nmp, stereo=stereo)
    m = pkg.ORBmatcher(ratio, True, max_kps=4096)
    F = _frame(pkg, kps, desc, ur, bounds, scale)
    nm = m.SearchByProjection(F, mps, mpd, th, blocked=blocked)
    eout, enm = O.search_by_projection(kps, desc, ur, bounds, scale, blocked, mps, mpd, th, ratio)
    assert nm == enm and np.array_equal(m.last_projection, eout)
    if nmp:
        assert nm > 300


def test_search_by_projection_sequential_fallback(pkg, O, monkeypatch):
    """One fixed-point round only: the in-kernel sequential pass must give the same result."""
    kps, desc, ur, bounds, scale, blocked, mps, mpd = projection_case(O, 7, nmp=4000, stereo=True)
    monkeypatch.setenv("ORBX_PROJ_ROUNDS", "1")
    m = pkg.ORBmatcher(0.8, True, max_kps=4096)
    nm = m.SearchByProjection(_frame(pkg, kps, desc, ur, bounds, scale), mps, mpd, 3.0, blocked=blocked)
    eout, enm = O.search_by_projection(kps, desc, ur, bounds, scale, blocked, mps, mpd, 3.0, 0.8)
    assert nm == enm and np.array_equal(m.last_projection, eout)


def test_search_by_projection_batch(pkg, O):
    from orb_slam_cuda_amd import _lib
    B, K, M = 4, 2100, 5000
    cases = [projection_case(O, 20 + i, nmp=3000 + 500 * i, stereo=bool(i % 2)) for i in range(B)]
    kp = np.zeros((B, K), pkg.KP_DTYPE); ds = np.zeros((B, K, 32), np.uint8); ur = np.full((B, K), -1, np.float32)
    bl = np.zeros((B, K), np.uint8); mp = np.zeros((B, M), _lib.MAP_POINT_PROJ_DTYPE); md = np.zeros((B, M, 32), np.uint8)
    n = np.zeros(B, np.int32); nmp = np.zeros(B, np.int32)
    for i, (k, d, u, bounds, scale, b, p, q) in enumerate(cases):
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
    sc = np.ascontiguousarray(cases[0][4], np.float32)
    s = _lib.Stream()
    v = lambda a: C.c_void_p(a.ptr)
    _lib.check(_lib.lib().orbm_search_by_projection_batch(
        m.handle, v(dev["kp"]), v(dev["ds"]), v(dev["n"]), K, v(dev["ur"]), _lib.GridBounds(*cases[0][3]),
        sc.ctypes.data_as(C.c_void_p), len(sc), v(dev["bl"]), v(dev["mp"]), v(dev["md"]), v(dev["nmp"]), M, B,
        C.c_float(3.0), C.c_float(0.8), v(d_out), v(d_nm), s.s), matcher=True)
    s.synchronize()
    out = d_out.download(B * K, np.int32).reshape(B, K)
    nm = d_nm.download(B, np.int32)
    for i, (k, d, u, bounds, scale, b, p, q) in enumerate(cases):
        # the batch passes every frame a uRight array: -1 entries behave as mono keypoints
        uu = u if u is not None else np.full(len(k), -1, np.float32)
        eout, enm = O.search_by_projection(k, d, uu, bounds, scale, b, p, q, 3.0, 0.8)
        assert nm[i] == enm and np.array_equal(out[i, :n[i]], eout)
