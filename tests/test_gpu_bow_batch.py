"""Batched, device-resident SearchByBoW (orbm_search_by_bow_batch) against the
oracle: 2000-keypoint KITTI frames extracted in one batch, their
FeatureVectors from orbv_transform_batch (ComputeBoW, levelsup 4) on the
device, then KF-F (Tracking::TrackReferenceKeyFrame, ratio 0.7) and KF-KF
(ratio 0.75) matching of consecutive frames, one launch for all pairs."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[(10, 6), (16, 5), (10, 5), (4, 5), (2, 4)],
                ids=["k10L6", "k16L5", "k10L5", "k4L5", "k2L4"])
def voc(pkg, request):
    """k10 L6: ~100 FeatureVector nodes of ~20 features (the two-pass path);
    k16 L5 / k10 L5: 16 nodes of ~125 / 10 of ~200 (a row's candidates split
    over 4 / 8 lanes, long greedy chains, rescans by whole waves); k4 L5: 4
    nodes of ~500 (over a range's 256 rows: the per-wave fallback); k2 L4: the
    root only, one node of ~2000 (candidates streamed from global memory)."""
    from orb_slam_cuda_amd.synth import synthetic_vocabulary
    k, L = request.param
    v = synthetic_vocabulary(k, L, seed=1)
    return v, pkg.ORBVocabulary.from_arrays(v)


def _extract_and_bow(pkg, v, frames):
    from orb_slam_cuda_amd import _lib
    B, H, W = frames.shape
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=B)
    cap = ext.frame_capacity
    d_in = _lib.DeviceArray(frames.nbytes)
    d_in.upload(np.ascontiguousarray(frames))
    D = dict(kp=_lib.DeviceArray(B * cap * 28), desc=_lib.DeviceArray(B * cap * 32), n=_lib.DeviceArray(4 * B),
             bw=_lib.DeviceArray(B * cap * 4), bv=_lib.DeviceArray(B * cap * 8), bn=_lib.DeviceArray(4 * B),
             fn=_lib.DeviceArray(B * cap * 4), fo=_lib.DeviceArray(B * (cap + 1) * 4), fi=_lib.DeviceArray(B * cap * 4),
             fnn=_lib.DeviceArray(4 * B))
    s = _lib.Stream()
    ext.extract_batch_device(d_in.ptr, B, H * W, W, D["kp"].ptr, D["desc"].ptr, D["n"].ptr, s)
    vp = C.c_void_p
    _lib.check(_lib.lib().orbv_transform_batch(
        v.handle, vp(D["desc"].ptr), cap * 32, vp(D["n"].ptr), B, cap, 4, vp(D["bw"].ptr), vp(D["bv"].ptr),
        vp(D["bn"].ptr), vp(D["fn"].ptr), vp(D["fo"].ptr), vp(D["fi"].ptr), vp(D["fnn"].ptr), None, None, None, s.s),
        vocabulary=True)
    s.synchronize()
    host = dict(n=D["n"].download(B, np.int32), kp=D["kp"].download(B * cap, pkg.KP_DTYPE).reshape(B, cap),
                desc=D["desc"].download((B, cap, 32), np.uint8),
                fn=D["fn"].download(B * cap, np.uint32).reshape(B, cap),
                fo=D["fo"].download(B * (cap + 1), np.int32).reshape(B, cap + 1),
                fi=D["fi"].download(B * cap, np.int32).reshape(B, cap), fnn=D["fnn"].download(B, np.int32))
    return ext, cap, D, host, s


@pytest.mark.parametrize("kf_vs_kf,ratio,ori,rounds", [(0, 0.7, 1, None), (1, 0.75, 1, None), (0, 0.75, 0, None),
                                                      (0, 0.7, 1, "0"), (1, 0.75, 1, "1")])
def test_search_by_bow_batch_parity(pkg, O, voc, kf_vs_kf, ratio, ori, rounds, monkeypatch):
    """ORBX_BOW_ROUNDS=0 / 1: the greedy resolved by the wave-per-node
    sequential pass (after 0 / 1 fixed-point rounds), the same answers."""
    if rounds is not None:
        monkeypatch.setenv("ORBX_BOW_ROUNDS", rounds)
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    v, V = voc
    P = 6
    frames = SynthSequence(31, 1241, 376).frames(P + 1)
    ext, cap, D, h, s = _extract_and_bow(pkg, V, frames)
    rng = np.random.default_rng(7 + kf_vs_kf)
    mp = (rng.random((P + 1, cap)) > 0.25).astype(np.uint8)  # KF features with a good MapPoint
    d_mp = _lib.DeviceArray(mp.nbytes)
    d_mp.upload(mp)
    m = pkg.ORBmatcher(ratio, bool(ori), max_pairs=P, max_kps=cap)
    d_out, d_nm = _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * 4)
    off = lambda arr, k, pitch, size: C.c_void_p(arr.ptr + k * pitch * size)
    args = []
    for side in (0, 1):  # A = frames 0..P-1, B = frames 1..P
        args += [off(D["kp"], side, cap, 28), off(D["desc"], side, cap, 32), off(D["n"], side, 1, 4),
                 off(d_mp, side, cap, 1) if (side == 0 or kf_vs_kf) else None,
                 off(D["fn"], side, cap, 4), off(D["fo"], side, cap + 1, 4), off(D["fi"], side, cap, 4),
                 off(D["fnn"], side, 1, 4)]
    _lib.check(_lib.lib().orbm_search_by_bow_batch(m.handle, P, cap, cap, *args, C.c_float(ratio), ori, kf_vs_kf,
                                                   C.c_void_p(d_out.ptr), C.c_void_p(d_nm.ptr), s.s), matcher=True)
    s.synchronize()
    out = d_out.download(P * cap, np.int32).reshape(P, cap)
    nm = d_nm.download(P, np.int32)
    assert m.status() == 0
    for p in range(P):
        a, b = p, p + 1
        na, nb = h["n"][a], h["n"][b]
        csr = lambda f: (h["fn"][f, :h["fnn"][f]], h["fo"][f, :h["fnn"][f] + 1], h["fi"][f, :h["fo"][f, h["fnn"][f]]])
        rout, rnm = O.search_by_bow(h["desc"][a, :na], h["kp"][a, :na]["angle"], mp[a, :na], csr(a),
                                    h["desc"][b, :nb], h["kp"][b, :nb]["angle"],
                                    mp[b, :nb] if kf_vs_kf else np.ones(nb, np.uint8), csr(b), ratio, ori, kf_vs_kf)
        nout = na if kf_vs_kf else nb
        assert nm[p] == rnm and np.array_equal(out[p, :nout], rout), p
        assert rnm > 20


def test_search_by_bow_batch_reuse(pkg, O, voc):
    """One matcher over calls of growing size: the row-record scratch the
    finalize kernel restores must be clean for pairs a previous call never
    touched (2 pairs, then 6 twice)."""
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    v, V = voc
    P = 6
    frames = SynthSequence(32, 1241, 376).frames(P + 1)
    ext, cap, D, h, s = _extract_and_bow(pkg, V, frames)
    mp = np.ones((P + 1, cap), np.uint8)
    d_mp = _lib.DeviceArray(mp.nbytes)
    d_mp.upload(mp)
    m = pkg.ORBmatcher(0.7, True, max_pairs=P, max_kps=cap)
    off = lambda arr, k, pitch, size: C.c_void_p(arr.ptr + k * pitch * size)
    args = []
    for side in (0, 1):
        args += [off(D["kp"], side, cap, 28), off(D["desc"], side, cap, 32), off(D["n"], side, 1, 4),
                 off(d_mp, side, cap, 1) if side == 0 else None,
                 off(D["fn"], side, cap, 4), off(D["fo"], side, cap + 1, 4), off(D["fi"], side, cap, 4),
                 off(D["fnn"], side, 1, 4)]
    csr = lambda f: (h["fn"][f, :h["fnn"][f]], h["fo"][f, :h["fnn"][f] + 1], h["fi"][f, :h["fo"][f, h["fnn"][f]]])
    ref = [O.search_by_bow(h["desc"][p, :h["n"][p]], h["kp"][p, :h["n"][p]]["angle"], mp[p, :h["n"][p]], csr(p),
                           h["desc"][p + 1, :h["n"][p + 1]], h["kp"][p + 1, :h["n"][p + 1]]["angle"],
                           np.ones(h["n"][p + 1], np.uint8), csr(p + 1), 0.7, 1, 0) for p in range(P)]
    for pairs in (2, P, P):
        d_out, d_nm = _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * 4)
        _lib.check(_lib.lib().orbm_search_by_bow_batch(m.handle, pairs, cap, cap, *args, C.c_float(0.7), 1, 0,
                                                       C.c_void_p(d_out.ptr), C.c_void_p(d_nm.ptr), s.s),
                   matcher=True)
        s.synchronize()
        out = d_out.download(P * cap, np.int32).reshape(P, cap)
        nm = d_nm.download(P, np.int32)
        assert m.status() == 0
        for p in range(pairs):
            rout, rnm = ref[p]
            nb = h["n"][p + 1]
            assert nm[p] == rnm and np.array_equal(out[p, :nb], rout), (pairs, p)
            assert (out[p, nb:] == -1).all()
