"""Scenes for the C++ shim host's --scene mode (shim/host/scene.cc): the
Frame / KeyFrame / MapPoint state one ORBmatcher call sees, built from the
same synthetic cases the C-ABI parity tests use (posecase.py, projcase.py),
written as [u32 name length][name][u32 dtype 0 u8 / 1 i32 / 2 f32][u32 count]
[elements] records. Each builder returns (records, expected result) with the
expectation computed by the oracle and translated into the pointer state the
reference's method leaves (MapPoints as pool indices, -1 = NULL)."""
import numpy as np

from posecase import CX, CY, FX, FY, MB, fuse_case, keyframe_case, last_frame_case, sim3_case, sim3_match_case, \
    triangulation_case
from projcase import projection_case

OPS = dict(local_map=1, last_frame=2, keyframe=3, sim3=4, fuse=5, fuse_sim3=6, sim3_match=7, triangulation=8,
           bow=9)

# the oracle call of the last scene built, as a zero-argument callable
# (bench.py times the single-thread CPU restatement on the scene's own inputs)
LAST_CPU = [None]


def _cpu(fn):
    LAST_CPU[0] = fn
    return fn()


def write_scene(path, recs):
    with open(path, "wb") as f:
        for name, a in recs.items():
            a = np.asarray(a)
            if a.dtype == np.uint8 or a.dtype == np.bool_:
                dt, a = 0, a.astype(np.uint8)
            elif a.dtype.kind in "iu":
                dt, a = 1, a.astype(np.int32)
            elif a.dtype.kind == "f":
                dt, a = 2, a.astype(np.float32)
            else:  # structured keypoints: raw bytes
                dt, a = 0, np.ascontiguousarray(a).view(np.uint8)
            a = np.ascontiguousarray(a).reshape(-1)
            nb = name.encode()
            f.write(np.uint32(len(nb)).tobytes() + nb + np.uint32(dt).tobytes() + np.uint32(a.size).tobytes())
            f.write(a.tobytes())


def _cam(fx=FX, fy=FY, cx=CX, cy=CY, mb=MB, mbf=MB * FX):
    return np.array([fx, fy, cx, cy, mb, mbf], np.float32)


def _side(X, kps, desc, bounds, scale, T=None, uright=None, mps=None, cam=None, **extra):
    r = {f"{X}_kps": kps, f"{X}_desc": np.ascontiguousarray(desc, np.uint8), f"{X}_bounds": np.float32(bounds),
         f"{X}_scale": np.float32(scale), f"{X}_sf": np.float32([1.2]), f"{X}_cam": _cam() if cam is None else cam}
    if T is not None:
        r[f"{X}_T"] = np.float32(T).reshape(-1)
    if uright is not None:
        r[f"{X}_uright"] = np.float32(uright)
    if mps is not None:
        r[f"{X}_mps"] = np.int32(mps)
    for k, v in extra.items():
        r[f"{X}_{k}"] = v
    return r


def local_map(O, seed, th=3.0, ratio=0.8, stereo=True, nmp=3000):
    """SearchByProjection(F, vpMapPoints, th): Frame::isInFrustum fields per point."""
    kps, desc, ur, bounds, scale, blocked, mps, mpd = projection_case(O, seed, nmp=nmp, stereo=stereo)
    M, n = len(mps), len(kps)
    holder = M  # an extra point with observations holds the blocked keypoints
    track = np.stack([mps["proj_x"], mps["proj_y"], mps["proj_xr"], mps["view_cos"]], 1)
    recs = dict(op=np.int32([OPS["local_map"]]), th=np.float32([th]), nnratio=np.float32([ratio]),
                mp_desc=np.concatenate([mpd, np.zeros((1, 32), np.uint8)]),
                mp_track=np.concatenate([track, np.zeros((1, 4))]).astype(np.float32),
                mp_level=np.concatenate([mps["predicted_level"], [0]]).astype(np.int32),
                mp_inview=np.concatenate([mps["track_in_view"], [0]]).astype(np.uint8),
                mp_nobs=np.concatenate([mps["obs_positive"].astype(np.int32), [1]]).astype(np.int32),
                vp=np.arange(M, dtype=np.int32))
    cur = np.where(blocked == 1, holder, -1).astype(np.int32)
    recs.update(_side("A", kps, desc, bounds, scale, uright=ur, mps=cur))
    eout, enm = _cpu(lambda: O.search_by_projection(kps, desc, ur, bounds, scale, blocked, mps, mpd, th, ratio))
    want = cur.copy()
    want[eout >= 0] = eout[eout >= 0]
    return recs, np.concatenate([[enm], want]).astype(np.int32)


def last_frame(O, seed, th=7.0, stereo=True, motion="forward"):
    """SearchByProjection(CurrentFrame, LastFrame, th, bMono): LastFrame keypoint i holds point i."""
    c = last_frame_case(O, seed, stereo=stereo, motion=motion)
    mps = c["mps"]
    M = len(mps)
    lk = np.zeros(M, O.KP_DTYPE)
    lk["angle"], lk["octave"] = mps["angle"], mps["octave"]
    holder = int(np.nonzero(mps["obs_positive"])[0][0])
    cur = np.where(c["blocked"] == 1, holder, -1).astype(np.int32)
    cam = c["cam"]
    recs = dict(op=np.int32([OPS["last_frame"]]), th=np.float32([th]), mono=np.int32([int(c["mono"])]),
                nnratio=np.float32([0.9]), mp_desc=c["mpdesc"], mp_pos=mps["pos"],
                mp_nobs=mps["obs_positive"].astype(np.int32))
    recs.update(_side("B", lk, np.zeros((M, 32), np.uint8), c["bounds"], c["scale"], T=c["Tlw"],
                      mps=np.arange(M), outlier=(~mps["valid"].astype(bool)).astype(np.uint8)))
    recs.update(_side("A", c["kps"], c["desc"], c["bounds"], c["scale"], T=np.float32(list(cam.Tcw)),
                      uright=c["uright"], mps=cur, cam=_cam(cam.fx, cam.fy, cam.cx, cam.cy, cam.mb, cam.mbf)))
    eout, enm = _cpu(lambda: O.search_by_projection_last_frame(c["kps"], c["desc"], c["uright"], c["bounds"],
                                                               c["scale"], c["blocked"], c["cam"], c["Tlw"], mps,
                                                               c["mpdesc"], th, c["mono"]))
    want = cur.copy()
    want[eout >= 0] = eout[eout >= 0]
    want[eout == -2] = -1
    return recs, np.concatenate([[enm], want]).astype(np.int32)


def keyframe(O, seed, th=10.0, orb_dist=100):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist): the keyframe's keypoint i holds
    point i; the points the case marks invalid are bad (even ones) or already found (odd ones)."""
    c = keyframe_case(O, seed)
    mps = c["mps"]
    M = len(mps)
    inval = np.nonzero(~mps["valid"].astype(bool))[0]
    bad = np.zeros(M, np.uint8)
    bad[inval[0::2]] = 1
    kk = np.zeros(M, O.KP_DTYPE)
    kk["angle"] = mps["angle"]
    cur = np.where(c["has_mp"] == 1, M, -1).astype(np.int32)  # an extra point fills CurrentFrame's own slots
    cam = c["cam"]
    recs = dict(op=np.int32([OPS["keyframe"]]), th=np.float32([th]), orb_dist=np.int32([orb_dist]),
                nnratio=np.float32([0.75]), mp_desc=np.concatenate([c["mpdesc"], np.zeros((1, 32), np.uint8)]),
                mp_pos=np.concatenate([mps["pos"], np.zeros((1, 3), np.float32)]),
                mp_dist=np.concatenate([np.stack([mps["min_distance"], mps["max_distance"]], 1),
                                        np.ones((1, 2), np.float32)]).astype(np.float32),
                mp_bad=np.concatenate([bad, [0]]).astype(np.uint8),
                mp_nobs=np.ones(M + 1, np.int32), already=np.int32(inval[1::2]))
    recs.update(_side("B", kk, np.zeros((M, 32), np.uint8), c["bounds"], c["scale"], mps=np.arange(M)))
    recs.update(_side("A", c["kps"], c["desc"], c["bounds"], c["scale"], T=np.float32(list(cam.Tcw)), mps=cur,
                      cam=_cam(cam.fx, cam.fy, cam.cx, cam.cy, cam.mb, cam.mbf)))
    eout, enm = O.search_by_projection_keyframe(c["kps"], c["desc"], c["bounds"], c["scale"], 1.2, c["has_mp"],
                                                c["cam"], mps, c["mpdesc"], th, orb_dist)
    want = cur.copy()
    want[eout >= 0] = eout[eout >= 0]
    want[eout == -2] = -1
    return recs, np.concatenate([[enm], want]).astype(np.int32)


def sim3(O, seed, th=10, s=1.3):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th): vpMatched holds extra points where the case
    marks a keypoint matched."""
    c = sim3_case(O, seed, s=s)
    mps = c["mps"]
    M, n = len(mps), len(c["kps"])
    setm = c["matched"] >= 0
    matched = np.where(setm, M + np.arange(n), -1).astype(np.int32)
    cam = c["cam"]
    z = lambda k, w: np.zeros((n, w), np.float32) if w > 1 else np.zeros(n, np.float32)
    recs = dict(op=np.int32([OPS["sim3"]]), thi=np.int32([th]),
                mp_desc=np.concatenate([c["mpdesc"], np.zeros((n, 32), np.uint8)]),
                mp_pos=np.concatenate([mps["pos"], z(0, 3)]), mp_normal=np.concatenate([mps["normal"], z(0, 3)]),
                mp_dist=np.concatenate([np.stack([mps["min_distance"], mps["max_distance"]], 1), z(0, 2)]),
                mp_bad=np.concatenate([~mps["valid"].astype(bool), np.zeros(n, bool)]).astype(np.uint8),
                mp_nobs=np.ones(M + n, np.int32), vp=np.arange(M, dtype=np.int32), matched=matched,
                Scw=np.float32(list(cam.Tcw)))
    recs.update(_side("A", c["kps"], c["desc"], c["bounds"], c["scale"],
                      cam=_cam(cam.fx, cam.fy, cam.cx, cam.cy, 0.0, 0.0)))
    eout, enm = O.search_by_projection_sim3(c["kps"], c["desc"], c["bounds"], c["scale"], 1.2, c["cam"], mps,
                                            c["mpdesc"], th, c["matched"])
    want = matched.copy()
    want[eout >= 0] = eout[eout >= 0]
    return recs, np.concatenate([[enm], want]).astype(np.int32)


def _fuse_holders(rng, n, M, frac=0.15):
    """Keypoints of the keyframe that already hold a MapPoint: extra points M, M+1, ... with 1..4 observations."""
    held = np.nonzero(rng.random(n) < frac)[0]
    kmp = np.full(n, -1, np.int32)
    kmp[held] = M + np.arange(len(held))
    return kmp, rng.integers(1, 5, len(held)).astype(np.int32)


def fuse(O, seed, th=3.0):
    """Fuse(pKF, vpMapPoints, th): candidates 0..M-1 (bad where the case marks them invalid), keypoints holding
    extra points; expected state from the oracle's per-point matches and the reference's in-order tail
    (src/ORBmatcher.cc:951-971; MapPoint::Replace / AddObservation / ComputeDistinctiveDescriptors)."""
    c = fuse_case(O, seed, stereo=True)
    mps = c["mps"]
    M, n = len(mps), len(c["kps"])
    rng = np.random.default_rng(700 + seed)
    kmp, hobs = _fuse_holders(rng, n, M)
    H = len(hobs)
    nobs = np.concatenate([rng.integers(0, 4, M), hobs]).astype(np.int32)
    bad = np.concatenate([~mps["valid"].astype(bool), np.zeros(H, bool)])
    cam = c["cam"]
    zeros = lambda w: np.zeros((H, w), np.float32)
    recs = dict(op=np.int32([OPS["fuse"]]), th=np.float32([th]),
                mp_desc=np.concatenate([c["mpdesc"], np.zeros((H, 32), np.uint8)]),
                mp_pos=np.concatenate([mps["pos"], zeros(3)]), mp_normal=np.concatenate([mps["normal"], zeros(3)]),
                mp_dist=np.concatenate([np.stack([mps["min_distance"], mps["max_distance"]], 1), zeros(2)]),
                mp_bad=bad.astype(np.uint8), mp_nobs=nobs, vp=np.arange(M, dtype=np.int32))
    recs.update(_side("A", c["kps"], c["desc"], c["bounds"], c["scale"], T=np.float32(list(cam.Tcw)),
                      uright=c["uright"], mps=kmp, invsigma2=np.float32(c["inv_sigma2"]),
                      cam=_cam(cam.fx, cam.fy, cam.cx, cam.cy, cam.mb, cam.mbf)))
    eout, _ = _cpu(lambda: O.fuse(c["kps"], c["desc"], c["uright"], c["bounds"], c["scale"], c["inv_sigma2"], 1.2,
                                  cam, mps, c["mpdesc"], th))
    # the reference's tail on a model of the map: observations in this keyframe only
    kmp_now = kmp.copy()
    bad_now = bad.copy()
    nobs_now = nobs.copy()
    in_kf = np.zeros(M + H, bool)
    in_kf[M:] = True
    obs_idx = np.full(M + H, -1)
    obs_idx[kmp[kmp >= 0]] = np.nonzero(kmp >= 0)[0]
    ur = c["uright"]
    weight = lambda idx: 2 if ur[idx] >= 0 else 1
    nf = 0
    for i in range(M):
        if eout[i] < 0 or bad_now[i] or in_kf[i]:
            continue
        idx = int(eout[i])
        q = int(kmp_now[idx])
        if q >= 0:
            if not bad_now[q]:
                if nobs_now[q] > nobs_now[i]:      # pMP->Replace(pMPinKF): pMP has no observation to move
                    bad_now[i] = True
                else:                              # pMPinKF->Replace(pMP): its keypoint moves to pMP
                    bad_now[q] = True
                    in_kf[q] = False
                    kmp_now[idx] = i
                    in_kf[i] = True
                    nobs_now[i] += weight(idx)
        else:                                      # AddObservation + AddMapPoint
            kmp_now[idx] = i
            in_kf[i] = True
            nobs_now[i] += weight(idx)
        nf += 1
    return recs, np.concatenate([[nf], kmp_now, bad_now.astype(np.int32), nobs_now]).astype(np.int32)


def fuse_sim3(O, seed, th=4.0, s=1.1):
    """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)."""
    c = sim3_case(O, seed, s=s)
    mps = c["mps"]
    M, n = len(mps), len(c["kps"])
    rng = np.random.default_rng(800 + seed)
    kmp, hobs = _fuse_holders(rng, n, M)
    H = len(hobs)
    bad_h = rng.random(H) < 0.2  # some held points are bad: no replacement recorded for them
    cam = c["cam"]
    zeros = lambda w: np.zeros((H, w), np.float32)
    recs = dict(op=np.int32([OPS["fuse_sim3"]]), th=np.float32([th]),
                mp_desc=np.concatenate([c["mpdesc"], np.zeros((H, 32), np.uint8)]),
                mp_pos=np.concatenate([mps["pos"], zeros(3)]), mp_normal=np.concatenate([mps["normal"], zeros(3)]),
                mp_dist=np.concatenate([np.stack([mps["min_distance"], mps["max_distance"]], 1), zeros(2)]),
                mp_bad=np.concatenate([~mps["valid"].astype(bool), bad_h]).astype(np.uint8),
                mp_nobs=np.ones(M + H, np.int32), vp=np.arange(M, dtype=np.int32), Scw=np.float32(list(cam.Tcw)))
    recs.update(_side("A", c["kps"], c["desc"], c["bounds"], c["scale"], mps=kmp,
                      cam=_cam(cam.fx, cam.fy, cam.cx, cam.cy, 0.0, 0.0)))
    eout, _ = O.fuse_sim3(c["kps"], c["desc"], c["bounds"], c["scale"], 1.2, cam, mps, c["mpdesc"], th)
    kmp_now = kmp.copy()
    rep = np.full(M, -1, np.int32)
    bad = np.concatenate([~mps["valid"].astype(bool), bad_h])
    nf = 0
    for i in range(M):
        if eout[i] < 0:
            continue
        idx = int(eout[i])
        q = int(kmp_now[idx])
        if q >= 0:
            if not bad[q]:
                rep[i] = q
        else:
            kmp_now[idx] = i
        nf += 1
    return recs, np.concatenate([[nf], kmp_now, rep]).astype(np.int32)


def sim3_match(O, seed, th=7.5, s12=1.0):
    """SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th): KF1 keypoint i holds point i, KF2 keypoint j
    holds point n1 + j; invalid records are bad points."""
    kf1, kf2, cam1, s, R, t = sim3_match_case(O, seed, s12=s12)
    n1, n2 = len(kf1["kps"]), len(kf2["kps"])
    m1, m2 = kf1["mps"], kf2["mps"]
    cat = lambda f: np.concatenate([m1[f], m2[f]])
    recs = dict(op=np.int32([OPS["sim3_match"]]), th=np.float32([th]), s12=np.float32([s]), R12=np.float32(R),
                t12=np.float32(t), mp_desc=np.concatenate([kf1["mpdesc"], kf2["mpdesc"]]), mp_pos=cat("pos"),
                mp_dist=np.stack([cat("min_distance"), cat("max_distance")], 1).astype(np.float32),
                mp_bad=(~cat("valid").astype(bool)).astype(np.uint8), mp_nobs=np.ones(n1 + n2, np.int32),
                matched=np.full(n1, -1, np.int32))
    cam = _cam(cam1.fx, cam1.fy, cam1.cx, cam1.cy, 0.0, 0.0)
    recs.update(_side("A", kf1["kps"], kf1["desc"], kf1["bounds"], kf1["scale"], T=kf1["Tcw"], mps=np.arange(n1),
                      cam=cam))
    recs.update(_side("B", kf2["kps"], kf2["desc"], kf2["bounds"], kf2["scale"], T=kf2["Tcw"],
                      mps=n1 + np.arange(n2), cam=cam))
    e1, enf, _, _ = O.search_by_sim3(kf1, kf2, cam1, s, R, t, th)
    want = np.where(e1 >= 0, n1 + e1, -1)
    return recs, np.concatenate([[enf], want]).astype(np.int32)


def triangulation(O, seed, only_stereo=False):
    """SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo); pKF1's pose [I | -cw1] puts its
    camera centre at the case's cw1."""
    kf1, kf2, cw1, T2w, cam2, sig2, F12 = triangulation_case(O, seed)
    n1, n2 = len(kf1["kps"]), len(kf2["kps"])
    T1 = np.eye(4, dtype=np.float32)[:3].copy()
    T1[:, 3] = -cw1
    cam = _cam(*cam2, 0.0, 0.0)
    held = lambda k: np.where(k["has_mp"] == 1, 0, -1).astype(np.int32)
    fv = lambda k: dict(fv_nodes=np.int32(k["fv"][0]), fv_off=np.int32(k["fv"][1]), fv_idx=np.int32(k["fv"][2]))
    recs = dict(op=np.int32([OPS["triangulation"]]), only_stereo=np.int32([int(only_stereo)]),
                F12=np.float32(F12), mp_desc=np.zeros((1, 32), np.uint8), mp_nobs=np.ones(1, np.int32))
    recs.update(_side("A", kf1["kps"], kf1["desc"], (0.0, 1241.0, 0.0, 376.0), kf2["scale"], T=T1,
                      uright=kf1["uright"], mps=held(kf1), cam=cam, **fv(kf1)))
    recs.update(_side("B", kf2["kps"], kf2["desc"], (0.0, 1241.0, 0.0, 376.0), kf2["scale"], T=T2w,
                      uright=kf2["uright"], mps=held(kf2), cam=cam, sigma2=np.float32(sig2), **fv(kf2)))
    e, enm = _cpu(lambda: O.search_for_triangulation(kf1, kf2, cw1, T2w, cam2, sig2, F12, only_stereo, True))
    pairs = [(i, int(j)) for i, j in enumerate(e) if j >= 0]
    return recs, np.array([enm] + [v for p in pairs for v in p], np.int32)


def _featvec_csr(desc, seed, nodes=100):
    """A stand-in DBoW2 FeatureVector at the reference's level (Frame::ComputeBoW
    levelsup 4 on the 10^6-word vocabulary: ~100 nodes): node = a hash of 7
    descriptor bits, so near descriptors tend to share a node."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(256)[:7]
    bits = np.unpackbits(np.ascontiguousarray(desc, np.uint8), axis=1)[:, perm]
    node = (bits * (1 << np.arange(7))).sum(1) % nodes
    ids = np.unique(node)
    off = np.zeros(len(ids) + 1, np.int32)
    idx = []
    for k, v in enumerate(ids):
        idx += np.nonzero(node == v)[0].tolist()
        off[k + 1] = len(idx)
    return (ids * 11 + 5).astype(np.int32), off, np.array(idx, np.int32)


def bow(O, seed, ratio=0.7, W=1241, H=376, nf=2000):
    """SearchByBoW(pKF, F, vpMapPointMatches) (Tracking::TrackReferenceKeyFrame,
    src/Tracking.cc:839-842): the reference keyframe is frame t of a synthetic
    sequence, the current frame t + 1; every 4th keyframe keypoint has no
    MapPoint and every 9th is bad."""
    from orb_slam_cuda_amd.synth import SynthSequence
    fr = SynthSequence(seed, W, H).frames(2)
    cfg = O.config(nfeatures=nf, width=W, height=H)
    (k1, d1), (k2, d2) = O.extract(cfg, fr[0]), O.extract(cfg, fr[1])
    n1 = len(k1)
    kmp = np.where(np.arange(n1) % 4 == 3, -1, np.arange(n1)).astype(np.int32)
    bad = (np.arange(n1) % 9 == 4).astype(np.uint8)
    good = ((kmp >= 0) & (bad[np.maximum(kmp, 0)] == 0)).astype(np.uint8)
    fa, fb = _featvec_csr(d1, seed), _featvec_csr(d2, seed)
    info = O.level_info(cfg)
    recs = dict(op=np.int32([OPS["bow"]]), nnratio=np.float32([ratio]), check_ori=np.int32([1]),
                mp_desc=np.ascontiguousarray(d1, np.uint8), mp_bad=bad)
    recs.update(_side("B", k1, d1, (0, W, 0, H), info["scale"], mps=kmp, fv_nodes=fa[0], fv_off=fa[1],
                      fv_idx=fa[2]))
    recs.update(_side("A", k2, d2, (0, W, 0, H), info["scale"], fv_nodes=fb[0], fv_off=fb[1], fv_idx=fb[2]))
    out, nm = _cpu(lambda: O.search_by_bow(d1, k1["angle"], good, tuple(x.astype(np.uint32) if i == 0 else x
                                                                        for i, x in enumerate(fa)),
                                           d2, k2["angle"], np.ones(len(d2), np.uint8),
                                           tuple(x.astype(np.uint32) if i == 0 else x for i, x in enumerate(fb)),
                                           ratio, True, False))
    want = np.where(out >= 0, kmp[np.maximum(out, 0)], -1)
    return recs, np.concatenate([[nm], want]).astype(np.int32)
