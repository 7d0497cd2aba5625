"""Synthetic inputs for the pose-projection SearchByProjection overloads
(src/ORBmatcher.cc:290-403, 1328-1470, 1472-1599): a frame extracted by the
oracle, world points back-projected from its keypoints through a KITTI-like
camera at random depths (so they project back near the keypoints once the
pose is applied), descriptor noise, angle noise (some points land in the
rotation bins the consistency check clears), duplicated points racing for one
keypoint, and points that fail the depth / image / distance / viewing tests."""
import numpy as np

FX, FY, CX, CY, MB = 718.856, 718.856, 607.1928, 185.2157, 0.54


def rodrigues(w):
    w = np.asarray(w, np.float64)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def pose(rng, rot=0.05, trans=1.0):
    T = np.eye(4)
    T[:3, :3] = rodrigues(rng.normal(0, rot, 3))
    T[:3, 3] = rng.normal(0, trans, 3)
    return T


def _frame(O, seed, W, H, nf):
    from orb_slam_cuda_amd.synth import synth_frame
    cfg = O.config(nfeatures=nf, width=W, height=H)
    kps, desc = O.extract(cfg, synth_frame(seed, W, H))
    return kps, desc, O.level_info(cfg)["scale"]


def _noisy(rng, desc, rate_hi=0.12):
    m = len(desc)
    flips = rng.random((m, 32, 8)) < rng.uniform(0, rate_hi, (m, 1, 1))
    return (desc ^ np.packbits(flips, axis=2).reshape(m, 32)).astype(np.uint8)


def _points(rng, kps, Tcw, nmp, W, H, near_frac=0.8, px_noise=1.0):
    """World points: a near_frac share back-projected from keypoints (src index, depth z),
    the rest random in front of / behind the camera."""
    n = len(kps)
    src = rng.integers(0, n, nmp)
    near = rng.random(nmp) < near_frac
    z = rng.uniform(2.0, 45.0, nmp)
    u = np.where(near, kps["x"][src] + rng.normal(0, px_noise, nmp), rng.uniform(-40, W + 40, nmp))
    v = np.where(near, kps["y"][src] + rng.normal(0, px_noise, nmp), rng.uniform(-40, H + 40, nmp))
    z = np.where(near | (rng.random(nmp) < 0.8), z, -z)
    Xc = np.stack([(u - CX) / FX * z, (v - CY) / FY * z, z], 1)
    Twc = np.linalg.inv(Tcw)
    Xw = Xc @ Twc[:3, :3].T + Twc[:3, 3]
    return src, near, Xw.astype(np.float32), z


def _dups(rng, mps, mpd, frac=0.1):
    dup = np.nonzero(rng.random(len(mps)) < frac)[0]
    dup = dup[dup > 0]
    if len(dup):
        s = rng.integers(0, dup, len(dup))
        mps[dup] = mps[s]
        mpd[dup] = mpd[s]


def last_frame_case(O, seed, W=1241, H=376, nf=2000, nmp=2000, stereo=False, motion="none", mono=None):
    """CurrentFrame + LastFrame records for SearchByProjection(CurrentFrame, LastFrame, th, bMono).
    motion: 'forward' / 'backward' puts the last camera ahead of / behind the current one
    along z by more than mb (the bForward / bBackward level windows), 'none' keeps it close."""
    kps, desc, scale = _frame(O, seed, W, H, nf)
    rng = np.random.default_rng(1000 + seed)
    Tcw = pose(rng)
    Tlw = Tcw.copy()
    dz = {"none": 0.1, "forward": 2.0, "backward": -2.0}[motion]
    Tlw[2, 3] += dz  # tlc = Rlw*twc + tlw = (0, 0, dz) for Rlw = Rcw
    src, near, Xw, z = _points(rng, kps, Tcw, nmp, W, H)
    mps = np.zeros(nmp, O.MPW_DTYPE)
    mps["pos"] = Xw
    oct_ = np.where(near, kps["octave"][src] + rng.integers(-1, 2, nmp), rng.integers(0, 8, nmp))
    mps["octave"] = np.clip(oct_, 0, 7)
    ang = kps["angle"][src] + rng.normal(0, 3.0, nmp)
    wild = rng.random(nmp) < 0.15
    mps["angle"] = np.mod(np.where(wild, rng.uniform(0, 360, nmp), ang), 360.0)
    mps["valid"] = rng.random(nmp) < 0.92
    mps["obs_positive"] = rng.random(nmp) < 0.8
    mpd = np.where(near[:, None], _noisy(rng, desc[src]), rng.integers(0, 256, (nmp, 32))).astype(np.uint8)
    _dups(rng, mps, mpd)
    uright = None
    if stereo:
        n = len(kps)
        zk = rng.uniform(2.0, 45.0, n)
        zk[src[near]] = z[near]
        uright = np.where(rng.random(n) < 0.7, kps["x"] - FX * MB / zk, -1.0).astype(np.float32)
    blocked = (rng.random(len(kps)) < 0.08).astype(np.uint8)
    cam = O.camera(FX, FY, CX, CY, MB, MB * FX, Tcw[:3])
    if mono is None:
        mono = not stereo
    return dict(kps=kps, desc=desc, uright=uright, bounds=(0.0, float(W), 0.0, float(H)), scale=scale,
                blocked=blocked, cam=cam, Tcw=Tcw[:3].astype(np.float32), Tlw=Tlw[:3].astype(np.float32),
                mps=mps, mpdesc=mpd, mono=mono)


def _distances(rng, mps, Xw, Tcw, src, near, kps, sf=1.2, L=8):
    """mfMaxDistance / mfMinDistance so that PredictScale lands near the source octave."""
    Ow = np.linalg.inv(Tcw)[:3, 3]
    d = np.linalg.norm(Xw.astype(np.float64) - Ow, axis=1)
    lvl = np.where(near, kps["octave"][src], rng.integers(0, L, len(d)))
    maxd = d * sf ** (lvl - rng.uniform(0.05, 0.95, len(d)))
    out = rng.random(len(d)) < 0.05  # outside the scale-invariance region
    maxd = np.where(out, d * 0.5, maxd)
    mps["max_distance"] = maxd.astype(np.float32)
    mps["min_distance"] = (maxd / sf ** (L - 1)).astype(np.float32)
    return d


def keyframe_case(O, seed, W=1241, H=376, nf=2000, nmp=2000):
    """CurrentFrame + KeyFrame map points for the relocalization overload."""
    kps, desc, scale = _frame(O, seed, W, H, nf)
    rng = np.random.default_rng(2000 + seed)
    Tcw = pose(rng)
    src, near, Xw, z = _points(rng, kps, Tcw, nmp, W, H)
    mps = np.zeros(nmp, O.MPW_DTYPE)
    mps["pos"] = Xw
    _distances(rng, mps, Xw, Tcw, src, near, kps)
    ang = kps["angle"][src] + rng.normal(0, 3.0, nmp)
    wild = rng.random(nmp) < 0.15
    mps["angle"] = np.mod(np.where(wild, rng.uniform(0, 360, nmp), ang), 360.0)
    mps["valid"] = rng.random(nmp) < 0.9
    mps["obs_positive"] = 1
    mpd = np.where(near[:, None], _noisy(rng, desc[src]), rng.integers(0, 256, (nmp, 32))).astype(np.uint8)
    _dups(rng, mps, mpd)
    has_mp = (rng.random(len(kps)) < 0.15).astype(np.uint8)
    cam = O.camera(FX, FY, CX, CY, MB, MB * FX, Tcw[:3])
    return dict(kps=kps, desc=desc, bounds=(0.0, float(W), 0.0, float(H)), scale=scale, has_mp=has_mp, cam=cam,
                mps=mps, mpdesc=mpd)


def sim3_case(O, seed, W=1241, H=376, nf=2000, nmp=3000, s=1.3):
    """KeyFrame + candidate points for the loop-closing overload; Scw = s * [R | t]."""
    kps, desc, scale = _frame(O, seed, W, H, nf)
    rng = np.random.default_rng(3000 + seed)
    Tcw = pose(rng)
    src, near, Xw, z = _points(rng, kps, Tcw, nmp, W, H)
    mps = np.zeros(nmp, O.MPW_DTYPE)
    mps["pos"] = Xw
    d = _distances(rng, mps, Xw, Tcw, src, near, kps)
    Ow = np.linalg.inv(Tcw)[:3, 3]
    nrm = (Xw - Ow) / d[:, None]
    flip = rng.random(nmp) < 0.08  # viewing angle test fails
    tilt = nrm + rng.normal(0, 0.3, (nmp, 3))
    tilt /= np.linalg.norm(tilt, axis=1, keepdims=True)
    mps["normal"] = np.where(flip[:, None], -nrm, tilt).astype(np.float32)
    mps["valid"] = rng.random(nmp) < 0.9
    mps["obs_positive"] = 1
    mpd = np.where(near[:, None], _noisy(rng, desc[src], 0.08), rng.integers(0, 256, (nmp, 32))).astype(np.uint8)
    _dups(rng, mps, mpd)
    matched = np.where(rng.random(len(kps)) < 0.1, rng.integers(0, 10**6, len(kps)), -1).astype(np.int32)
    Scw = Tcw[:3].copy()
    Scw[:, :3] *= s  # sRcw = s*R; the overload divides by s = |row 0|
    Scw[:, 3] *= s
    cam = O.camera(FX, FY, CX, CY, MB, MB * FX, Scw)
    return dict(kps=kps, desc=desc, bounds=(0.0, float(W), 0.0, float(H)), scale=scale, cam=cam, mps=mps,
                mpdesc=mpd, matched=matched)


def fuse_case(O, seed, W=1241, H=376, nf=2000, nmp=3000, stereo=True):
    """KeyFrame (with mvuRight) + candidate points for Fuse(pKF, vpMapPoints, th)."""
    kps, desc, scale = _frame(O, seed, W, H, nf)
    cfg = O.config(nfeatures=nf, width=W, height=H)
    info = O.level_info(cfg)
    rng = np.random.default_rng(4000 + seed)
    Tcw = pose(rng)
    src, near, Xw, z = _points(rng, kps, Tcw, nmp, W, H, px_noise=1.2)
    mps = np.zeros(nmp, O.MPW_DTYPE)
    mps["pos"] = Xw
    d = _distances(rng, mps, Xw, Tcw, src, near, kps)
    Ow = np.linalg.inv(Tcw)[:3, 3]
    nrm = (Xw - Ow) / d[:, None]
    flip = rng.random(nmp) < 0.06
    mps["normal"] = np.where(flip[:, None], -nrm, nrm).astype(np.float32)
    mps["valid"] = rng.random(nmp) < 0.9
    mps["obs_positive"] = 1
    mpd = np.where(near[:, None], _noisy(rng, desc[src], 0.06), rng.integers(0, 256, (nmp, 32))).astype(np.uint8)
    _dups(rng, mps, mpd, 0.05)
    uright = None
    if stereo:
        n = len(kps)
        zk = rng.uniform(2.0, 45.0, n)
        zk[src[near]] = z[near]
        uright = np.where(rng.random(n) < 0.6, kps["x"] - FX * MB / zk + rng.normal(0, 0.8, n), -1.0).astype(np.float32)
    cam = O.camera(FX, FY, CX, CY, MB, MB * FX, Tcw[:3])
    return dict(kps=kps, desc=desc, uright=uright, bounds=(0.0, float(W), 0.0, float(H)), scale=scale,
                inv_sigma2=info["inv_sigma2"], cam=cam, mps=mps, mpdesc=mpd)


def _kf2_from_kf1(rng, O, kps1, desc1, T1w, T2w, W, H, frac=0.85, extra=300):
    """A second keyframe seeing KF1's keypoints from pose T2w: each KF1 keypoint i (with frac
    probability) is back-projected at a random depth and re-projected into KF2 with pixel noise
    and descriptor noise; plus `extra` random keypoints. Returns (kps2, desc2, Xw1, src2) with
    src2[j] = the KF1 keypoint behind KF2 keypoint j (-1 for the extras)."""
    n1 = len(kps1)
    z = rng.uniform(3.0, 40.0, n1)
    Xc1 = np.stack([(kps1["x"] - CX) / FX * z, (kps1["y"] - CY) / FY * z, z], 1)
    T1 = np.eye(4); T1[:3] = T1w
    T2 = np.eye(4); T2[:3] = T2w
    Xw = Xc1 @ np.linalg.inv(T1)[:3, :3].T + np.linalg.inv(T1)[:3, 3]
    Xc2 = Xw @ T2[:3, :3].T + T2[:3, 3]
    u2 = FX * Xc2[:, 0] / Xc2[:, 2] + CX + rng.normal(0, 0.7, n1)
    v2 = FY * Xc2[:, 1] / Xc2[:, 2] + CY + rng.normal(0, 0.7, n1)
    keep = (rng.random(n1) < frac) & (Xc2[:, 2] > 0) & (u2 > 20) & (u2 < W - 20) & (v2 > 20) & (v2 < H - 20)
    src = np.nonzero(keep)[0]
    m = len(src) + extra
    kps2 = np.zeros(m, kps1.dtype)
    kps2["x"][:len(src)] = u2[src]; kps2["y"][:len(src)] = v2[src]
    kps2["octave"][:len(src)] = kps1["octave"][src]
    kps2["angle"][:len(src)] = np.mod(kps1["angle"][src] + rng.normal(0, 4.0, len(src)), 360.0)
    kps2["x"][len(src):] = rng.uniform(20, W - 20, extra); kps2["y"][len(src):] = rng.uniform(20, H - 20, extra)
    kps2["octave"][len(src):] = rng.integers(0, 8, extra)
    kps2["angle"][len(src):] = rng.uniform(0, 360, extra)
    kps2["size"] = 31.0; kps2["class_id"] = -1
    desc2 = np.concatenate([_noisy(rng, desc1[src], 0.08), rng.integers(0, 256, (extra, 32)).astype(np.uint8)])
    perm = rng.permutation(m)
    src2 = np.concatenate([src, -np.ones(extra, np.int64)])[perm]
    return kps2[perm], desc2[perm], Xw.astype(np.float32), src2


def sim3_match_case(O, seed, W=1241, H=376, nf=1500, s12=1.0):
    """Two keyframes for SearchBySim3; map points: KF1 keypoints -> their world points, KF2 keypoints
    -> the same world points (or random ones for extras)."""
    kps1, desc1, scale = _frame(O, seed, W, H, nf)
    rng = np.random.default_rng(5000 + seed)
    T1 = pose(rng, 0.03, 0.5)
    T2 = T1.copy()
    T2[:3, :3] = rodrigues(rng.normal(0, 0.03, 3)) @ T1[:3, :3]
    T2[:3, 3] += rng.normal(0, 0.3, 3)
    kps2, desc2, Xw, src2 = _kf2_from_kf1(rng, O, kps1, desc1, T1[:3], T2[:3], W, H)
    n1, n2 = len(kps1), len(kps2)

    def records(kps, Xpts, Tcw, dsc):
        m = np.zeros(len(kps), O.MPW_DTYPE)
        m["pos"] = Xpts
        Ow = np.linalg.inv(Tcw)[:3, 3]
        d = np.linalg.norm(Xpts.astype(np.float64) - Ow, axis=1)
        maxd = d * 1.2 ** (kps["octave"] - rng.uniform(0.05, 0.95, len(kps)))
        m["max_distance"] = maxd.astype(np.float32)
        m["min_distance"] = (maxd / 1.2 ** 7).astype(np.float32)
        m["valid"] = rng.random(len(kps)) < 0.85
        m["obs_positive"] = 1
        return m, _noisy(rng, dsc, 0.05)
    mps1, mpd1 = records(kps1, Xw, T1, desc1)
    X2 = np.where((src2 >= 0)[:, None], Xw[np.maximum(src2, 0)], rng.normal(0, 10, (n2, 3)) + [0, 0, 20])
    mps2, mpd2 = records(kps2, X2.astype(np.float32), T2, desc2)
    # Sim3 S12 mapping camera-2 coordinates to camera 1: p1 = s R12 p2 + t12
    R12 = T1[:3, :3] @ T2[:3, :3].T
    t12 = T1[:3, 3] - R12 @ T2[:3, 3]
    bounds = (0.0, float(W), 0.0, float(H))
    kf1 = dict(kps=kps1, desc=desc1, bounds=bounds, scale=scale, Tcw=T1[:3].astype(np.float32), mps=mps1, mpdesc=mpd1)
    kf2 = dict(kps=kps2, desc=desc2, bounds=bounds, scale=scale, Tcw=T2[:3].astype(np.float32), mps=mps2, mpdesc=mpd2)
    cam1 = O.camera(FX, FY, CX, CY, MB, MB * FX, T1[:3])
    return kf1, kf2, cam1, np.float32(s12), R12.astype(np.float32), (t12 * s12).astype(np.float32)


def _skew(t):
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])


def triangulation_case(O, seed, W=1241, H=376, nf=2000, stereo_frac=0.4, nodes=80):
    """Two keyframes for SearchForTriangulation with FeatureVectors (CSR) whose nodes are shared by
    corresponding keypoints, F12 from the relative pose (LocalMapping::ComputeF12)."""
    kps1, desc1, scale = _frame(O, seed, W, H, nf)
    cfg = O.config(nfeatures=nf, width=W, height=H)
    info = O.level_info(cfg)
    rng = np.random.default_rng(6000 + seed)
    T1 = pose(rng, 0.03, 0.5)
    T2 = T1.copy()
    T2[:3, :3] = rodrigues(rng.normal(0, 0.03, 3)) @ T1[:3, :3]
    T2[:3, 3] += rng.normal(0, 0.4, 3)
    kps2, desc2, Xw, src2 = _kf2_from_kf1(rng, O, kps1, desc1, T1[:3], T2[:3], W, H)
    n1, n2 = len(kps1), len(kps2)
    node1 = rng.integers(0, nodes, n1)
    node2 = np.where((src2 >= 0) & (rng.random(n2) < 0.9), node1[np.maximum(src2, 0)], rng.integers(0, nodes, n2))
    node2 = np.where(rng.random(n2) < 0.05, nodes + rng.integers(0, 5, n2), node2)  # nodes KF1 lacks

    def csr(node, n):
        ids = np.unique(node)
        off = np.zeros(len(ids) + 1, np.int32)
        idx = []
        for k, i in enumerate(ids):
            v = np.nonzero(node == i)[0]
            idx.extend(v.tolist())
            off[k + 1] = off[k] + len(v)
        return (ids * 7 + 3).astype(np.uint32), off, np.asarray(idx, np.int32)
    ur1 = np.where(rng.random(n1) < stereo_frac, kps1["x"] - rng.uniform(2, 40, n1), -1).astype(np.float32)
    ur2 = np.where(rng.random(n2) < stereo_frac, kps2["x"] - rng.uniform(2, 40, n2), -1).astype(np.float32)
    kf1 = dict(kps=kps1, desc=desc1, uright=ur1, has_mp=(rng.random(n1) < 0.25).astype(np.uint8), fv=csr(node1, n1))
    kf2 = dict(kps=kps2, desc=desc2, uright=ur2, has_mp=(rng.random(n2) < 0.25).astype(np.uint8), fv=csr(node2, n2),
               scale=scale)
    cw1 = np.linalg.inv(T1)[:3, 3].astype(np.float32)
    R12 = T1[:3, :3] @ T2[:3, :3].T
    t12 = T1[:3, 3] - R12 @ T2[:3, 3]
    K = np.array([[FX, 0, CX], [0, FY, CY], [0, 0, 1]])
    F12 = (np.linalg.inv(K).T @ _skew(t12) @ R12 @ np.linalg.inv(K)).astype(np.float32)
    cam2 = np.array([FX, FY, CX, CY], np.float32)
    return kf1, kf2, cw1, T2[:3].astype(np.float32), cam2, info["sigma2"], F12
