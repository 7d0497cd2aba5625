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
