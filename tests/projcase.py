"""Synthetic inputs for ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th):
a frame extracted by the oracle plus projected MapPoints near (and away from)
its keypoints, with descriptor noise, duplicated points (several points racing
for one keypoint, which exercises the sequential blocking of src/ORBmatcher.cc:
86-88 / 115), stereo right coordinates and pre-blocked keypoints."""
import numpy as np


def projection_case(O, seed, W=1241, H=376, nf=2000, nmp=3000, stereo=False):
    from orb_slam_cuda_amd.synth import synth_frame
    img = synth_frame(seed, W, H)
    cfg = O.config(nfeatures=nf, width=W, height=H)
    kps, desc = O.extract(cfg, img)
    scale = O.level_info(cfg)["scale"]
    rng = np.random.default_rng(seed)
    n = len(kps)
    mps = np.zeros(nmp, O.MP_DTYPE)
    mpd = rng.integers(0, 256, (nmp, 32), dtype=np.uint8)
    near = rng.random(nmp) < 0.7
    src = rng.integers(0, n, nmp)
    mps["proj_x"] = np.where(near, kps["x"][src] + rng.normal(0, 1.5, nmp), rng.uniform(-20, W + 20, nmp))
    mps["proj_y"] = np.where(near, kps["y"][src] + rng.normal(0, 1.5, nmp), rng.uniform(-20, H + 20, nmp))
    lvl = np.where(near, kps["octave"][src] + rng.integers(-1, 2, nmp), rng.integers(0, 8, nmp))
    mps["predicted_level"] = np.clip(lvl, 0, 7)
    flips = rng.random((nmp, 32, 8)) < rng.uniform(0, 0.12, (nmp, 1, 1))
    noise = np.packbits(flips, axis=2).reshape(nmp, 32)
    mpd = np.where(near[:, None], desc[src] ^ noise, mpd).astype(np.uint8)
    mps["view_cos"] = rng.uniform(0.99, 1.0, nmp)
    mps["track_in_view"] = rng.random(nmp) < 0.92
    mps["obs_positive"] = rng.random(nmp) < 0.85
    # duplicates: later points copying earlier ones race for the same keypoint
    dup = np.nonzero(rng.random(nmp) < 0.12)[0]
    dup = dup[dup > 0]
    srcd = rng.integers(0, dup, len(dup)) if len(dup) else dup
    mps[dup] = mps[srcd]
    mpd[dup] = mpd[srcd]
    uright = None
    if stereo:
        disp = rng.uniform(3, 40, n).astype(np.float32)
        uright = np.where(rng.random(n) < 0.7, kps["x"] - disp, -1.0).astype(np.float32)
        mps["proj_xr"] = np.where(near, np.where(uright[src] > 0, uright[src], kps["x"][src] - 10)
                                  + rng.normal(0, 2.0, nmp), rng.uniform(0, W, nmp))
    blocked = (rng.random(n) < 0.1).astype(np.uint8)
    bounds = (0.0, float(W), 0.0, float(H))
    return kps, desc, uright, bounds, scale, blocked, mps, mpd
