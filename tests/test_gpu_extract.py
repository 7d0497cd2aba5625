"""GPU parity of the HIP extractor (liborbx.so) against the CPU oracle.

Bar: bit-exact keypoints (x, y, size, angle, response, octave, class_id, and
their order) and descriptor bytes, plus the stage probes (pyramid levels,
blurred levels, per-cell FAST candidates). All calls go through the C ABI.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def assert_same(kp, desc, rkp, rdesc):
    assert len(kp) == len(rkp), (len(kp), len(rkp))
    for f in FIELDS:
        if not np.array_equal(kp[f], rkp[f]):
            i = int(np.argmax(kp[f] != rkp[f]))
            raise AssertionError(f"field {f} differs first at {i}: {kp[i]} vs {rkp[i]}")
    assert np.array_equal(desc, rdesc), f"descriptor rows differ: {np.nonzero((desc != rdesc).any(1))[0][:10]}"


def oracle_cfg(O, nf, W, H, **kw):
    return O.config(nfeatures=nf, width=W, height=H, scale_mode=1 if kw.get("scale_mode") == "F" else 0,
                    pattern_mode=1 if kw.get("pattern") == "upstream" else 0,
                    scale_factor=kw.get("scale_factor", 1.2), nlevels=kw.get("nlevels", 8),
                    ini_th=kw.get("ini", 20), min_th=kw.get("mn", 7))


@pytest.mark.parametrize("seed", [0, 1, 2, 9])
def test_kitti_full_frame_parity(pkg, O, seed):
    from orb_slam_cuda_amd.synth import synth_frame
    W, H = 1241, 376
    img = synth_frame(seed, W, H)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    kp, desc = ext(img)
    rkp, rdesc = O.extract(oracle_cfg(O, 2000, W, H), img)
    assert_same(kp, desc, rkp, rdesc)
    assert 1990 <= len(kp) <= 2016


def test_stage_probes(pkg, O):
    from orb_slam_cuda_amd.synth import synth_frame
    W, H = 1241, 376
    img = synth_frame(5, W, H)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    ext(img)
    cfg = oracle_cfg(O, 2000, W, H)
    for l in range(8):
        assert np.array_equal(ext.level_image(l), O.pyramid_level(cfg, img, l)), f"pyramid {l}"
        assert np.array_equal(ext.level_image(l, blurred=True), O.blur_level(cfg, img, l)), f"blur {l}"
        g, r = ext.fast_candidates(l), O.fast_level(cfg, img, l)
        assert len(g) == len(r)
        for f in ("x", "y", "response"):
            assert np.array_equal(g[f], r[f]), f"fast {l} {f}"
    pyr = ext.mvImagePyramid
    assert [p.shape for p in pyr] == [(376, 1241), (313, 1034), (261, 862), (218, 718), (181, 598),
                                      (151, 499), (126, 416), (105, 346)]


@pytest.mark.parametrize("name", ["kitti_s0", "euroc_s3", "kitti_s4_modeF"])
def test_golden_vectors(pkg, name):
    from orb_slam_cuda_amd.synth import synth_frame
    g = np.load(os.path.join(GOLDEN, f"extract_{name}.npz"))
    W, H = int(g["W"]), int(g["H"])
    img = synth_frame(int(g["seed"]), W, H)
    assert sha(img) == str(g["image_sha"])
    ext = pkg.ORBextractor(int(g["nfeatures"]), 1.2, 8, 20, 7, W, H, scale_mode="UF"[int(g["scale_mode"])])
    kp, desc = ext(img)
    assert np.array_equal(kp.view(np.uint8).reshape(len(kp), 28), g["keypoints"])
    assert np.array_equal(desc, g["descriptors"])
    for l in range(8):
        assert sha(ext.level_image(l)) == g["pyramid_sha"][l]
        assert sha(ext.level_image(l, blurred=True)) == g["blur_sha"][l]
        assert len(ext.fast_candidates(l)) == g["fast_counts"][l]


@pytest.mark.parametrize("kw", [
    dict(nf=4000),                                  # the 2x initialisation extractor (Tracking.cc:133)
    dict(nf=1000, W=752, H=480),                    # EuRoC
    dict(nf=500),
    dict(nf=2000, scale_mode="F"),                  # fork's VX ORB-scale override
    dict(nf=2000, pattern="upstream"),              # upstream BRIEF table
    dict(nf=1500, nlevels=4),
    dict(nf=800, scale_factor=2.0, nlevels=4, W=1280, H=720),  # exact 2x: INTER_AREA path
    dict(nf=1200, scale_factor=1.5, nlevels=5),
    dict(nf=2000, ini=30, mn=10),
    dict(nf=2000, ini=5, mn=12),                    # iniTh < minTh
    dict(nf=0),                                     # no features requested
    dict(nf=600, W=369, H=300),                     # 39-px cells at level 5: FAST's 48-byte ROI stride, full
    dict(nf=600, W=420, H=300),                     # 43-px cells at level 7: FAST's 80-byte ROI stride path
])
def test_config_parity(pkg, O, kw):
    from orb_slam_cuda_amd.synth import synth_frame
    W, H, nf = kw.pop("W", 1241), kw.pop("H", 376), kw.pop("nf")
    img = synth_frame(21, W, H)
    extra = {k: kw[k] for k in ("scale_mode", "pattern") if k in kw}
    ext = pkg.ORBextractor(nf, kw.get("scale_factor", 1.2), kw.get("nlevels", 8), kw.get("ini", 20),
                           kw.get("mn", 7), W, H, **extra)
    kp, desc = ext(img)
    rkp, rdesc = O.extract(oracle_cfg(O, nf, W, H, **kw), img)
    assert_same(kp, desc, rkp, rdesc)


def test_dense_noise_uses_global_quadtree_path(pkg, O):
    # pure noise: tens of thousands of FAST candidates per level, beyond the LDS key budget
    rng = np.random.default_rng(4)
    W, H = 1241, 376
    img = rng.integers(0, 256, size=(H, W), dtype=np.uint8)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    kp, desc = ext(img)
    assert len(ext.fast_candidates(0)) > 10000
    rkp, rdesc = O.extract(oracle_cfg(O, 2000, W, H), img)
    assert_same(kp, desc, rkp, rdesc)


@pytest.mark.parametrize("W,H", [(1241, 376), (752, 480)])
def test_fast_noise_ramp(pkg, O, W, H):
    # noise of rising amplitude across the frame: cells from a handful of
    # compass survivors to nearly every band pixel listed, from no corners to
    # hundreds detected (the multi-chunk NMS path), per-cell FAST candidates
    # and the full extraction
    rng = np.random.default_rng(6)
    amp = np.repeat(np.linspace(2, 128, 16), -(-W // 16))[:W][None, :]
    base = np.linspace(60, 190, H)[:, None]
    img = np.clip(base + rng.uniform(-1, 1, size=(H, W)) * amp, 0, 255).astype(np.uint8)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    kp, desc = ext(img)
    cfg = oracle_cfg(O, 2000, W, H)
    for l in range(8):
        g, r = ext.fast_candidates(l), O.fast_level(cfg, img, l)
        assert len(g) == len(r), (l, len(g), len(r))
        for f in ("x", "y", "response"):
            assert np.array_equal(g[f], r[f]), f"fast {l} {f}"
    rkp, rdesc = O.extract(cfg, img)
    assert_same(kp, desc, rkp, rdesc)


def test_generic_quadtree_rounds(pkg, O, monkeypatch):
    # the generic quadtree rounds (plans whose node table does not fit the lean
    # rounds' 16-bit packing) on a normal frame and on dense noise
    from orb_slam_cuda_amd.synth import synth_frame
    monkeypatch.setenv("ORBX_QT_GENERIC", "1")
    W, H = 1241, 376
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    rng = np.random.default_rng(5)
    for img in (synth_frame(33, W, H), rng.integers(0, 256, size=(H, W), dtype=np.uint8)):
        kp, desc = ext(img)
        rkp, rdesc = O.extract(oracle_cfg(O, 2000, W, H), img)
        assert_same(kp, desc, rkp, rdesc)


def _clustered_frame(W, H, seed=11, patches=40, side=10):
    # flat background with small noise patches: few keys per level (K ~ N),
    # so the quadtree splits nodes far below the sorted path's bin depth
    rng = np.random.default_rng(seed)
    img = np.full((H, W), 128, np.uint8)
    for _ in range(patches):
        x, y = int(rng.integers(20, W - 30)), int(rng.integers(20, H - 30))
        img[y:y + side, x:x + side] = rng.integers(0, 256, (side, side))
    return img


@pytest.mark.parametrize("W,H,nf", [(1241, 376, 2000), (752, 480, 1000), (1241, 376, 4000)])
def test_quadtree_sorted_path(pkg, O, monkeypatch, W, H, nf):
    """The sorted-key DistributeOctTree (every node a contiguous range of keys
    binned by quadtree path code, orbx_quadtree.hip) runs on every level of
    textured frames and equals the oracle, ties and list order included; the
    legacy rounds (ORBX_QT_SORTED=0) give the same keypoints."""
    from orb_slam_cuda_amd.synth import synth_frame
    cfg = oracle_cfg(O, nf, W, H)
    for seed in (3, 12):
        img = synth_frame(seed, W, H)
        ext = pkg.ORBextractor(nf, 1.2, 8, 20, 7, W, H)
        kp, desc = ext(img)
        assert (ext.quadtree_paths() == 1).all(), ext.quadtree_paths()
        rkp, rdesc = O.extract(cfg, img)
        assert_same(kp, desc, rkp, rdesc)
        assert np.array_equal(ext.tie_stats(), _tie_stats_legacy(pkg, monkeypatch, nf, W, H, img))


def _tie_stats_legacy(pkg, monkeypatch, nf, W, H, img):
    with monkeypatch.context() as m:
        m.setenv("ORBX_QT_SORTED", "0")
        ext = pkg.ORBextractor(nf, 1.2, 8, 20, 7, W, H)
        ext(img)
        assert (ext.quadtree_paths() == 0).all()
        return ext.tie_stats()


@pytest.mark.parametrize("W,H,nf,nl,ini,mn", [(1241, 376, 2000, 8, 20, 7), (1920, 1080, 2000, 3, 10, 4)])
def test_quadtree_spill_mode(pkg, O, W, H, nf, nl, ini, mn):
    """Levels with more keys than the workgroup holds in registers (dense noise
    at KITTI size; intcatch-1080p's yaml, 1920x1080, 3 levels, thresholds
    10/4): the sorted path keeps the keys in a compact global copy and finds
    each key's kept node through the per-bin node map; bit-exact, and at least
    one such level runs the sorted path."""
    from orb_slam_cuda_amd.synth import synth_frame
    rng = np.random.default_rng(8)
    img = (rng.integers(0, 256, size=(H, W), dtype=np.uint8) if W == 1241 else synth_frame(91, W, H))
    ext = pkg.ORBextractor(nf, 1.2, nl, ini, mn, W, H)
    kp, desc = ext(img)
    big = [l for l in range(nl) if len(ext.fast_candidates(l)) > (4096 if W == 1241 else 8192)]
    assert big and (ext.quadtree_paths()[0][big] == 1).any(), (big, ext.quadtree_paths())
    rkp, rdesc = O.extract(oracle_cfg(O, nf, W, H, nlevels=nl, ini=ini, mn=mn), img)
    assert_same(kp, desc, rkp, rdesc)


def test_quadtree_sorted_path_falls_back(pkg, O):
    """Corners in small scattered patches: some level must split a node below
    the bins' depth, its workgroup falls back to the legacy rounds, and every
    level still equals the oracle."""
    W, H = 1241, 376
    img = _clustered_frame(W, H)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    kp, desc = ext(img)
    assert (ext.quadtree_paths() == 0).any()
    rkp, rdesc = O.extract(oracle_cfg(O, 2000, W, H), img)
    assert_same(kp, desc, rkp, rdesc)


def test_edge_images(pkg, O):
    W, H = 640, 360
    ext = pkg.ORBextractor(1000, 1.2, 8, 20, 7, W, H)
    cfg = oracle_cfg(O, 1000, W, H)
    flat = np.full((H, W), 128, np.uint8)
    kp, desc = ext(flat)
    assert len(kp) == 0 and desc.shape == (0, 32)
    # one bright square: only a handful of corners, few quadtree nodes
    sq = flat.copy()
    sq[100:140, 200:260] = 250
    kp, desc = ext(sq)
    rkp, rdesc = O.extract(cfg, sq)
    assert_same(kp, desc, rkp, rdesc)
    assert 0 < len(kp) < 50
    # saturated extremes
    ext_img = (np.indices((H, W)).sum(0) % 7 == 0).astype(np.uint8) * 255
    kp, desc = ext(ext_img)
    rkp, rdesc = O.extract(cfg, ext_img)
    assert_same(kp, desc, rkp, rdesc)
    # empty image: outputs untouched / empty (src/ORBextractor.cc:1542-1543)
    kp, desc = ext(np.zeros((0, 0), np.uint8))
    assert len(kp) == 0


def test_strided_input_and_replan(pkg, O):
    from orb_slam_cuda_amd.synth import synth_frame
    big = synth_frame(8, 1400, 500)
    view = big[40:40 + 376, 100:100 + 1241]  # non-contiguous rows
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, 1241, 376)
    kp, desc = ext(view)
    rkp, rdesc = O.extract(oracle_cfg(O, 2000, 1241, 376), np.ascontiguousarray(view))
    assert_same(kp, desc, rkp, rdesc)
    # a different image size on the same handle re-plans (the reference accepts any size)
    img2 = synth_frame(9, 800, 600)
    kp, desc = ext(img2)
    rkp, rdesc = O.extract(oracle_cfg(O, 2000, 800, 600), img2)
    assert_same(kp, desc, rkp, rdesc)
    assert ext.levels_info()["w"][0] == 800


def test_deferred_plan_without_camera_size(pkg, O):
    """width/height 0 x 0 (Tracking's values for the mono yamls without
    Camera.width/height, src/Tracking.cc:124-133): scale mode U plans on the
    first image; the scales are there before it; mode F and one-sided zeros are
    refused (mode F's scale override needs the width, src/ORBextractor.cc:674-680)."""
    from orb_slam_cuda_amd.synth import synth_frame
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, 0, 0)
    W, H = 1241, 376
    cfg = oracle_cfg(O, 2000, W, H)
    assert np.array_equal(np.asarray(ext.GetScaleFactors(), np.float32), O.level_info(cfg)["scale"])
    img = synth_frame(17, W, H)
    kp, desc = ext(img)
    rkp, rdesc = O.extract(cfg, img)
    assert_same(kp, desc, rkp, rdesc)
    with pytest.raises(pkg.OrbxError):
        pkg.ORBextractor(2000, 1.2, 8, 20, 7, 0, 0, scale_mode="F")
    with pytest.raises(pkg.OrbxError):
        pkg.ORBextractor(2000, 1.2, 8, 20, 7, 0, 376)


def test_invalid_inputs_raise(pkg):
    with pytest.raises(pkg.OrbxError):
        pkg.ORBextractor(2000, 1.0, 8, 20, 7, 1241, 376)       # scaleFactor must be > 1
    with pytest.raises(pkg.OrbxError):
        pkg.ORBextractor(2000, 1.2, 8, 20, 7, 100, 60)         # top levels smaller than one cell
    ext = pkg.ORBextractor(500, 1.2, 4, 20, 7, 320, 240)
    with pytest.raises(pkg.OrbxError):
        ext(np.zeros((240, 320, 3), np.uint8))                 # not CV_8UC1


def test_batch_api_matches_single_calls(pkg):
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, B = 1241, 376, 6
    frames = SynthSequence(31, W, H).frames(B)
    single = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    ref = [single(f) for f in frames]
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=B)
    cap = ext.frame_capacity
    pitch = 1280
    host = np.zeros((B, H, pitch), np.uint8)
    host[:, :, :W] = frames
    d_in = _lib.DeviceArray(host.nbytes)
    d_in.upload(host)
    d_kp, d_desc, d_n = _lib.DeviceArray(B * cap * 28), _lib.DeviceArray(B * cap * 32), _lib.DeviceArray(B * 4)
    s = _lib.Stream()
    ext.extract_batch_device(d_in.ptr, B, H * pitch, pitch, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
    s.synchronize()
    n = d_n.download(B, np.int32)
    kps = d_kp.download(B * cap, pkg.KP_DTYPE).reshape(B, cap)
    descs = d_desc.download((B, cap, 32), np.uint8)
    for i in range(B):
        assert n[i] == len(ref[i][0])
        assert np.array_equal(kps[i, :n[i]].view(np.uint8), ref[i][0].view(np.uint8))
        assert np.array_equal(descs[i, :n[i]], ref[i][1])
    # determinism across repeated launches
    ext.extract_batch_device(d_in.ptr, B, H * pitch, pitch, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
    s.synchronize()
    assert np.array_equal(d_desc.download((B, cap, 32), np.uint8), descs)


def test_full_batch_properties(pkg):
    """At the bench's full batch size: counts within [N-?, N+16], keypoints inside the
    image and sorted by octave, descriptors distinct, results invariant to batch position."""
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, B = 1241, 376, 64
    frames = SynthSequence(77, W, H).frames(B)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=B)
    cap = ext.frame_capacity
    host = np.ascontiguousarray(frames)
    d_in = _lib.DeviceArray(host.nbytes)
    d_in.upload(host)
    d_kp, d_desc, d_n = _lib.DeviceArray(B * cap * 28), _lib.DeviceArray(B * cap * 32), _lib.DeviceArray(B * 4)
    s = _lib.Stream()
    ext.extract_batch_device(d_in.ptr, B, H * W, W, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
    s.synchronize()
    n = d_n.download(B, np.int32)
    kps = d_kp.download(B * cap, pkg.KP_DTYPE).reshape(B, cap)
    assert (n >= 1900).all() and (n <= 2016).all()
    for i in range(B):
        k = kps[i, :n[i]]
        assert (np.diff(k["octave"]) >= 0).all()
        assert (k["x"] >= 0).all() and (k["x"] < W).all() and (k["y"] >= 0).all() and (k["y"] < H).all()
        assert ((k["angle"] >= 0) & (k["angle"] < 360)).all()
    # frame 10 alone == frame 10 inside the batch
    one = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    kp10, _ = one(frames[10])
    assert np.array_equal(kps[10, :n[10]].view(np.uint8), kp10.view(np.uint8))


def test_batch_mode_f_parity(pkg, O):
    """The fork's buildGraph scale override (scale_mode F, src/ORBextractor.cc:674-680,
    what the reference as written always computes) through the device batch API:
    every frame of a batch equals the oracle in mode F."""
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, B = 1241, 376, 8
    frames = SynthSequence(44, W, H).frames(B)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=B, scale_mode="F")
    cap = ext.frame_capacity
    host = np.ascontiguousarray(frames)
    d_in = _lib.DeviceArray(host.nbytes)
    d_in.upload(host)
    d_kp, d_desc, d_n = _lib.DeviceArray(B * cap * 28), _lib.DeviceArray(B * cap * 32), _lib.DeviceArray(B * 4)
    s = _lib.Stream()
    ext.extract_batch_device(d_in.ptr, B, H * W, W, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
    s.synchronize()
    n = d_n.download(B, np.int32)
    kps = d_kp.download(B * cap, pkg.KP_DTYPE).reshape(B, cap)
    descs = d_desc.download((B, cap, 32), np.uint8)
    cfg = oracle_cfg(O, 2000, W, H, scale_mode="F")
    for i in range(B):
        rkp, rdesc = O.extract(cfg, frames[i])
        assert_same(kps[i, :n[i]], descs[i, :n[i]], rkp, rdesc)


@pytest.mark.parametrize("W,H,nl,sf", [(1241, 376, 8, 1.2), (752, 480, 8, 1.2), (1920, 1080, 3, 1.2),
                                       (641, 243, 8, 1.2), (1280, 720, 4, 2.0), (1241, 376, 5, 1.5)])
def test_every_pyramid_plan(pkg, O, monkeypatch, W, H, nl, sf):
    """Every band x column-tile plan of the one-launch pyramid (ORBX_PYR_PLAN
    forces plan i per launch; an index past the plan count falls back to the
    picker) gives the oracle's levels: raw and blurred, and the keypoints."""
    from orb_slam_cuda_amd.synth import synth_frame
    img = synth_frame(W + nl, W, H)
    cfg = O.config(nfeatures=1000, width=W, height=H, nlevels=nl, scale_factor=sf)
    ref = [O.pyramid_level(cfg, img, l) for l in range(nl)]
    rkp, rdesc = O.extract(cfg, img)
    for i in range(8):
        monkeypatch.setenv("ORBX_PYR_PLAN", str(i))
        ext = pkg.ORBextractor(1000, sf, nl, 20, 7, W, H)  # a fresh handle: its first call runs unrecorded
        kp, desc = ext(img)
        for l in range(1, nl):
            assert np.array_equal(ext.level_image(l), ref[l]), (i, l)
        assert_same(kp, desc, rkp, rdesc)


def test_pyramid_plans_random_geometries(pkg, O, monkeypatch):
    """Every kept band x column-tile plan on seeded random image sizes, scale
    factors and level counts (the plan's walk-down rules on shapes the named
    configs do not have): raw pyramid levels equal the oracle's."""
    from orb_slam_cuda_amd.synth import synth_frame
    rng = np.random.default_rng(2024)
    done = 0
    while done < 10:
        W, H = int(rng.integers(300, 2000)), int(rng.integers(200, 1100))
        sf = float(rng.choice([1.1, 1.2, 1.25, 1.5, 2.0]))
        nl = int(rng.integers(2, 9))
        try:
            pkg.ORBextractor(500, sf, nl, 20, 7, W, H)
        except pkg.OrbxError:
            continue  # a level below one FAST cell: refused, as the reference cannot run it
        img = synth_frame(W * 7 + H, W, H)
        cfg = O.config(nfeatures=500, width=W, height=H, nlevels=nl, scale_factor=sf)
        ref = [O.pyramid_level(cfg, img, l) for l in range(nl)]
        for i in range(8):
            monkeypatch.setenv("ORBX_PYR_PLAN", str(i))
            ext = pkg.ORBextractor(500, sf, nl, 20, 7, W, H)
            ext(img)
            for l in range(1, nl):
                assert np.array_equal(ext.level_image(l), ref[l]), (W, H, sf, nl, i, l)
        done += 1
