"""GPU parity at the extractor settings the reference itself ships.

Each case is one yaml of `Examples/` (ORBextractor.nFeatures / nLevels /
iniThFAST / minThFAST and the camera size; src/Tracking.cc:123-141 reads
them into `ORBextractor(...)`, src/ORBextractor.cc:496-560):

* KITTI14.yaml: 10 levels, 17/7 on the KITTI 04-12 camera (1226x370): the
  pyramid past 8 levels and the >8-level orient+BRIEF instantiation;
* KITTI06.yaml: 1226x370, 12/7;
* intcatch-1080p.yaml: 1920x1080 (cx 957 / cy 531), 3 levels, 10/4;
* intcatch-720p2.yaml: 1280x720, nF 1500, 7 levels, 30/8;
* intcatch-720p.yaml: 1280x720, nF 1500, 8 levels, 35/7;
* intcatch-nvidia.yaml: 1280x720, nF 1500, 25/9;
* TUM1.yaml: 640x480, nF 1000.

Checked bit-exact against the oracle (the checker): keypoints (all fields and
order), descriptors, every pyramid and blurred level, per-level FAST
candidates, and the device batch API (B = 32 frames of a sequence in one
`orbx_extract_batch`)."""
import numpy as np
import pytest

from test_gpu_extract import assert_same

pytestmark = pytest.mark.gpu

# name: (W, H, nfeatures, nlevels, iniThFAST, minThFAST)
YAMLS = {
    "KITTI14": (1226, 370, 2000, 10, 17, 7),
    "KITTI06": (1226, 370, 2000, 8, 12, 7),
    "intcatch-1080p": (1920, 1080, 2000, 3, 10, 4),
    "intcatch-720p2": (1280, 720, 1500, 7, 30, 8),
    "intcatch-720p": (1280, 720, 1500, 8, 35, 7),
    "intcatch-nvidia": (1280, 720, 1500, 8, 25, 9),
    "TUM1": (640, 480, 1000, 8, 20, 7),
}


def _cfg(O, W, H, nf, L, ini, mn):
    return O.config(nfeatures=nf, width=W, height=H, nlevels=L, ini_th=ini, min_th=mn)


@pytest.mark.parametrize("name", sorted(YAMLS))
def test_yaml_single_frame_parity(pkg, O, name):
    from orb_slam_cuda_amd.synth import synth_frame
    W, H, nf, L, ini, mn = YAMLS[name]
    ext = pkg.ORBextractor(nf, 1.2, L, ini, mn, W, H)
    cfg = _cfg(O, W, H, nf, L, ini, mn)
    for seed in (3, 40):
        img = synth_frame(seed, W, H)
        kp, desc = ext(img)
        rkp, rdesc = O.extract(cfg, img)
        assert_same(kp, desc, rkp, rdesc)
        assert len(kp) > 0.8 * nf
        assert int(kp["octave"].max()) == L - 1
        for l in range(L):
            assert np.array_equal(ext.level_image(l), O.pyramid_level(cfg, img, l)), f"pyramid {l}"
            assert np.array_equal(ext.level_image(l, blurred=True), O.blur_level(cfg, img, l)), f"blur {l}"
            g, r = ext.fast_candidates(l), O.fast_level(cfg, img, l)
            assert len(g) == len(r), (l, len(g), len(r))
            for f in ("x", "y", "response"):
                assert np.array_equal(g[f], r[f]), f"fast {l} {f}"


@pytest.mark.parametrize("name", sorted(YAMLS))
def test_yaml_batch_parity(pkg, O, name):
    from concurrent.futures import ThreadPoolExecutor

    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, nf, L, ini, mn = YAMLS[name]
    B = 32
    frames = SynthSequence(70, W, H).frames(B)
    ext = pkg.ORBextractor(nf, 1.2, L, ini, mn, W, H, max_batch=B)
    cap = ext.frame_capacity
    pitch = (W + 63) & ~63
    host = np.zeros((B, H, pitch), np.uint8)
    host[:, :, :W] = frames
    d_in = _lib.DeviceArray(host.nbytes)
    d_in.upload(host)
    d_kp, d_desc, d_n = _lib.DeviceArray(B * cap * 28), _lib.DeviceArray(B * cap * 32), _lib.DeviceArray(B * 4)
    s = _lib.Stream()
    ext.extract_batch_device(d_in.ptr, B, H * pitch, pitch, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
    s.synchronize()
    assert ext.status() == 0
    n = d_n.download(B, np.int32)
    kps = d_kp.download(B * cap, pkg.KP_DTYPE).reshape(B, cap)
    descs = d_desc.download((B, cap, 32), np.uint8)
    cfg = _cfg(O, W, H, nf, L, ini, mn)
    with ThreadPoolExecutor(8) as ex:  # the oracle's C calls release the GIL
        ref = list(ex.map(lambda f: O.extract(cfg, f), frames))
    for i in range(B):
        rkp, rdesc = ref[i]
        assert_same(kps[i, :n[i]], descs[i, :n[i]], rkp, rdesc)
