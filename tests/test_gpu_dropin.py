"""GPU checks of the drop-in per-frame path (round 5): the pinned host
pyramid orbx_extract fills beside its kernels (mvImagePyramid,
include/ORBextractor.h:116, src/ORBextractor.cc:1837-1863) and the stereo
matcher that reads the two extractions' device outputs in place
(orbm_compute_stereo_matches_last, src/Frame.cc:77-89, 465-639). Both are
checked bit-exactly against the oracle (the checker)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MB, MBF = 0.54, np.float32(0.54 * 718.856)


def test_host_pyramid_equals_oracle(pkg, O):
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H = 1241, 376
    frames = SynthSequence(31, W, H).frames(3)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    cfg = O.config(nfeatures=2000, width=W, height=H)
    ext(frames[0])
    with pytest.raises(pkg.OrbxError):
        ext.host_pyramid()  # off by default
    ext.set_host_pyramid(True)
    with pytest.raises(pkg.OrbxError):
        ext.host_pyramid()  # no call since it was enabled
    for i, f in enumerate(frames):
        # the first call after enabling runs plain stream operations, later
        # ones replay the captured graph with its copy branch
        kp, desc = ext(f)
        rkp, rdesc = O.extract(cfg, f)
        assert np.array_equal(kp.view(np.uint8), rkp.view(np.uint8)) and np.array_equal(desc, rdesc), i
        hp = ext.host_pyramid()
        assert np.array_equal(hp[0], f), i
        for l in range(1, 8):
            assert np.array_equal(hp[l], O.pyramid_level(cfg, f, l)), (i, l)
        # orbx_get_level serves level reads from the same copy
        assert np.array_equal(ext.level_image(3), hp[3])
    ext.set_host_pyramid(False)
    ext(frames[0])
    with pytest.raises(pkg.OrbxError):
        ext.host_pyramid()
    # the device read path (stream-scoped wait, no device-wide sync) still serves mvImagePyramid
    assert np.array_equal(ext.level_image(2), O.pyramid_level(cfg, frames[0], 2))


def test_host_pyramid_new_image_size_and_batch(pkg, O):
    """A new image size re-plans the handle (the copy's layout with it); a batch
    call invalidates the host copy (it holds an earlier orbx_extract's frame)."""
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import synth_frame
    ext = pkg.ORBextractor(1000, 1.2, 8, 20, 7, 752, 480)
    ext.set_host_pyramid(True)
    for (W, H) in ((752, 480), (640, 240), (752, 480)):
        f = synth_frame(W + H, W, H)
        ext(f)
        hp = ext.host_pyramid()
        cfg = O.config(nfeatures=1000, width=W, height=H)
        assert np.array_equal(hp[0], f)
        for l in (1, 4, 7):
            assert np.array_equal(hp[l], O.pyramid_level(cfg, f, l)), (W, H, l)
    W, H = 752, 480
    pitch = (W + 63) & ~63
    d = _lib.DeviceArray(H * pitch)
    img = np.zeros((H, pitch), np.uint8)
    img[:, :W] = synth_frame(5, W, H)
    d.upload(img)
    cap = ext.frame_capacity
    dk, dd, dc = _lib.DeviceArray(cap * 28), _lib.DeviceArray(cap * 32), _lib.DeviceArray(16)
    ext.extract_batch_device(d.ptr, 1, H * pitch, pitch, dk.ptr, dd.ptr, dc.ptr)
    with pytest.raises(pkg.OrbxError):
        ext.host_pyramid()
    assert ext.status() == 0


@pytest.mark.parametrize("seed", [3, 8])
def test_stereo_last_equals_oracle(pkg, O, seed):
    from orb_slam_cuda_amd.synth import stereo_pair
    W, H = 1241, 376
    imL, imR = stereo_pair(seed, W, H)
    eL = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    eR = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    m = pkg.ORBmatcher(max_kps=4096)
    for _ in range(2):  # plain first call, then the graph replay
        kL, dL = eL(imL)
        kR, dR = eR(imR)
        F = pkg.Frame.from_extraction(kL, dL, W, H)
        F.mvKeysRight, F.mDescriptorsRight, F.mb, F.mbf = kR, dR, MB, float(MBF)
        kept = pkg.ComputeStereoMatchesLast(F, eL, eR, m)
        cfg = O.config(nfeatures=2000, width=W, height=H)
        li = O.level_info(cfg)
        uR, dep, ekept = O.compute_stereo_matches(kL, dL, kR, dR, O.pyramid(cfg, imL), O.pyramid(cfg, imR),
                                                  li["scale"], li["inv_scale"], MB, MBF)
        assert kept == ekept > 0.3 * len(kL)
        assert np.array_equal(F.mvuRight, uR) and np.array_equal(F.mvDepth, dep)


def test_stereo_last_refuses_batch_extraction(pkg):
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import stereo_pair
    W, H = 640, 240
    imL, imR = stereo_pair(2, W, H)
    eL = pkg.ORBextractor(500, 1.2, 8, 20, 7, W, H)
    eR = pkg.ORBextractor(500, 1.2, 8, 20, 7, W, H)
    m = pkg.ORBmatcher(max_kps=4096)
    eL(imL)
    eR(imR)
    pitch = (W + 63) & ~63
    d = _lib.DeviceArray(H * pitch)
    img = np.zeros((H, pitch), np.uint8)
    img[:, :W] = imL
    d.upload(img)
    cap = eL.frame_capacity
    dk, dd, dc = _lib.DeviceArray(cap * 28), _lib.DeviceArray(cap * 32), _lib.DeviceArray(16)
    eL.extract_batch_device(d.ptr, 1, H * pitch, pitch, dk.ptr, dd.ptr, dc.ptr)
    F = pkg.Frame.from_extraction(np.zeros(0, pkg.KP_DTYPE), np.zeros((0, 32), np.uint8), W, H)
    F.mb, F.mbf = MB, float(MBF)
    with pytest.raises(pkg.OrbxError):
        pkg.ComputeStereoMatchesLast(F, eL, eR, m)
    n = C.c_int(0)
    assert _lib.lib().orbx_get_status(eL.handle, 1, C.byref(n)) == 0 and n.value == 0
