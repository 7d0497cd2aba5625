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


def test_stereo_frame_one_round_trip_equals_oracle(pkg, O):
    """orbm_stereo_frame (the stereo Frame's two extractions + ComputeStereoMatches
    issued from one thread with one wait) gives the oracle's keypoints, descriptors,
    mvuRight and mvDepth: first call (plain launches), graph replays, a new image size
    (re-plan of both handles), an empty right image and images of different sizes (the
    steps one after the other)."""
    from orb_slam_cuda_amd.synth import stereo_pair
    eL = pkg.ORBextractor(2000, 1.2, 8, 20, 7, 1241, 376)
    eR = pkg.ORBextractor(2000, 1.2, 8, 20, 7, 1241, 376)
    m = pkg.ORBmatcher(max_kps=4096)

    def oracle(imL, imR):
        W, H = imL.shape[1], imL.shape[0]
        cfg = O.config(nfeatures=2000, width=W, height=H)
        li = O.level_info(cfg)
        kL, dL = O.extract(cfg, imL)
        kR, dR = O.extract(cfg, imR)
        uR, dep, kept = O.compute_stereo_matches(kL, dL, kR, dR, O.pyramid(cfg, imL), O.pyramid(cfg, imR),
                                                 li["scale"], li["inv_scale"], MB, MBF)
        return kL, dL, kR, dR, uR, dep, kept

    cases = [(3, 1241, 376), (4, 1241, 376), (5, 1241, 376), (6, 752, 480), (7, 1241, 376)]
    for seed, W, H in cases:
        imL, imR = stereo_pair(seed, W, H)
        got = pkg.ExtractStereo(eL, eR, imL, imR, m, MB, float(MBF))
        want = oracle(imL, imR)
        for g, w, name in zip(got[:4], want[:4], ("kL", "dL", "kR", "dR")):
            assert np.array_equal(np.asarray(g).view(np.uint8), np.asarray(w).view(np.uint8)), (seed, name)
        assert np.array_equal(got[4], want[4]) and np.array_equal(got[5], want[5]), seed
        assert got[6] == want[6] > 0.3 * len(want[0]), seed
        # the same handles then serve the separate calls (the pyramids are the pair's)
        n = C.c_int(0)
        assert pkg.lib().orbx_get_status(eL.handle, 1, C.byref(n)) == 0 and n.value == 0
    # an empty right image: the left keypoints match nothing
    imL, _ = stereo_pair(9, 1241, 376)
    kL, dL, kR, dR, uR, dep, kept = pkg.ExtractStereo(eL, eR, imL, np.zeros((0, 0), np.uint8), m, MB, float(MBF))
    cfg = O.config(nfeatures=2000, width=1241, height=376)
    rkL, rdL = O.extract(cfg, imL)
    assert np.array_equal(kL.view(np.uint8), rkL.view(np.uint8)) and len(kR) == 0
    assert kept == 0 and np.all(uR == -1) and np.all(dep == -1) and len(uR) == len(kL)
    # different sizes: the steps one after the other; the stereo matcher refuses the pair
    imR2, _ = stereo_pair(10, 752, 480)
    with pytest.raises(pkg.OrbxError):
        pkg.ExtractStereo(eL, eR, imL, imR2, m, MB, float(MBF))
    # and the pair path again after all that
    imL, imR = stereo_pair(11, 1241, 376)
    got = pkg.ExtractStereo(eL, eR, imL, imR, m, MB, float(MBF))
    want = oracle(imL, imR)
    assert np.array_equal(got[4], want[4]) and got[6] == want[6]


def test_stereo_frames_from_two_threads(pkg, O):
    """Two host threads each running orbm_stereo_frame on their own extractor
    pair and matcher (the library's one staging helper thread serves one call
    at a time; the other copies inline): every frame equals the same call made
    alone."""
    import threading

    from orb_slam_cuda_amd.synth import stereo_pair
    W, H = 1241, 376
    pairs = [stereo_pair(40 + i, W, H) for i in range(6)]
    ref = {}
    eL, eR, m = (pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H), pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H),
                 pkg.ORBmatcher(max_kps=4096))
    for i, (L, R) in enumerate(pairs):
        ref[i] = pkg.ExtractStereo(eL, eR, L, R, m, MB, float(MBF))
    errors = []

    def worker(t):
        try:
            a, b, mm = (pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H), pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H),
                        pkg.ORBmatcher(max_kps=4096))
            for rep in range(4):
                for i in range(t, len(pairs), 2):
                    got = pkg.ExtractStereo(a, b, pairs[i][0], pairs[i][1], mm, MB, float(MBF))
                    for g, w in zip(got[:6], ref[i][:6]):
                        if not np.array_equal(np.asarray(g).view(np.uint8), np.asarray(w).view(np.uint8)):
                            errors.append((t, rep, i))
                    if got[6] != ref[i][6]:
                        errors.append((t, rep, i, "kept"))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]
