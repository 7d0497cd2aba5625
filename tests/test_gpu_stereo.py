"""GPU parity of Frame::ComputeStereoMatches (liborbx.so, orbx_stereo.hip) against
the CPU oracle (oracle/orb_oracle.cpp, itself cross-checked against tests/refpy.py
in test_oracle.py). Outputs mvuRight / mvDepth and the kept count must be
bit-identical."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MB, MBF = 0.54, np.float32(0.54 * 718.856)


def _oracle(O, cfg, imL, imR, kL, dL, kR, dR, mb=MB, mbf=MBF):
    li = O.level_info(cfg)
    return O.compute_stereo_matches(kL, dL, kR, dR, O.pyramid(cfg, imL), O.pyramid(cfg, imR), li["scale"],
                                    li["inv_scale"], mb, mbf)


@pytest.mark.parametrize("seed,W,H,nf", [(3, 1241, 376, 2000), (4, 1241, 376, 2000), (9, 752, 480, 1200),
                                         (12, 640, 240, 500)])
def test_stereo_matches_parity(pkg, O, seed, W, H, nf):
    from orb_slam_cuda_amd.synth import stereo_pair
    imL, imR = stereo_pair(seed, W, H)
    eL = pkg.ORBextractor(nf, 1.2, 8, 20, 7, W, H)
    eR = pkg.ORBextractor(nf, 1.2, 8, 20, 7, W, H)
    kL, dL = eL(imL)
    kR, dR = eR(imR)
    m = pkg.ORBmatcher(max_kps=4096)
    F = pkg.Frame.from_extraction(kL, dL, W, H)
    F.mvKeysRight, F.mDescriptorsRight, F.mb, F.mbf = kR, dR, MB, float(MBF)
    kept = pkg.ComputeStereoMatches(F, eL, eR, m)
    cfg = O.config(nfeatures=nf, width=W, height=H)
    uR, dep, ekept = _oracle(O, cfg, imL, imR, kL, dL, kR, dR)
    assert kept == ekept and kept > 0.3 * len(kL)
    assert np.array_equal(F.mvuRight, uR)
    assert np.array_equal(F.mvDepth, dep)


def test_stereo_matches_edges(pkg, O):
    from orb_slam_cuda_amd.synth import stereo_pair
    W, H = 640, 240
    imL, imR = stereo_pair(5, W, H)
    eL = pkg.ORBextractor(500, 1.2, 8, 20, 7, W, H)
    eR = pkg.ORBextractor(500, 1.2, 8, 20, 7, W, H)
    kL, dL = eL(imL)
    kR, dR = eR(imR)
    m = pkg.ORBmatcher(max_kps=4096)
    cfg = O.config(nfeatures=500, width=W, height=H)

    def run(kl, dl, kr, dr, mb=MB, mbf=MBF):
        F = pkg.Frame.from_extraction(kl, dl, W, H)
        F.mvKeysRight, F.mDescriptorsRight, F.mb, F.mbf = kr, dr, mb, float(mbf)
        k = pkg.ComputeStereoMatches(F, eL, eR, m)
        return F.mvuRight, F.mvDepth, k

    # no right keypoints: nothing matched
    u, d, k = run(kL, dL, kR[:0], dR[:0])
    assert k == 0 and (u == -1).all() and (d == -1).all()
    # no left keypoints
    u, d, k = run(kL[:0], dL[:0], kR, dR)
    assert k == 0 and len(u) == 0
    # duplicated right keypoints: ties go to the lowest index
    kR2, dR2 = np.concatenate([kR, kR]), np.concatenate([dR, dR])
    u, d, k = run(kL, dL, kR2, dR2)
    eu, ed, ek = _oracle(O, cfg, imL, imR, kL, dL, kR2, dR2)
    assert k == ek and np.array_equal(u, eu) and np.array_equal(d, ed)
    # a short baseline (narrow disparity range) and a long one
    for mb, mbf in ((0.05, np.float32(0.05 * 400)), (1.5, np.float32(1.5 * 900))):
        u, d, k = run(kL, dL, kR, dR, mb, mbf)
        eu, ed, ek = _oracle(O, cfg, imL, imR, kL, dL, kR, dR, mb, mbf)
        assert k == ek and np.array_equal(u, eu) and np.array_equal(d, ed)


def test_stereo_matches_batch(pkg, O):
    """Left and right frames extracted in ONE batch (left = frames 0..P-1, right =
    P..2P-1) and matched pairwise on the device."""
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import stereo_pair
    W, H, P = 1241, 376, 6
    pairs = [stereo_pair(40 + i, W, H) for i in range(P)]
    frames = np.ascontiguousarray(np.stack([p[0] for p in pairs] + [p[1] for p in pairs]))
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=2 * P)
    cap = ext.frame_capacity
    d_in = _lib.DeviceArray(frames.nbytes)
    d_in.upload(frames)
    d_kp, d_desc, d_n = _lib.DeviceArray(2 * P * cap * 28), _lib.DeviceArray(2 * P * cap * 32), _lib.DeviceArray(8 * P)
    s = _lib.Stream()
    ext.extract_batch_device(d_in.ptr, 2 * P, H * W, W, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
    m = pkg.ORBmatcher(max_pairs=P, max_kps=cap)
    d_u, d_d, d_k = _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * 4)
    kpb, db = P * cap * 28, P * cap * 32
    _lib.check(_lib.lib().orbm_compute_stereo_matches_batch(
        m.handle, ext.handle, 0, ext.handle, P, C.c_void_p(d_kp.ptr), C.c_void_p(d_desc.ptr),
        C.c_void_p(d_n.ptr), C.c_void_p(d_kp.ptr + kpb), C.c_void_p(d_desc.ptr + db), C.c_void_p(d_n.ptr + 4 * P),
        cap, P, C.c_float(MB), C.c_float(MBF), C.c_void_p(d_u.ptr), C.c_void_p(d_d.ptr), C.c_void_p(d_k.ptr), s.s),
        matcher=True)
    s.synchronize()
    n = d_n.download(2 * P, np.int32)
    kps = d_kp.download(2 * P * cap, pkg.KP_DTYPE).reshape(2 * P, cap)
    desc = d_desc.download((2 * P, cap, 32), np.uint8)
    u = d_u.download(P * cap, np.float32).reshape(P, cap)
    d = d_d.download(P * cap, np.float32).reshape(P, cap)
    kept = d_k.download(P, np.int32)
    cfg = O.config(nfeatures=2000, width=W, height=H)
    for i in range(P):
        nl, nr = n[i], n[P + i]
        eu, ed, ek = _oracle(O, cfg, pairs[i][0], pairs[i][1], kps[i, :nl], desc[i, :nl], kps[P + i, :nr],
                             desc[P + i, :nr])
        assert kept[i] == ek > 0
        assert np.array_equal(u[i, :nl], eu) and np.array_equal(d[i, :nl], ed)
