"""CPU checks of the C-ABI library: it loads, exports every declared symbol,
matches the header's struct layouts, and fails loudly without a GPU."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_function():
    import orb_slam_cuda_amd as pkg
    L = pkg.lib()
    names = pkg.header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_so_is_gfx950_code_object():
    so = os.path.join(ROOT, "orb_slam_cuda_amd", "liborbx.so")
    blob = open(so, "rb").read()
    # the .hip_fatbin bundle names its device code object by target triple
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_struct_layouts_match_header():
    from orb_slam_cuda_amd._lib import KP_DTYPE, GridBounds, OrbxConfig
    assert KP_DTYPE.itemsize == 28  # cv::KeyPoint
    assert C.sizeof(OrbxConfig) == 16 * 4
    assert C.sizeof(GridBounds) == 16
    hdr = open(os.path.join(ROOT, "include", "orbx_c.h")).read()
    body = re.search(r"typedef struct orbx_config \{(.*?)\} orbx_config;", hdr, re.S).group(1)
    ints = sum(int(n) if n else 1 for n in re.findall(r"(?:int|float)\s+[a-z_, ]+?(?:\[(\d+)\])?;", body))
    assert ints >= 12


def test_descriptor_distance_is_host_exact():
    import numpy as np

    import orb_slam_cuda_amd as pkg
    D = np.load(os.path.join(ROOT, "tests", "golden", "mapyml_descriptors.npy"))
    for i in range(0, 775, 37):
        j = (i * 7 + 3) % 775
        assert pkg.ORBmatcher.DescriptorDistance(D[i], D[j]) == int(np.unpackbits(D[i] ^ D[j]).sum())


def test_stage_order_is_a_valid_launch_order():
    """orbx_get_stage_order (host only): the five stages once each, the
    pyramid first, FAST before the quadtree, orient+BRIEF last (after the blur
    and the quadtree it reads); the default is pyramid, FAST, quadtree, blur."""
    from orb_slam_cuda_amd import _lib
    order = _lib.stage_order()
    assert sorted(order) == sorted(["pyramid", "blur", "fast_grid", "quadtree", "orient_brief"])
    assert order[0] == "pyramid" and order[-1] == "orient_brief"
    assert order.index("fast_grid") < order.index("quadtree")
    if "ORBX_EXTRACT_ORDER" not in os.environ:
        assert order == ["pyramid", "fast_grid", "quadtree", "blur", "orient_brief"]


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="only meaningful without a GPU")
def test_no_gpu_fails_loudly():
    import orb_slam_cuda_amd as pkg
    with pytest.raises(pkg.OrbxError):
        pkg.ORBextractor(2000, 1.2, 8, 20, 7, 1241, 376)
    with pytest.raises(pkg.OrbxError):
        pkg.ORBmatcher(0.9, True)


def test_descriptor_sincosf_matches_host_libm():
    """The kernels' sin/cos of the descriptor rotation (glibc sinf/cosf
    restated, csrc/orbx_sincosf.h) against this host's libm on 2M samples of
    [0, 2pi) plus the quadrant edges. (tools/check_sincosf.cpp runs all
    1,086,918,619 floats of [0, 2pi): 0 mismatches.)"""
    import numpy as np

    import orb_slam_cuda_amd as pkg
    from oracle import oracle as O
    rng = np.random.default_rng(11)
    x = rng.uniform(0, 2 * np.pi, 2_000_000).astype(np.float32)
    edges = np.float32(np.pi / 4) * np.arange(0, 9, dtype=np.float32)
    near = np.concatenate([np.nextafter(edges, np.float32(-1)), edges, np.nextafter(edges, np.float32(9))])
    x = np.concatenate([x, near[near >= 0], np.float32([0.0, 0.75, 2.0 ** -12, 6.2831855])]).astype(np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    from orb_slam_cuda_amd._lib import check
    check(pkg.lib().orbx_sincosf_glibc(x.ctypes.data, len(x), s.ctypes.data, c.ctypes.data))
    rs, rc = O.sincosf(x)
    assert np.array_equal(s.view(np.uint32), rs.view(np.uint32))
    assert np.array_equal(c.view(np.uint32), rc.view(np.uint32))


def test_predict_scale_thresholds_match_logf():
    """MapPoint::PredictScale (src/MapPoint.cc:407-422) as the pose-projection kernels
    evaluate it (thresholds on mfMaxDistance/dist found with the host logf) equals the
    oracle's direct ceil(logf(ratio)/logf(sf)) on every float within 2^15 ulps of each
    threshold, on a wide random sample and on the special values."""
    import ctypes as C

    from oracle import oracle as O
    from orb_slam_cuda_amd import _lib
    for sf, L in [(1.2, 8), (1.2, 12), (1.5, 5), (2.0, 4)]:
        thr = np.zeros(16, np.float32)
        _lib.check(_lib.lib().orbm_predict_scale_thresholds(C.c_float(sf), L, thr.ctypes.data_as(C.c_void_p)))
        t = thr[:L - 1]
        assert np.all(np.diff(t) > 0)
        bits = t.view(np.uint32).astype(np.int64)
        near = (bits[:, None] + np.arange(-(1 << 15), 1 << 15)[None, :]).reshape(-1).astype(np.uint32).view(np.float32)
        rng = np.random.default_rng(L)
        wide = np.exp(rng.uniform(-12, 12, 200000)).astype(np.float32)
        special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, 3.4e38, -1.0, 1.0], np.float32)
        r = np.concatenate([near, wide, special])
        with np.errstate(invalid="ignore"):
            lvl = np.where(np.isinf(r), 0, (r[:, None] >= t[None, :]).sum(1))
        assert np.array_equal(lvl, O.predict_scale_ratios(r, sf, L)), (sf, L)


def test_prepare_pose_level_mode():
    """orbm_prepare_pose: bForward / bBackward of the motion-model search (src/ORBmatcher.cc:1338-1349)
    and the Sim3 decomposition (:298-304)."""
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    T = np.eye(4, dtype=np.float32)[:3]
    cam = _lib.camera(700, 700, 600, 180, 0.5, 350, T)
    for dz, mono, want in [(1.0, 0, 1), (-1.0, 0, 2), (0.2, 0, 0), (1.0, 1, 0)]:
        Tl = T.copy()
        Tl[2, 3] = dz
        p = _lib.OrbmPose()
        _lib.check(_lib.lib().orbm_prepare_pose(_lib.ORBM_PROJ_LAST_FRAME, C.byref(cam),
                                                Tl.ctypes.data_as(C.c_void_p), mono, C.byref(p)), matcher=True)
        assert p.level_mode == want
    S = T.copy() * 2.0
    p = _lib.OrbmPose()
    _lib.check(_lib.lib().orbm_prepare_pose(_lib.ORBM_PROJ_SIM3, C.byref(_lib.camera(700, 700, 600, 180, 0.5, 350, S)),
                                            None, 0, C.byref(p)), matcher=True)
    assert np.allclose(np.array(p.Rt).reshape(3, 4), T)


def test_fast_frame_index_magic_is_exact():
    """FAST's frame index (orbx_fast.hip) is mulhi(id, m) with m = ceil(2^32 / d),
    d = cells per frame, which orbx_host.hip enables only while
    d * B * (m * d - 2^32) < 2^32. Checked here at the worst ids (the last
    id of each frame, where the remainder is d - 1) for every d the planner can
    produce and the largest B that passes the check, plus a random sample."""
    import numpy as np
    rng = np.random.default_rng(7)
    for d in list(range(2, 5001)) + [8191, 12000, 40000]:
        m = ((1 << 32) + d - 1) // d
        e = m * d - (1 << 32)
        bmax = ((1 << 32) - 1) // (d * e) if e else 1 << 20
        bmax = min(bmax, 1 << 14)
        if bmax < 1:
            continue
        ids = [(q + 1) * d - 1 for q in range(0, bmax, max(1, bmax // 64))] + [d * bmax - 1]
        ids += [int(x) for x in rng.integers(0, d * bmax, 16)]
        for i in ids:
            assert (i * m) >> 32 == i // d, (d, bmax, i)


def test_brief_cvround_by_magic_add():
    """orient_brief_kernel rounds a test coordinate with fl(v + 1.5 * 2^23) and
    reads the integer from the sum's bit pattern; the reference's cvRound is
    round-half-even (lrint). Checked in float32 for every coordinate the
    kernels form: fl(fl(x*b) + fl(y*a)) and fl(fl(x*a) - fl(y*b)) over all
    512 pattern points (both tables) and 20,000 random (a, b) = (cos, sin)
    pairs, plus every quarter-integer in [-40, 40]."""
    import numpy as np
    from orb_slam_cuda_amd import _lib
    pts = []
    for mode in (0, 1):
        arr = (C.c_int * 1024)()
        assert _lib.lib().orbx_get_pattern(mode, arr) == 0
        t = np.frombuffer(arr, dtype=np.int32).reshape(256, 4)
        pts.append(t[:, 0:2])
        pts.append(t[:, 2:4])
    p = np.unique(np.concatenate(pts).astype(np.float32), axis=0)
    x, y = p[:, 0:1], p[:, 1:2]
    rng = np.random.default_rng(3)
    ang = rng.uniform(0, 2 * np.pi, 20000).astype(np.float32)
    a, b = np.cos(ang).astype(np.float32)[None, :], np.sin(ang).astype(np.float32)[None, :]
    vy = (x * b).astype(np.float32) + (y * a).astype(np.float32)
    vx = (x * a).astype(np.float32) - (y * b).astype(np.float32)
    q = np.arange(-160, 161, dtype=np.float32) / np.float32(4)
    for v in (vy.ravel(), vx.ravel(), q):
        v = v.astype(np.float32)
        s = (v + np.float32(12582912.0)).astype(np.float32)
        got = s.view(np.int32).astype(np.int64) - 0x4B400000
        assert np.array_equal(got, np.rint(v).astype(np.int64))
