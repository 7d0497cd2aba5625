"""GPU checks of the runtime contract around the kernels: the quadtree
tie-rule counter against the oracle's, the device status words, handle-size
independence of the LDS limits, and the stream order of shared workspaces.
All calls go through the C ABI."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MB, MBF = 0.54, np.float32(0.54 * 718.856)


@pytest.mark.parametrize("seed,W,H,nf", [(0, 1241, 376, 2000), (3, 752, 480, 1000), (11, 1241, 376, 4000)])
def test_tie_stats_match_oracle(pkg, O, seed, W, H, nf):
    from orb_slam_cuda_amd.synth import synth_frame
    img = synth_frame(seed, W, H)
    ext = pkg.ORBextractor(nf, 1.2, 8, 20, 7, W, H)
    ext(img)
    t = ext.tie_stats(0, 1)[0]
    r = O.tie_stats(O.config(nfeatures=nf, width=W, height=H), img)
    assert np.array_equal(t[:, 0], r["events"]), (t, r)
    assert np.array_equal(t[:, 1], r["nodes"]), (t, r)
    assert np.array_equal(t[:, 2], r["kps"]), (t, r)
    assert ext.status() == 0


def test_tie_stats_batch(pkg, O):
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H, B = 1241, 376, 6
    frames = np.ascontiguousarray(SynthSequence(77, W, H).frames(B))
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=B)
    cap = ext.frame_capacity
    d_in = _lib.DeviceArray(frames.nbytes)
    d_in.upload(frames)
    d_kp, d_desc, d_n = _lib.DeviceArray(B * cap * 28), _lib.DeviceArray(B * cap * 32), _lib.DeviceArray(4 * B)
    s = _lib.Stream()
    ext.extract_batch_device(d_in.ptr, B, H * W, W, d_kp.ptr, d_desc.ptr, d_n.ptr, s)
    s.synchronize()
    t = ext.tie_stats(0, B)
    cfg = O.config(nfeatures=2000, width=W, height=H)
    for i in range(B):
        r = O.tie_stats(cfg, frames[i])
        assert np.array_equal(t[i], np.stack([r["events"], r["nodes"], r["kps"]], 1)), i
    assert ext.status() == 0


def test_small_handle_does_not_shrink_lds_limit(pkg, O):
    """A handle with a small plan created after a large one must not lower the
    per-kernel LDS limit the large one launches with."""
    from orb_slam_cuda_amd.synth import synth_frame
    W, H = 1241, 376
    big = pkg.ORBextractor(4000, 1.2, 8, 20, 7, W, H)
    small = pkg.ORBextractor(100, 1.2, 8, 20, 7, 320, 240)
    small(synth_frame(2, 320, 240))
    img = synth_frame(4, W, H)
    kp, desc = big(img)
    rkp, rdesc = O.extract(O.config(nfeatures=4000, width=W, height=H), img)
    assert np.array_equal(kp.view(np.uint8), rkp.view(np.uint8)) and np.array_equal(desc, rdesc)


def test_hamming_top2_status_on_rows_past_cap(pkg, O):
    """nA > a_cap: the rows past a_cap have no output slot; the kernel searches
    only the first a_cap, writes nothing past its pair's rows, and reports
    status bit 16 (it used to clamp silently)."""
    from orb_slam_cuda_amd import _lib
    rng = np.random.default_rng(5)
    cap, P = 64, 2
    A = rng.integers(0, 256, (P, 100, 32), np.uint8)
    Bd = rng.integers(0, 256, (P, 90, 32), np.uint8)
    m = pkg.ORBmatcher(max_pairs=P, max_kps=128)
    d_A, d_B = _lib.DeviceArray(A.nbytes), _lib.DeviceArray(Bd.nbytes)
    d_A.upload(A)
    d_B.upload(Bd)
    nA = np.array([100, 40], np.int32)
    nB = np.array([90, 90], np.int32)
    d_nA, d_nB = _lib.DeviceArray(8), _lib.DeviceArray(8)
    d_nA.upload(nA)
    d_nB.upload(nB)
    sentinel = np.full(P * cap + 16, -7, np.int32)
    outs = [_lib.DeviceArray(sentinel.nbytes) for _ in range(3)]
    for o in outs:
        o.upload(sentinel)
    assert m.status() == 0
    _lib.check(_lib.lib().orbm_hamming_top2(m.handle, C.c_void_p(d_A.ptr), 100 * 32, C.c_void_p(d_nA.ptr), cap,
                                            C.c_void_p(d_B.ptr), 90 * 32, C.c_void_p(d_nB.ptr), P,
                                            *(C.c_void_p(o.ptr) for o in outs), None), matcher=True)
    bi = outs[0].download(P * cap + 16, np.int32)
    assert (bi[P * cap:] == -7).all()          # nothing past the last pair
    assert (bi[cap + 40:2 * cap] == -7).all()  # pair 1 wrote only its 40 rows
    for p, n in ((0, cap), (1, 40)):
        ri, rd, _ = O.hamming_top2(A[p, :n], Bd[p])
        assert np.array_equal(bi[p * cap:p * cap + n], ri)
    assert m.status() == 16
    assert m.status() == 0  # reset by the first read


def test_stereo_batches_on_two_streams_share_one_matcher(pkg, O):
    """Two stereo batches issued back to back on different streams through ONE
    matcher (its SAD scratch is shared): the library orders them, so both
    results equal the oracle's (the second batch's match kernel
    used to overwrite the first's SADs before its median pass read them)."""
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import stereo_pair
    W, H, P = 1241, 376, 4
    m = pkg.ORBmatcher(max_pairs=P, max_kps=4096)
    cfg = O.config(nfeatures=2000, width=W, height=H)
    runs = []
    for r in range(2):
        pairs = [stereo_pair(60 + 10 * r + i, W, H) for i in range(P)]
        frames = np.ascontiguousarray(np.stack([p[0] for p in pairs] + [p[1] for p in pairs]))
        ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=2 * P)
        cap = ext.frame_capacity
        d_in = _lib.DeviceArray(frames.nbytes)
        d_in.upload(frames)
        bufs = dict(kp=_lib.DeviceArray(2 * P * cap * 28), desc=_lib.DeviceArray(2 * P * cap * 32),
                    n=_lib.DeviceArray(8 * P), u=_lib.DeviceArray(P * cap * 4), d=_lib.DeviceArray(P * cap * 4),
                    k=_lib.DeviceArray(P * 4))
        runs.append(dict(pairs=pairs, ext=ext, cap=cap, d_in=d_in, s=_lib.Stream(), **bufs))
    for R in runs:  # extract both first, then issue both stereo batches without host syncs
        R["ext"].extract_batch_device(R["d_in"].ptr, 2 * P, H * W, W, R["kp"].ptr, R["desc"].ptr, R["n"].ptr, R["s"])
    for R in runs:
        cap = R["cap"]
        kpb, db = P * cap * 28, P * cap * 32
        _lib.check(_lib.lib().orbm_compute_stereo_matches_batch(
            m.handle, R["ext"].handle, 0, R["ext"].handle, P, C.c_void_p(R["kp"].ptr), C.c_void_p(R["desc"].ptr),
            C.c_void_p(R["n"].ptr), C.c_void_p(R["kp"].ptr + kpb), C.c_void_p(R["desc"].ptr + db),
            C.c_void_p(R["n"].ptr + 4 * P), cap, P, C.c_float(MB), C.c_float(MBF), C.c_void_p(R["u"].ptr),
            C.c_void_p(R["d"].ptr), C.c_void_p(R["k"].ptr), R["s"].s), matcher=True)
    for R in runs:
        R["s"].synchronize()
    for R in runs:
        cap = R["cap"]
        n = R["n"].download(2 * P, np.int32)
        kps = R["kp"].download(2 * P * cap, pkg.KP_DTYPE).reshape(2 * P, cap)
        desc = R["desc"].download((2 * P, cap, 32), np.uint8)
        u = R["u"].download(P * cap, np.float32).reshape(P, cap)
        kept = R["k"].download(P, np.int32)
        for i in range(P):
            nl, nr = n[i], n[P + i]
            ru, rd, rk = O.compute_stereo_matches(
                kps[i, :nl], desc[i, :nl], kps[P + i, :nr], desc[P + i, :nr],
                O.pyramid(cfg, R["pairs"][i][0]), O.pyramid(cfg, R["pairs"][i][1]),
                O.level_info(cfg)["scale"], O.level_info(cfg)["inv_scale"], MB, MBF)
            assert kept[i] == rk and np.array_equal(u[i, :nl], ru)


def test_stage_order_per_handle(pkg, O):
    """orbx_set_stage_order: every valid launch order gives the oracle's output
    (single-frame calls re-capture their graph with the new order, batch calls
    launch in it); an invalid order is refused and leaves the handle's order."""
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence
    W, H = 1241, 376
    frames = SynthSequence(7, W, H).frames(2)
    cfg = O.config(nfeatures=2000, width=W, height=H)
    want = [O.extract(cfg, f) for f in frames]
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H, max_batch=2)
    pitch = (W + 63) & ~63
    d = _lib.DeviceArray(2 * H * pitch)
    img = np.zeros((2, H, pitch), np.uint8)
    img[:, :, :W] = frames
    d.upload(img)
    cap = ext.frame_capacity
    dk, dd, dc = _lib.DeviceArray(2 * cap * 28), _lib.DeviceArray(2 * cap * 32), _lib.DeviceArray(16)
    for order in ("pbfqo", "pfbqo", "pfqbo"):
        ext.set_stage_order(order)
        assert "".join("f" if s == "fast_grid" else s[0] for s in ext.stage_order()) == order
        for _ in range(2):  # plain launches, then the captured graph
            for f, (wk, wd) in zip(frames, want):
                k, dsc = ext(f)
                assert np.array_equal(k.view(np.uint8), wk.view(np.uint8)) and np.array_equal(dsc, wd), order
        ext.extract_batch_device(d.ptr, 2, H * pitch, pitch, dk.ptr, dd.ptr, dc.ptr)
        n = dc.download(2, np.int32)
        kb = dk.download(2 * cap * 28, np.uint8).reshape(2, cap, 28)
        for i, (wk, wd) in enumerate(want):
            assert n[i] == len(wk) and np.array_equal(kb[i, :n[i]].reshape(-1), wk.view(np.uint8).reshape(-1)), order
    for bad in ("pqfbo", "bpfqo", "pfqob", "pfq", "pfqbx", ""):
        with pytest.raises(pkg.OrbxError):
            ext.set_stage_order(bad)
    assert ext.stage_order()[1] == "fast_grid"  # still "pfqbo"
    st = C.c_int(0)
    assert _lib.lib().orbx_get_status(ext.handle, 1, C.byref(st)) == 0 and st.value == 0
