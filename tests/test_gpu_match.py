"""GPU parity of the HIP matchers (liborbx.so) against the CPU oracle.

Inputs are the oracle's own keypoints/descriptors so that the matcher is
tested in isolation; outputs must be identical (match indices, counts,
updated vbPrevMatched)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu




def _pair(O, seed, W=1241, H=376, nf=2000):
    from orb_slam_cuda_amd.synth import SynthSequence
    fr = SynthSequence(seed, W, H).frames(2)
    cfg = O.config(nfeatures=nf, width=W, height=H)
    return O.extract(cfg, fr[0]), O.extract(cfg, fr[1])


@pytest.mark.parametrize("seed,ratio,ori,window", [(5, 0.9, True, 100), (6, 0.9, False, 100),
                                                   (7, 0.7, True, 50), (8, 0.9, True, 200)])
def test_search_for_initialization_parity(pkg, O, seed, ratio, ori, window):
    W, H = 1241, 376
    (k1, d1), (k2, d2) = _pair(O, seed)
    F1 = pkg.Frame.from_extraction(k1, d1, W, H)
    F2 = pkg.Frame.from_extraction(k2, d2, W, H)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    m = pkg.ORBmatcher(ratio, ori, max_kps=4096)
    v12 = []
    nm = m.SearchForInitialization(F1, F2, prev, v12, window)
    r12, rnm, rprev = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  window, ratio, ori)
    assert nm == rnm
    assert np.array_equal(np.array(v12, np.int32), r12)
    assert np.array_equal(prev, rprev)
    assert nm > 20
    # second round from the updated vbPrevMatched (as Tracking does on the next frame)
    nm2 = m.SearchForInitialization(F1, F2, prev, v12, window)
    r12b, rnm2, rprev2 = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), rprev, window, ratio, ori)
    assert nm2 == rnm2 and np.array_equal(np.array(v12, np.int32), r12b) and np.array_equal(prev, rprev2)


def test_search_for_initialization_golden(pkg, O):
    g = np.load(os.path.join(GOLDEN, "match_kitti_seq5.npz"))
    W, H = int(g["W"]), int(g["H"])
    (k1, d1), (k2, d2) = _pair(O, int(g["seed"]))
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    m = pkg.ORBmatcher(0.9, True, max_kps=4096)
    v12 = []
    nm = m.SearchForInitialization(pkg.Frame.from_extraction(k1, d1, W, H), pkg.Frame.from_extraction(k2, d2, W, H),
                                   prev, v12, 100)
    assert nm == int(g["nmatches"]) and np.array_equal(np.array(v12, np.int32), g["matches12"])
    assert np.array_equal(prev, g["prev_after"])


def test_search_for_initialization_edges(pkg, O):
    W, H = 1241, 376
    (k1, d1), (k2, d2) = _pair(O, 12)
    m = pkg.ORBmatcher(0.9, True, max_kps=4096)
    empty = np.zeros(0, pkg.KP_DTYPE)
    F1 = pkg.Frame.from_extraction(k1, d1, W, H)
    F0 = pkg.Frame.from_extraction(empty, np.zeros((0, 32), np.uint8), W, H)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    assert m.SearchForInitialization(F1, F0, prev, None, 100) == 0
    assert m.SearchForInitialization(F0, F1, np.zeros((0, 2), np.float32), None, 100) == 0
    # identical frames: every level-0 keypoint matches itself at distance 0 (unless a twin steals it)
    nm = m.SearchForInitialization(F1, F1, prev.copy(), None, 100)
    r12, rnm, _ = O.search_for_initialization(k1, d1, k1, d1, (0, W, 0, H), prev, 100, 0.9, True)
    assert nm == rnm and np.array_equal(m.last_matches12, r12)
    # windows hanging off the image (prev positions outside the grid)
    far = prev + np.float32(900)
    nm = m.SearchForInitialization(F1, F1, far.copy(), None, 100)
    r12, rnm, _ = O.search_for_initialization(k1, d1, k1, d1, (0, W, 0, H), far, 100, 0.9, True)
    assert nm == rnm and np.array_equal(m.last_matches12, r12)


def test_batch_search_init_with_null_prev(pkg, O):
    """The device-resident batch entry with prev=NULL (windows on F1's keypoints)."""
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    W, H = 1241, 376
    pairs = [_pair(O, s) for s in (40, 41, 42)]
    P, cap = len(pairs), 2100
    kp = np.zeros((2 * P, cap), pkg.KP_DTYPE)
    de = np.zeros((2 * P, cap, 32), np.uint8)
    n = np.zeros(2 * P, np.int32)
    for p, ((k1, d1), (k2, d2)) in enumerate(pairs):
        kp[p, :len(k1)], de[p, :len(k1)], n[p] = k1, d1, len(k1)
        kp[P + p, :len(k2)], de[P + p, :len(k2)], n[P + p] = k2, d2, len(k2)
    dk, dd, dn = (_lib.DeviceArray(a.nbytes) for a in (kp, de, n))
    dk.upload(kp), dd.upload(de), dn.upload(n)
    dm, dnm = _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * 4)
    m = pkg.ORBmatcher(0.9, True, max_pairs=P, max_kps=cap)
    L = _lib.lib()
    _lib.check(L.orbm_search_for_initialization_batch(
        m.handle, C.c_void_p(dk.ptr), C.c_void_p(dd.ptr), C.c_void_p(dn.ptr),
        C.c_void_p(dk.ptr + P * cap * 28), C.c_void_p(dd.ptr + P * cap * 32), C.c_void_p(dn.ptr + P * 4),
        cap, P, _lib.GridBounds(0, W, 0, H), None, 100, C.c_float(0.9), 1, C.c_void_p(dm.ptr),
        C.c_void_p(dnm.ptr), None), matcher=True)
    L.orbx_stream_synchronize(None)
    got = dm.download((P, cap), np.int32)
    gnm = dnm.download(P, np.int32)
    for p, ((k1, d1), (k2, d2)) in enumerate(pairs):
        r12, rnm, _ = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  100, 0.9, True)
        assert gnm[p] == rnm and np.array_equal(got[p, :len(k1)], r12)


def test_hamming_top2_parity(pkg, O):
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    D = np.load(os.path.join(GOLDEN, "mapyml_descriptors.npy"))
    rng = np.random.default_rng(3)
    sets = []
    for na, nb in ((775, 775), (2003, 1998), (1, 300), (300, 1), (0, 5)):
        A = D[rng.integers(0, 775, na)] if na else np.zeros((0, 32), np.uint8)
        B = np.concatenate([D[rng.integers(0, 775, nb // 2)], rng.integers(0, 256, (nb - nb // 2, 32),
                                                                             dtype=np.uint8)])
        sets.append((A, B))
    P, cap = len(sets), 2048
    A_ = np.zeros((P, cap, 32), np.uint8)
    B_ = np.zeros((P, cap, 32), np.uint8)
    nA = np.array([len(a) for a, _ in sets], np.int32)
    nB = np.array([len(b) for _, b in sets], np.int32)
    for p, (a, b) in enumerate(sets):
        A_[p, :len(a)], B_[p, :len(b)] = a, b
    dA, dB, dnA, dnB = (_lib.DeviceArray(x.nbytes) for x in (A_, B_, nA, nB))
    for d, x in ((dA, A_), (dB, B_), (dnA, nA), (dnB, nB)):
        d.upload(x)
    outs = [_lib.DeviceArray(P * cap * 4) for _ in range(3)]
    m = pkg.ORBmatcher(0.9, True, max_pairs=P, max_kps=cap)
    L = _lib.lib()
    _lib.check(L.orbm_hamming_top2(m.handle, C.c_void_p(dA.ptr), cap * 32, C.c_void_p(dnA.ptr), cap,
                                   C.c_void_p(dB.ptr), cap * 32, C.c_void_p(dnB.ptr), P,
                                   *(C.c_void_p(o.ptr) for o in outs), None), matcher=True)
    L.orbx_stream_synchronize(None)
    bi, bd, sd = (o.download((P, cap), np.int32) for o in outs)
    for p, (a, b) in enumerate(sets):
        ri, rd, rs = O.hamming_top2(a, b)
        assert np.array_equal(bi[p, :len(a)], ri) and np.array_equal(bd[p, :len(a)], rd)
        assert np.array_equal(sd[p, :len(a)], rs)


@pytest.mark.parametrize("kernel", ["mfma", "valu"])
@pytest.mark.parametrize("na,nb,dups", [(300, 40000, 0), (517, 3001, 1), (64, 33, 1), (2, 32769, 1)])
def test_hamming_top2_blocks_and_ties(pkg, O, na, nb, dups, kernel, monkeypatch):
    """Candidate counts past one 32768-index key block of the MFMA kernel, ragged
    tiles, and exact ties (duplicated candidate rows: the earlier index must win
    and the second distance equals the best); also distance-256 complements.
    Both kernels: the FP4 MFMA one (default) and the VALU one (ORBX_TOP2_VALU=1)."""
    import ctypes as C
    if kernel == "valu":
        monkeypatch.setenv("ORBX_TOP2_VALU", "1")
    else:
        monkeypatch.delenv("ORBX_TOP2_VALU", raising=False)

    from orb_slam_cuda_amd import _lib
    rng = np.random.default_rng(na * 7 + nb)
    A = rng.integers(0, 256, (na, 32), dtype=np.uint8)
    B = rng.integers(0, 256, (nb, 32), dtype=np.uint8)
    if dups:
        # near copies of the queries, each twice at scattered positions, plus exact complements
        for i in range(min(na, nb // 4)):
            a = A[i].copy()
            a[i % 32] ^= np.uint8(1 << (i % 8)) if i % 3 else np.uint8(0)
            B[rng.integers(0, nb)] = a
            B[rng.integers(0, nb)] = a
            B[rng.integers(0, nb)] = ~A[i]
    cap_a, cap_b = na, nb
    dA, dB = _lib.DeviceArray(A.nbytes), _lib.DeviceArray(B.nbytes)
    dA.upload(A)
    dB.upload(B)
    dnA, dnB = _lib.DeviceArray(4), _lib.DeviceArray(4)
    dnA.upload(np.array([na], np.int32))
    dnB.upload(np.array([nb], np.int32))
    outs = [_lib.DeviceArray(cap_a * 4) for _ in range(3)]
    m = pkg.ORBmatcher(0.9, True, max_pairs=1, max_kps=max(cap_a, cap_b))
    L = _lib.lib()
    _lib.check(L.orbm_hamming_top2(m.handle, C.c_void_p(dA.ptr), cap_a * 32, C.c_void_p(dnA.ptr), cap_a,
                                   C.c_void_p(dB.ptr), cap_b * 32, C.c_void_p(dnB.ptr), 1,
                                   *(C.c_void_p(o.ptr) for o in outs), None), matcher=True)
    L.orbx_stream_synchronize(None)
    bi, bd, sd = (o.download(cap_a, np.int32) for o in outs)
    ri, rd, rs = O.hamming_top2(A, B)
    assert np.array_equal(bd, rd) and np.array_equal(sd, rs)
    assert np.array_equal(bi, ri)


def _featvec(rng, n, nodes):
    node = rng.integers(0, nodes, size=n)
    ids = sorted(set(int(v) * 13 + 1 for v in node))
    lut = {v: [] for v in ids}
    for i, v in enumerate(node):
        lut[int(v) * 13 + 1].append(i)
    return {k: v for k, v in lut.items()}


@pytest.mark.parametrize("kf_vs_kf,nodes,ratio,ori", [(False, 40, 0.7, True), (False, 3, 0.75, True),
                                                      (True, 40, 0.75, True), (True, 200, 0.7, False)])
def test_search_by_bow_parity(pkg, O, kf_vs_kf, nodes, ratio, ori):
    from orb_slam_cuda_amd.matcher import feature_vector_csr
    (k1, d1), (k2, d2) = _pair(O, 50)
    rng = np.random.default_rng(nodes)
    fa, fb = _featvec(rng, len(d1), nodes), _featvec(rng, len(d2), nodes)
    mpA = (rng.random(len(d1)) > 0.3).astype(np.uint8)
    mpB = (rng.random(len(d2)) > 0.3).astype(np.uint8)
    KF = pkg.KeyFrame(k1, d1, mpA, fa)
    B = pkg.KeyFrame(k2, d2, mpB, fb) if kf_vs_kf else pkg.Frame.from_extraction(k2, d2, 1241, 376, fb)
    m = pkg.ORBmatcher(ratio, ori)
    out = []
    nm = m.SearchByBoW(KF, B, out)
    rout, rnm = O.search_by_bow(d1, k1["angle"], mpA, feature_vector_csr(fa), d2, k2["angle"],
                                mpB if kf_vs_kf else np.ones(len(d2), np.uint8), feature_vector_csr(fb),
                                ratio, ori, kf_vs_kf)
    assert nm == rnm and np.array_equal(np.array(out, np.int32), rout)
    assert nm > 5


def test_search_by_bow_golden(pkg, O):
    from orb_slam_cuda_amd.matcher import feature_vector_csr
    import importlib.util
    g = np.load(os.path.join(GOLDEN, "match_kitti_seq5.npz"))
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    (k1, d1), (k2, d2) = _pair(O, int(g["seed"]))
    fa, fb = mg.synthetic_featvec(d1, 1), mg.synthetic_featvec(d2, 1)
    to_dict = lambda csr: {int(n): csr[2][csr[1][k]:csr[1][k + 1]].tolist() for k, n in enumerate(csr[0])}
    mp = (np.arange(len(k1)) % 5 != 0).astype(np.uint8)
    m = pkg.ORBmatcher(0.7, True)
    out = []
    nm = m.SearchByBoW(pkg.KeyFrame(k1, d1, mp, to_dict(fa)), pkg.Frame.from_extraction(k2, d2, 1241, 376,
                                                                                      to_dict(fb)), out)
    assert nm == int(g["bow_nmatches"]) and np.array_equal(np.array(out, np.int32), g["bow_kf_f"])
    assert feature_vector_csr(to_dict(fa))[0].tolist() == fa[0].tolist()


def _kps(pkg, xs, ys, angles=None):
    k = np.zeros(len(xs), pkg.KP_DTYPE)
    k["x"], k["y"], k["size"], k["response"] = xs, ys, 31.0, 1.0
    k["angle"] = 0.0 if angles is None else angles
    return k


def _flip(rng, base, nbits):
    d = base.copy()
    for b in rng.choice(256, nbits, replace=False):
        d[b // 8] ^= np.uint8(1 << (b % 8))
    return d


@pytest.mark.parametrize("n", [20, 70])
def test_search_for_initialization_steal_chain(pkg, O, n):
    """A chain of greedy dependencies as long as the query list: query i (i>=1)
    sees targets t_i and t_i+1 at equal distance (ambiguous -> rejected) unless
    query i-1 took t_i, which it does only when query i-2 took t_i-1, and so
    on down to query 0, whose window holds t_1 alone. Resolution order matters
    at every link (the n=70 chain exceeds the parallel rounds' cap and runs
    the sequential path)."""
    W, H = 1241, 376
    rng = np.random.default_rng(3)
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    tdesc = _flip(rng, base, 30)
    tx = 20.0 + 16.0 * np.arange(n + 1)
    k2 = _kps(pkg, tx, np.full(n + 1, 100.0))
    qx = np.concatenate([[tx[1]], tx[1:n] + 8.0])
    k1 = _kps(pkg, qx, np.full(n, 100.0))
    d1 = np.repeat(base[None], n, 0)
    d2 = np.repeat(tdesc[None], n + 1, 0)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    m = pkg.ORBmatcher(0.9, True, max_kps=4096)
    v12 = []
    nm = m.SearchForInitialization(pkg.Frame.from_extraction(k1, d1, W, H), pkg.Frame.from_extraction(k2, d2, W, H),
                                   prev, v12, 12)
    r12, rnm, rprev = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  12, 0.9, True)
    assert rnm == n and np.array_equal(r12, np.arange(1, n + 1, dtype=np.int32))
    assert nm == rnm and np.array_equal(np.array(v12, np.int32), r12) and np.array_equal(prev, rprev)


@pytest.mark.parametrize("seed,ratio", [(0, 0.9), (1, 0.7), (2, 1.0)])
def test_search_for_initialization_contention(pkg, O, seed, ratio):
    """Heavy contention: 600 queries and 500 targets crowded into one window,
    descriptors a few bits from a common base, so most queries compete for
    the same targets and steals cascade."""
    W, H = 1241, 376
    rng = np.random.default_rng(100 + seed)
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    n1, n2 = 600, 500
    k1 = _kps(pkg, rng.uniform(300, 360, n1), rng.uniform(150, 210, n1), rng.uniform(0, 360, n1))
    k2 = _kps(pkg, rng.uniform(300, 360, n2), rng.uniform(150, 210, n2), rng.uniform(0, 360, n2))
    d1 = np.stack([_flip(rng, base, int(rng.integers(0, 20))) for _ in range(n1)])
    d2 = np.stack([_flip(rng, base, int(rng.integers(0, 20))) for _ in range(n2)])
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    for ori in (True, False):
        m = pkg.ORBmatcher(ratio, ori, max_kps=4096)
        p = prev.copy()
        v12 = []
        nm = m.SearchForInitialization(pkg.Frame.from_extraction(k1, d1, W, H),
                                       pkg.Frame.from_extraction(k2, d2, W, H), p, v12, 100)
        r12, rnm, rprev = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), prev, 100, ratio, ori)
        assert nm == rnm and np.array_equal(np.array(v12, np.int32), r12) and np.array_equal(p, rprev)


def test_search_for_initialization_dense_window_no_capacity_cliff(pkg, O):
    """2100 x 2100 level-0 keypoints in one window: 4.41 M candidate entries,
    more than the matcher's per-pair list area (min(max_kps^2, 4M)). The host
    entry point (the shim's path) grows its workspace and returns the
    reference's matches instead of ECAPACITY; the next call is exact too."""
    W, H = 1241, 376
    rng = np.random.default_rng(9)
    n = 2100
    k1 = _kps(pkg, rng.uniform(500, 560, n), rng.uniform(150, 210, n), rng.uniform(0, 360, n))
    k2 = _kps(pkg, rng.uniform(500, 560, n), rng.uniform(150, 210, n), rng.uniform(0, 360, n))
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    d1 = np.stack([_flip(rng, base, int(rng.integers(0, 40))) for _ in range(n)])
    d2 = np.stack([_flip(rng, base, int(rng.integers(0, 40))) for _ in range(n)])
    m = pkg.ORBmatcher(0.9, True, max_kps=n)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    v12 = []
    nm = m.SearchForInitialization(pkg.Frame.from_extraction(k1, d1, W, H), pkg.Frame.from_extraction(k2, d2, W, H),
                                   prev, v12, 100)
    r12, rnm, rprev = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  100, 0.9, True)
    assert nm == rnm and np.array_equal(np.array(v12, np.int32), r12) and np.array_equal(prev, rprev)
    (a1, e1), (a2, e2) = _pair(O, 5)
    prev = np.stack([a1["x"], a1["y"]], 1).astype(np.float32)
    v12 = []
    nm = m.SearchForInitialization(pkg.Frame.from_extraction(a1, e1, W, H), pkg.Frame.from_extraction(a2, e2, W, H),
                                   prev, v12, 100)
    r12, rnm, rprev = O.search_for_initialization(a1, e1, a2, e2, (0, W, 0, H), np.stack([a1["x"], a1["y"]], 1),
                                                  100, 0.9, True)
    assert nm == rnm and np.array_equal(np.array(v12, np.int32), r12) and np.array_equal(prev, rprev)


def test_search_for_initialization_shim_sized_matcher_dense_level0(pkg, O):
    """The shim's matcher (max_kps 8192, shim/src/ORBmatcher.cc) on frames of
    6000 keypoints whose 3000 octave-0 keypoints crowd a 150-px square: frames
    larger than the kernel's per-keypoint LDS tables and 9 M candidate entries.
    Octave-0 compaction on the host and the grown workspace give the oracle's
    matches12 / vbPrevMatched (non-octave-0 queries untouched)."""
    W, H = 1241, 376
    rng = np.random.default_rng(21)
    n, n0 = 6000, 3000

    def frame():
        oc = np.concatenate([np.zeros(n0, np.int32), rng.integers(1, 8, n - n0).astype(np.int32)])
        rng.shuffle(oc)
        x = np.where(oc == 0, rng.uniform(400, 550, n), rng.uniform(20, W - 20, n))
        y = np.where(oc == 0, rng.uniform(120, 270, n), rng.uniform(20, H - 20, n))
        k = _kps(pkg, x, y, rng.uniform(0, 360, n))
        k["octave"] = oc
        return k

    k1, k2 = frame(), frame()
    # F2's descriptors: a few bits from a random F1 descriptor (repeats give steals)
    d1 = rng.integers(0, 256, (n, 32), np.uint8)
    src = rng.integers(0, n, n)
    d2 = np.stack([_flip(rng, d1[j], int(rng.integers(0, 12))) for j in src])
    prev0 = np.stack([k1["x"] + 3.0, k1["y"] - 2.0], 1).astype(np.float32)
    m = pkg.ORBmatcher(0.9, True, max_kps=8192)
    prev = prev0.copy()
    v12 = []
    nm = m.SearchForInitialization(pkg.Frame.from_extraction(k1, d1, W, H), pkg.Frame.from_extraction(k2, d2, W, H),
                                   prev, v12, 100)
    r12, rnm, rprev = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), prev0, 100, 0.9, True)
    assert rnm > 20
    assert nm == rnm and np.array_equal(np.array(v12, np.int32), r12) and np.array_equal(prev, rprev)


def test_batch_search_init_dense_pair(pkg, O):
    """The device batch entry with a dense pair (2100 x 2100 level-0 keypoints
    in one window, 4.4 M window candidates) beside a KITTI pair: both exact (no
    candidate lists are kept, so no workspace bound applies), status clean."""
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    W, H = 1241, 376
    rng = np.random.default_rng(9)
    cap = 2100
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    dense = [(_kps(pkg, rng.uniform(500, 560, cap), rng.uniform(150, 210, cap), rng.uniform(0, 360, cap)),
              np.stack([_flip(rng, base, int(rng.integers(0, 40))) for _ in range(cap)])) for _ in range(2)]
    pairs = [_pair(O, 40), (dense[0], dense[1])]
    P = len(pairs)
    kp = np.zeros((2 * P, cap), pkg.KP_DTYPE)
    de = np.zeros((2 * P, cap, 32), np.uint8)
    n = np.zeros(2 * P, np.int32)
    for p, ((k1, d1), (k2, d2)) in enumerate(pairs):
        kp[p, :len(k1)], de[p, :len(k1)], n[p] = k1, d1, len(k1)
        kp[P + p, :len(k2)], de[P + p, :len(k2)], n[P + p] = k2, d2, len(k2)
    dk, dd, dn = (_lib.DeviceArray(a.nbytes) for a in (kp, de, n))
    dk.upload(kp), dd.upload(de), dn.upload(n)
    dm, dnm = _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * 4)
    m = pkg.ORBmatcher(0.9, True, max_pairs=P, max_kps=cap)
    L = _lib.lib()
    _lib.check(L.orbm_search_for_initialization_batch(
        m.handle, C.c_void_p(dk.ptr), C.c_void_p(dd.ptr), C.c_void_p(dn.ptr),
        C.c_void_p(dk.ptr + P * cap * 28), C.c_void_p(dd.ptr + P * cap * 32), C.c_void_p(dn.ptr + P * 4),
        cap, P, _lib.GridBounds(0, W, 0, H), None, 100, C.c_float(0.9), 1, C.c_void_p(dm.ptr),
        C.c_void_p(dnm.ptr), None), matcher=True)
    L.orbx_stream_synchronize(None)
    got = dm.download((P, cap), np.int32)
    gnm = dnm.download(P, np.int32)
    assert m.status() == 0
    for p, ((k1, d1), (k2, d2)) in enumerate(pairs):
        r12, rnm, _ = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  100, 0.9, True)
        assert gnm[p] == rnm and np.array_equal(got[p, :len(k1)], r12), p


@pytest.mark.parametrize("cap,ratio", [(2101, 0.9), (2099, 0.7), (1999, 0.75)])
def test_batch_search_init_odd_pitch(pkg, O, cap, ratio):
    """Odd keypoint pitches (the per-pair workspace's key table
    must stay 16-byte aligned whatever the pitch; its int tables are padded to
    4 ints) at three ratios (6-, 7- and 7-bit distance clamps): exact against
    the oracle, status clean."""
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    W, H = 1241, 376
    pairs = [_pair(O, 40), _pair(O, 41), _pair(O, 42)]
    P = len(pairs)
    kp = np.zeros((2 * P, cap), pkg.KP_DTYPE)
    de = np.zeros((2 * P, cap, 32), np.uint8)
    n = np.zeros(2 * P, np.int32)
    for p, ((k1, d1), (k2, d2)) in enumerate(pairs):
        k1, d1, k2, d2 = k1[:cap], d1[:cap], k2[:cap], d2[:cap]
        kp[p, :len(k1)], de[p, :len(k1)], n[p] = k1, d1, len(k1)
        kp[P + p, :len(k2)], de[P + p, :len(k2)], n[P + p] = k2, d2, len(k2)
    dk, dd, dn = (_lib.DeviceArray(a.nbytes) for a in (kp, de, n))
    dk.upload(kp), dd.upload(de), dn.upload(n)
    dm, dnm = _lib.DeviceArray(P * cap * 4), _lib.DeviceArray(P * 4)
    m = pkg.ORBmatcher(ratio, True, max_pairs=P, max_kps=cap)
    L = _lib.lib()
    _lib.check(L.orbm_search_for_initialization_batch(
        m.handle, C.c_void_p(dk.ptr), C.c_void_p(dd.ptr), C.c_void_p(dn.ptr),
        C.c_void_p(dk.ptr + P * cap * 28), C.c_void_p(dd.ptr + P * cap * 32), C.c_void_p(dn.ptr + P * 4),
        cap, P, _lib.GridBounds(0, W, 0, H), None, 100, C.c_float(ratio), 1, C.c_void_p(dm.ptr),
        C.c_void_p(dnm.ptr), None), matcher=True)
    L.orbx_stream_synchronize(None)
    got = dm.download((P, cap), np.int32)
    gnm = dnm.download(P, np.int32)
    assert m.status() == 0
    for p in range(P):
        k1, d1, k2, d2 = kp[p, :n[p]], de[p, :n[p]], kp[P + p, :n[P + p]], de[P + p, :n[P + p]]
        r12, rnm, _ = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  100, ratio, True)
        assert gnm[p] == rnm and np.array_equal(got[p, :len(k1)], r12), p


def test_search_init_capacity_message_names_the_bound(pkg):
    """ECAPACITY at a pitch past 2^(20 - dbits): the message names the bound of
    the call's ratio, 8192 at 0.7."""
    import ctypes as C

    from orb_slam_cuda_amd import _lib
    cap = 8200
    m = pkg.ORBmatcher(0.7, True, max_pairs=1, max_kps=cap)
    L = _lib.lib()
    d = _lib.DeviceArray(cap * 32 * 2 + 64)
    rc = L.orbm_search_for_initialization_batch(
        m.handle, C.c_void_p(d.ptr), C.c_void_p(d.ptr), C.c_void_p(d.ptr), C.c_void_p(d.ptr), C.c_void_p(d.ptr),
        C.c_void_p(d.ptr), cap, 1, _lib.GridBounds(0, 1241, 0, 376), None, 100, C.c_float(0.7), 1,
        C.c_void_p(d.ptr), C.c_void_p(d.ptr), None)
    assert rc == _lib.ORBX_ECAPACITY
    assert b"8192" in L.orbm_last_error()
