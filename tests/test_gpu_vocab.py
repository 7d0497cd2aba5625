"""GPU parity of the DBoW2 vocabulary transform (Frame::ComputeBoW; liborbx.so,
orbx_vocab.hip) against the CPU oracle (oracle/orb_vocab.cpp, itself
cross-checked against tests/refpy.py in test_oracle.py). Per-feature words,
node ids and weights, the BowVector (words and double values) and the
FeatureVector must be identical. No ORBvoc.txt exists here: vocabularies are
synthetic (orb_slam_cuda_amd/synth.py), parity unpinned beyond the restatements."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(r, e):
    for key in ("word", "nid", "weight", "bow_words", "bow_values", "fv_nodes", "fv_off", "fv_idx"):
        assert np.array_equal(np.asarray(r[key]), np.asarray(e[key])), key


def _near_leaves(voc, n, seed, flips=2):
    rng = np.random.default_rng(seed)
    leaves = voc["desc"][voc["leaf"] == 1]
    d = leaves[rng.integers(0, len(leaves), n)].copy()
    for _ in range(flips):
        d ^= (1 << rng.integers(0, 8, (n, 32))).astype(np.uint8) * (rng.random((n, 32)) < 0.1)
    if n:
        d[::11] = d[0]  # duplicates: several features on one word
    return d


@pytest.mark.parametrize("k,L,levelsup,scoring,weighting", [(10, 4, 2, 0, 0), (5, 5, 4, 1, 0), (20, 3, 1, 5, 1),
                                                            (3, 6, 9, 0, 2), (7, 3, 0, 2, 3), (17, 3, 2, 4, 0)])
def test_voc_transform_parity(pkg, O, k, L, levelsup, scoring, weighting):
    from orb_slam_cuda_amd.synth import synthetic_vocabulary
    voc = synthetic_vocabulary(k, L, seed=k + L, scoring=scoring, weighting=weighting)
    v = pkg.ORBVocabulary.from_arrays(voc)
    assert v.size() == k ** L and v.getBranchingFactor() == k
    for n in (0, 1, 700, 2000):
        d = _near_leaves(voc, n, seed=n)
        _same(v.transform_arrays(d, levelsup), O.voc_transform(voc, d, levelsup))


def test_voc_irregular_tree(pkg, O):
    rng = np.random.default_rng(3)
    parent = [0, 0, 0, 0, 1, 1, 2, 2, 2, 4, 4]
    leaf = [0, 0, 0, 1, 0, 1, 1, 1, 0, 1, 1]
    desc = rng.integers(0, 256, (len(parent), 32), dtype=np.uint8)
    desc[7] = desc[6]
    weight = np.array([0, 0, 0, 0.5, 0, 0.25, 0.0, 1.5, 0.75, 2.0, 0.125])
    voc = dict(k=3, L=3, scoring=0, weighting=0, parent=np.array(parent, np.int32), leaf=np.array(leaf, np.uint8),
               desc=desc, weight=weight)
    v = pkg.ORBVocabulary.from_arrays(voc)
    d = np.concatenate([desc[[3, 5, 6, 7, 8, 9, 10]], rng.integers(0, 256, (300, 32), dtype=np.uint8)])
    for levelsup in (0, 1, 2, 3):
        _same(v.transform_arrays(d, levelsup), O.voc_transform(voc, d, levelsup))
    # a vocabulary without words transforms to empty vectors (if(empty()) return)
    empty = dict(k=0, L=1, scoring=0, weighting=0, parent=np.zeros(1, np.int32), leaf=np.zeros(1, np.uint8),
                 desc=np.zeros((1, 32), np.uint8), weight=np.zeros(1))
    r = pkg.ORBVocabulary.from_arrays(empty).transform_arrays(d, 4)
    assert len(r["bow_words"]) == 0 and len(r["fv_nodes"]) == 0


def test_voc_text_file(pkg, O, tmp_path):
    from orb_slam_cuda_amd.synth import synthetic_vocabulary, write_vocabulary_text
    voc = synthetic_vocabulary(8, 4, seed=5)
    path = str(tmp_path / "voc.txt")
    write_vocabulary_text(path, voc)
    v = pkg.ORBVocabulary()
    assert v.loadFromTextFile(path)
    ov = O.voc_load_text(path, 10000)
    d = _near_leaves(voc, 1500, seed=9)
    _same(v.transform_arrays(d, 4), O.voc_transform(ov, d, 4))


def test_voc_orbvoc_shape_batch(pkg, O):
    """ORBvoc.txt's shape (k 10, L 6: 1,111,111 nodes, 10^6 words, L1 / TF-IDF) on
    extracted ORB descriptors, batched on the device; ComputeBoW's levelsup 4."""
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence, synthetic_vocabulary
    voc = synthetic_vocabulary(10, 6, seed=1)
    v = pkg.ORBVocabulary.from_arrays(voc)
    W, H, B = 1241, 376, 3
    frames = SynthSequence(21, W, H).frames(B)
    ext = pkg.ORBextractor(2000, 1.2, 8, 20, 7, W, H)
    descs = [ext(f)[1] for f in frames]
    cap = 2100
    host = np.zeros((B, cap, 32), np.uint8)
    n = np.array([len(d) for d in descs], np.int32)
    for i, d in enumerate(descs):
        host[i, :len(d)] = d
    d_desc = _lib.DeviceArray(host.nbytes)
    d_desc.upload(host)
    d_n = _lib.DeviceArray(4 * B)
    d_n.upload(n)
    bw, bv, bn = _lib.DeviceArray(B * cap * 4), _lib.DeviceArray(B * cap * 8), _lib.DeviceArray(4 * B)
    fn, fo, fi, fnn = (_lib.DeviceArray(B * cap * 4), _lib.DeviceArray(B * (cap + 1) * 4),
                       _lib.DeviceArray(B * cap * 4), _lib.DeviceArray(4 * B))
    s = _lib.Stream()
    _lib.check(_lib.lib().orbv_transform_batch(
        v.handle, C.c_void_p(d_desc.ptr), cap * 32, C.c_void_p(d_n.ptr), B, cap, 4, C.c_void_p(bw.ptr),
        C.c_void_p(bv.ptr), C.c_void_p(bn.ptr), C.c_void_p(fn.ptr), C.c_void_p(fo.ptr), C.c_void_p(fi.ptr),
        C.c_void_p(fnn.ptr), None, None, None, s.s), vocabulary=True)
    s.synchronize()
    BW, BV = bw.download(B * cap, np.uint32).reshape(B, cap), bv.download(B * cap, np.float64).reshape(B, cap)
    FN, FO = fn.download(B * cap, np.uint32).reshape(B, cap), fo.download(B * (cap + 1), np.int32).reshape(B, -1)
    FI = fi.download(B * cap, np.int32).reshape(B, cap)
    NB, NF = bn.download(B, np.int32), fnn.download(B, np.int32)
    for i in range(B):
        e = O.voc_transform(voc, descs[i], 4)
        assert NB[i] == len(e["bow_words"]) > 1000
        assert np.array_equal(BW[i, :NB[i]], e["bow_words"]) and np.array_equal(BV[i, :NB[i]], e["bow_values"])
        assert NF[i] == len(e["fv_nodes"])
        assert np.array_equal(FN[i, :NF[i]], e["fv_nodes"]) and np.array_equal(FO[i, :NF[i] + 1], e["fv_off"])
        assert np.array_equal(FI[i, :FO[i, NF[i]]], e["fv_idx"])
    # ComputeBoW on a Frame, and the BowVector feeds the matcher's SearchByBoW inputs
    F = pkg.Frame.from_extraction(*ext(frames[0]), W, H)
    pkg.ComputeBoW(F, v)
    assert abs(sum(F.mBowVec.values()) - 1.0) < 1e-9 and sum(len(x) for x in F.mFeatVec.values()) == F.N
