"""Pins of the oracle (and the product's tables) to bytes the reference holds,
and the quadtree tie-rule exposure counter.

* bit_pattern_31_: tests/golden/bit_pattern.npy is parsed from the reference
  source text (tests/golden/make_pattern.py, src/ORBextractor.cc:236-494, the
  fork's `VX_FAILURE-2` element at :261-262). Both the oracle's table and the
  table liborbx.so uploads to the device must equal it; every descriptor bit
  depends on it.
* tie straddles: DistributeOctTree splits equal-size nodes in heap-pointer
  order (src/ORBextractor.cc:1041-1042); the oracle and the kernels use node
  creation order instead. The counter reports where that choice decided
  which keypoints were kept.
"""
import os

import numpy as np

from conftest import GOLDEN


def golden_pattern():
    return np.load(os.path.join(GOLDEN, "bit_pattern.npy"))


def test_pattern_golden_shape_and_fork_entry():
    t = golden_pattern()
    assert t.dtype == np.int8 and t.shape == (1024,)
    assert int(t[96]) == -3            # VX_FAILURE - 2 (src/ORBextractor.cc:261-262)
    assert t.min() >= -13 and t.max() <= 12  # 31x31 patch, as the descriptor assumes


def test_oracle_pattern_equals_reference_table(O):
    t = golden_pattern()
    assert np.array_equal(O.pattern(0), t)
    up = O.pattern(1)
    diff = np.nonzero(up != t)[0]
    assert diff.tolist() == [96] and int(up[96]) == -2  # upstream ORB-SLAM2


def test_product_pattern_equals_reference_table():
    from orb_slam_cuda_amd.extractor import brief_pattern
    t = golden_pattern().astype(np.int32)
    assert np.array_equal(brief_pattern("fork"), t)
    up = brief_pattern("upstream")
    assert np.nonzero(up != t)[0].tolist() == [96] and int(up[96]) == -2


def test_pattern_script_parses_reference_if_present():
    src = "/root/reference/src/ORBextractor.cc"
    if not os.path.exists(src):
        return  # the GPU box has no reference tree; the committed .npy is the pin
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_pattern", os.path.join(GOLDEN, "make_pattern.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    with open(src, encoding="utf-8", errors="replace") as f:
        assert np.array_equal(m.parse(f.read()), golden_pattern())


def _kps(xy):
    from oracle.oracle import KP_DTYPE
    k = np.zeros(len(xy), KP_DTYPE)
    k["x"] = [p[0] for p in xy]
    k["y"] = [p[1] for p in xy]
    k["response"] = 10
    k["octave"] = 0
    k["class_id"] = -1
    return k


def test_tie_straddle_known_case(O):
    # one 40x40 root, two keys in each quadrant (different sub-quadrants):
    # round 1 splits the root into four size-2 nodes (4 < N = 5); 4 + 4*3 > 5
    # starts the sorted phase over four EQUAL sizes; splitting the first one
    # reaches 5 nodes, so the tie rule alone chose which quadrant was split
    pts = [(5, 5), (15, 15), (25, 5), (35, 15), (5, 25), (15, 35), (25, 25), (35, 35)]
    kept = O.distribute(_kps(pts), 0, 40, 0, 40, 5)
    assert len(kept) == 5
    assert O.distribute_ties(_kps(pts), 0, 40, 0, 40, 5) == (1, 4, 5)  # event, 4 nodes, 2 + 3 kept keys


def test_no_tie_straddle_when_sizes_differ(O):
    # the same, but one quadrant holds 3 keys: it is split first, alone in its size group
    pts = [(5, 5), (15, 15), (12, 3), (25, 5), (35, 15), (5, 25), (15, 35), (25, 25), (35, 35)]
    assert O.distribute_ties(_kps(pts), 0, 40, 0, 40, 5) == (0, 0, 0)


def test_tie_stats_invariants_on_synthetic_frame(O):
    from orb_slam_cuda_amd.synth import synth_frame
    W, H = 640, 240
    cfg = O.config(nfeatures=600, width=W, height=H)
    img = synth_frame(3, W, H)
    st = O.tie_stats(cfg, img)
    kp, _ = O.extract(cfg, img)
    per_level = np.bincount(kp["octave"], minlength=8)
    assert set(np.unique(st["events"])) <= {0, 1}
    for l in range(8):
        if st["events"][l]:
            assert 2 <= st["nodes"][l] <= st["kps"][l] <= per_level[l]
        else:
            assert st["nodes"][l] == st["kps"][l] == 0


def test_scale_mode_pinned_by_reference_map(O):
    """The reference's own map (Examples/Monocular/map.yml, written by
    MapPoint::write, src/MapPoint.cc:489-490) pins the extractor's top-level
    scale factor: MapPoint::UpdateNormalAndDepth sets
    mfMinDistance = mfMaxDistance / mvScaleFactors[nLevels-1]
    (src/MapPoint.cc:68-69, 372-373) in float. All 775 stored pairs satisfy it
    with the upstream 1.2^7 table (scale mode U, the default here) and none
    with the fork's buildGraph override (mode F, src/ORBextractor.cc:674-680)
    at the KITTI width, so the run that wrote the reference's map used mode U.
    Values extracted by tests/golden/make_mapyml.py."""
    d = np.load(os.path.join(GOLDEN, "mapyml_distances.npy"))
    assert d.shape == (775, 2) and d.dtype == np.float32
    mx, mn = d[:, 0], d[:, 1]
    sU = O.level_info(O.config(scale_mode=0))["scale"]
    assert np.float32(sU[7]) == np.float32(3.5831816)  # iterative float product 1.2^7 (:505-509)
    assert np.array_equal(mx / np.float32(sU[7]), mn)
    for w, h in ((1241, 376), (752, 480), (640, 480)):
        sF = O.level_info(O.config(scale_mode=1, width=w, height=h))["scale"]
        assert not np.any(mx / np.float32(sF[7]) == mn), (w, h, sF[7])


def test_tie_rule_study_pointer_order_is_heap_history(O):
    """The reference breaks the quadtree's size ties by heap address
    (src/ORBextractor.cc:1041). The oracle's rule 1 runs a layout-identical
    ExtractorNode with the reference's allocation sequence on the real glibc
    heap. Measured on committed-seed C3 frames:
    * the product's creation-order rule is deterministic (rule 0 twice: equal);
    * the pointer rule is NOT reproducible by the reference itself: the same
      frames through it a second time (another heap history) keep a different
      keypoint list order at most levels and some different keypoints;
    * creation order differs from the pointer order by about as much as the
      pointer order differs from itself, in a small fraction of the kept keypoints."""
    from orb_slam_cuda_amd.synth import SynthSequence
    fr = SynthSequence(1000, 1241, 376).frames(6)  # the bench's rank-0 C3 sequence
    cfg = O.config()
    d00, k00 = O.tie_sequence(cfg, fr, 0, 0)
    assert not d00.any() and not k00.any()
    d01, k01 = O.tie_sequence(cfg, fr, 0, 1)
    d11, k11 = O.tie_sequence(cfg, fr, 1, 1)
    kept = 2000 * len(fr)
    assert d01.mean() > 0.5 and d11.mean() > 0.5        # list order: heap-dependent at most levels
    assert 0 < k01.sum() < 0.05 * kept and 0 < k11.sum() < 0.05 * kept
    # which node the cut-off split also moves a level's count within the reference's overshoot (N .. N + 2)
    a = O.extract_rule(cfg, fr[0], 0)[0]
    b = O.extract_rule(cfg, fr[0], 1)[0]
    assert np.abs(np.bincount(a["octave"], minlength=8) - np.bincount(b["octave"], minlength=8)).max() <= 2
