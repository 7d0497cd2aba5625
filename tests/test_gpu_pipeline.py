"""Parity of the TIMED pipeline itself: bench.MonoPipeline with the bench's
defaults (B = 64 frames per batch, --split 2 extraction launches on two
streams, 3 output sets, the t-1 carry on the high-priority matching stream,
a resident pool larger than one batch), run for several batches exactly as
bench.py's timed region runs them, and every pair of the last three batches
compared with the oracle:

* keypoints (all 7 cv::KeyPoint fields, order) and descriptor bytes of every
  frame, including slot 0 of each batch, which arrives through the carry copy
  of the previous batch's last frame (bench.py MonoPipeline.step, carry());
* the dense Hamming top-2 (best index, best and second distance) of frame t
  against frame t-1;
* SearchForInitialization (src/ORBmatcher.cc:405-520; windows on frame t-1's
  own keypoints, Tracking's initial vbPrevMatched, src/Tracking.cc:645-672):
  matches12 and the match count;
* with --bow-match, SearchByBoW(KF t-1, F t) (src/ORBmatcher.cc:159-288,
  ratio 0.7 as Tracking::TrackReferenceKeyFrame, src/Tracking.cc:839) of the
  last batch, with the oracle's own ComputeBoW FeatureVectors.

A missing event edge between the extraction, carry and matching streams
would show up here as a mismatch on a batch-boundary pair (slot 0)."""
import ctypes as C
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KP, DS = 28, 32


def _run_pipeline(argv, batches, host=False):
    import bench
    from orb_slam_cuda_amd import _lib, sharding
    from orb_slam_cuda_amd.synth import SynthSequence
    args = bench.parse_args(argv)
    cfg = bench.CONFIGS[args.config]
    W, H, B = cfg["W"], cfg["H"], args.batch
    frames = SynthSequence(sharding.sequence_seed(0), W, H).frames(args.pool)
    pipe = bench.MonoPipeline(args, cfg, 0, frames, host=host)
    assert pipe.S == 2 and pipe.NS == 3 and not args.serial and args.carry == "match" and not args.match_priority
    assert pipe.nbatches > 1  # the pool cycles: level 0 streams from a different slot every batch
    pipe.run(0, batches, None)  # the timed region's issue order, without the warmup split
    pipe.check_status()
    return args, cfg, frames, pipe, _lib


def _download_set(pipe, k):
    """Batch k's outputs (set k % 3) after the pipeline drained."""
    B, cap, s = pipe.B, pipe.cap, k % pipe.NS
    n = pipe.d_counts[s].download(B + 1, np.int32)
    import orb_slam_cuda_amd as pkg
    kps = pipe.d_kps[s].download((B + 1) * cap, pkg.KP_DTYPE).reshape(B + 1, cap)
    desc = pipe.d_desc[s].download(((B + 1), cap, 32), np.uint8)
    top = [a.download((B, cap), np.int32) for a in (pipe.d_bi[s], pipe.d_bd[s], pipe.d_sd[s])]
    m12 = pipe.d_m12[s].download((B, cap), np.int32)
    nm = pipe.d_nm[s].download(B, np.int32)
    return n, kps, desc, top, m12, nm


def _oracle_frames(O, cfg, frames, idx):
    import bench
    oc = bench.oracle_config(O, cfg)
    with ThreadPoolExecutor(8) as ex:  # the oracle's C calls release the GIL
        res = list(ex.map(lambda i: O.extract(oc, frames[i]), idx))
    return dict(zip(idx, res))


def _check_batches(O, cfg, frames, pipe, batches, check):
    B = pipe.B
    nb = pipe.nbatches
    W, H = cfg["W"], cfg["H"]
    # frame of slot j of batch k: the pool slot k % nb; slot 0 = the previous batch's last frame
    fidx = lambda k, j: ((k % nb) * B + j - 1) if j > 0 else (((k - 1) % nb) * B + B - 1)
    # the last batch's carry (step batches - 1) already wrote slot 0 of set batches % 3, i.e.
    # of batch batches - 3: after the run that slot holds the next batch's t-1 frame
    held = lambda k, j: fidx(batches, 0) if (j == 0 and k == batches - 3) else fidx(k, j)
    need = sorted({fidx(k, j) for k in check for j in range(B + 1)} | {held(k, 0) for k in check})
    ref = _oracle_frames(O, cfg, frames, need)
    pairs = []
    for k in check:
        n, kps, desc, (bi, bd, sd), m12, nm = _download_set(pipe, k)
        for j in range(B + 1):
            rk, rd = ref[held(k, j)]
            assert n[j] == len(rk), (k, j)
            assert np.array_equal(kps[j, :n[j]].view(np.uint8), rk.view(np.uint8)), ("keypoints", k, j)
            assert np.array_equal(desc[j, :n[j]], rd), ("descriptors", k, j)
        for p in range(B):
            pairs.append((k, p, ref[fidx(k, p)], ref[fidx(k, p + 1)], bi, bd, sd, m12, nm))

    def one(t):
        # inputs = the oracle's frames t-1 and t (equal to the device's, checked above)
        k, p, (k1, d1), (k2, d2), bi, bd, sd, m12, nm = t
        ri, rd, rs = O.hamming_top2(d2, d1)
        r12, rnm, _ = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  100, 0.9, True)
        na = len(k2)
        ok_top = (np.array_equal(bi[p, :na], ri) and np.array_equal(bd[p, :na], rd)
                  and np.array_equal(sd[p, :na], rs))
        ok_init = nm[p] == rnm and np.array_equal(m12[p, :len(k1)], r12)
        return k, p, ok_top, ok_init, int(rnm)

    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(one, pairs))
    bad = [(k, p, t, i) for k, p, t, i, _ in res if not (t and i)]
    assert not bad, f"pairs differing from the oracle (batch, pair, top2 ok, init ok): {bad[:10]}"
    boundary = [r for r in res if r[1] == 0]
    assert len(boundary) == len(check)
    # a boundary pair whose pool slot does not wrap holds consecutive frames of the sequence
    assert all(r[4] > 20 for r in boundary if r[0] % nb != 0), boundary
    assert np.mean([r[4] for r in res]) > 50


@pytest.mark.parametrize("config", ["kitti", "euroc", "kitti14", "intcatch1080"])
def test_timed_pipeline_matches_oracle(pkg, O, config):
    """kitti14: Examples/Monocular/KITTI14.yaml (10 levels, the >8-level orient+BRIEF
    instantiation); intcatch1080: intcatch-1080p.yaml (1920x1080, 3 levels, 10/4)."""
    batches = 5
    args, cfg, frames, pipe, _ = _run_pipeline(["--config", config, "--pool", str(4 * 64)], batches)
    assert pipe.B == 64
    # batches 2, 3, 4: set k % 3 still holds them; batch 4 reuses pool slot 0 (pool of 4 batches),
    # its slot 0 is the last frame of pool slot 3
    _check_batches(O, cfg, frames, pipe, batches, range(batches - 3, batches))


def test_timed_pipeline_bow_match_matches_oracle(pkg, O):
    from orb_slam_cuda_amd.synth import synthetic_vocabulary
    batches = 4
    args, cfg, frames, pipe, _lib = _run_pipeline(["--bow-match", "--pool", str(3 * 64)], batches)
    B, cap = pipe.B, pipe.cap
    _check_batches(O, cfg, frames, pipe, batches, [batches - 1])
    # SearchByBoW of the last batch: pair p = (KF slot p, F slot p + 1); every KF feature has a MapPoint
    n, kps, desc, *_ = _download_set(pipe, batches - 1)
    out = pipe.d_bow_out.download((B, cap), np.int32)
    nm = pipe.d_bow_nm.download(B, np.int32)
    voc = synthetic_vocabulary(10, 6, seed=1)  # the bench's vocabulary (MonoPipeline.__init__)
    fv = {}
    for j in range(B + 1):
        t = O.voc_transform(voc, desc[j, :n[j]], 4)
        fv[j] = (t["fv_nodes"], t["fv_off"], t["fv_idx"])
    for p in range(B):
        a, b = p, p + 1
        rout, rnm = O.search_by_bow(desc[a, :n[a]], kps[a, :n[a]]["angle"], np.ones(n[a], np.uint8), fv[a],
                                    desc[b, :n[b]], kps[b, :n[b]]["angle"], np.ones(n[b], np.uint8), fv[b],
                                    0.7, True, False)
        assert nm[p] == rnm and np.array_equal(out[p, :n[b]], rout), p
    assert nm.mean() > 20


@pytest.mark.parametrize("mode,parts", [("2d", 1), ("2d", 2), ("2d", 4), ("1d", 2), ("kernel", 2)])
def test_host_streamed_pipeline_matches_oracle(pkg, O, mode, parts):
    """The host-streamed leg (bench.py host_stream_leg): every batch uploaded
    from pinned host memory in `parts` pieces on their own copy streams, each
    extraction half waiting for its own pieces; outputs read back on a copy
    stream. Uploads: padded rows (1d DMA), unpadded rows into the device
    pitch (2d DMA rectangle, the default) or by the copy kernel. A missing
    upload edge would extract stale or partial frames."""
    batches = 4
    args, cfg, frames, pipe, _ = _run_pipeline(["--pool", str(3 * 64), "--h2d-split", str(parts), "--h2d-mode", mode],
                                               batches, host=True)
    assert len(pipe.s_h2ds) == parts
    _check_batches(O, cfg, frames, pipe, batches, [batches - 2, batches - 1])
    # the read-back of the last batch equals the device outputs
    k = batches - 1
    B, cap, s = pipe.B, pipe.cap, k % pipe.NS
    n, kps, desc, _, m12, nm = _download_set(pipe, k)
    assert np.array_equal(pipe.h_counts[s].a, n[1:])
    assert np.array_equal(pipe.h_kps[s].a.reshape(B, cap * KP), kps[1:].view(np.uint8).reshape(B, cap * KP))
    assert np.array_equal(pipe.h_desc[s].a.reshape(B, cap, 32), desc[1:])
    assert np.array_equal(pipe.h_nm[s].a, nm)
