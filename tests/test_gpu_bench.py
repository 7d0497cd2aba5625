"""bench.py end to end on the GPU through the worker launcher (--spawn with
--gpus 1: the same spawned-worker path an 8-GPU node takes), small sizes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_launcher_one_gpu():
    out = _bench(["--gpus", "1", "--spawn", "--steps", "3", "--warmup", "1", "--pool", "128", "--cpu-sample", "0",
                  "--host-steps", "3"])
    assert out["n_gpus"] == 1 and len(out["per_rank_frames_per_s"]) == 1
    assert out["value"] > 0 and out["unit"] == "frames/s"
    assert out["roofline"]["frac"] > 0 and out["roofline"]["bound"] == "hbm"
    assert 1900 <= out["keypoints_per_frame"] <= 2020
    assert out["init_matches_per_pair"] > 50
    lat = out["latency"]
    assert lat["extract_ms"]["median"] > 0 and lat["search_init_ms"]["median"] > 0
    assert out["host_stream"]["value"] > 0
    tie = out["quadtree_tie_straddle"]
    assert tie["frames"] == 64 and 0 <= tie["fraction_of_kept"] < 0.5


def test_bench_euroc_and_extract_only():
    out = _bench(["--config", "euroc", "--steps", "3", "--warmup", "1", "--pool", "64", "--cpu-sample", "0",
                  "--no-latency", "--no-host-stream"])
    assert out["n_gpus"] == 1 and 950 <= out["keypoints_per_frame"] <= 1020
    out = _bench(["--no-match", "--steps", "3", "--warmup", "1", "--pool", "64", "--cpu-sample", "0", "--no-latency",
                  "--no-host-stream"])
    assert out["match_roofline"] is None and "extract only" in out["config"]["workload"]


def test_bench_stereo():
    out = _bench(["--config", "stereo", "--steps", "3", "--warmup", "1", "--batch", "16", "--cpu-sample", "0"])
    assert out["unit"] == "stereo pairs/s" and out["stereo_matches_per_pair"] > 100


def test_split_sequence_boundary_pair_two_ranks(O, tmp_path):
    """bench.py --split-sequence with two ranks (both on device 0, a test-only
    flag) through the spawned-worker launcher: ONE sequence of 128 frames,
    rank 1's block starts at frame 64, and its first pair (frame 63 -> 64), whose
    t-1 frame rank 1 extracts itself, must match the oracle exactly: keypoints,
    descriptors, dense top-2 and SearchForInitialization (src/ORBmatcher.cc:405-520).
    Rank 0's first frame has no predecessor (count 0, no matches)."""
    import numpy as np
    from orb_slam_cuda_amd.synth import SynthStream
    out = _bench(["--gpus", "2", "--spawn", "--share-device", "--split-sequence", "--steps", "1", "--warmup", "0",
                  "--batches-per-step", "1", "--pool", "64", "--dump-pairs", str(tmp_path), "--cpu-sample", "0",
                  "--no-latency", "--no-host-stream"])
    assert out["n_gpus"] == 2 and "split" in out["config"]["parallelism"]
    W, H = 1241, 376
    stream = SynthStream(1000, W, H)
    cfg = O.config(nfeatures=2000, width=W, height=H)
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    assert list(r0["block"]) == [0, 64] and list(r1["block"]) == [64, 128] and int(r1["prev"][0]) == 63
    assert r0["counts"][0] == 0 and r0["nm"][0] == 0
    for pair in (0, 1, 37):  # the boundary pair and two interior ones of rank 1
        fa, fb = 63 + pair, 64 + pair
        k1, d1 = O.extract(cfg, stream.frame(fa))
        k2, d2 = O.extract(cfg, stream.frame(fb))
        n1, n2 = r1["counts"][pair], r1["counts"][pair + 1]
        assert n1 == len(k1) and n2 == len(k2)
        assert np.array_equal(r1["kps"][pair, :n1].view(np.uint8), k1.view(np.uint8))
        assert np.array_equal(r1["desc"][pair + 1, :n2], d2)
        ri, rd, rs = O.hamming_top2(d2, d1)
        assert np.array_equal(r1["bi"][pair, :n2], ri) and np.array_equal(r1["bd"][pair, :n2], rd)
        assert np.array_equal(r1["sd"][pair, :n2], rs)
        r12, rnm, _ = O.search_for_initialization(k1, d1, k2, d2, (0, W, 0, H), np.stack([k1["x"], k1["y"]], 1),
                                                  100, 0.9, True)
        assert r1["nm"][pair] == rnm > 20 and np.array_equal(r1["m12"][pair, :n1], r12)


def test_bench_torchrun_two_ranks_one_device():
    """The driver's multi-GPU launch command (python -m torch.distributed.run
    --nproc-per-node N ... bench.py --gpus N) with two ranks, both on device 0
    (--share-device, test only): every rank runs its own pipeline, the
    barrier + max-over-ranks timing holds, rank 0 prints the one line."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--share-device", "--steps", "3", "--warmup", "1", "--pool", "128", "--cpu-sample", "0",
           "--no-latency", "--no-host-stream"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and len(out["per_rank_frames_per_s"]) == 2
    assert out["value"] > 0 and out["scaling"] == "weak"
    assert out["cpu_baseline"] is None  # rank 0 at N = 1 only
