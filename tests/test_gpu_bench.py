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
