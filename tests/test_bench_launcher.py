"""CPU tests of bench.py's multi-GPU launcher and reporting path: `--gpus N`
spawns N worker processes that join the gloo control plane, and rank 0
reports the whole-job aggregate. The GPU work is replaced by a stub worker
(--stub-worker); everything else is the code the 8-GPU run executes."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_workers_and_aggregates(n):
    pytest.importorskip("torch")
    r = _run(["--gpus", str(n), "--steps", "5", "--warmup", "1", "--batch", "8", "--stub-worker"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["frames_total"] == n * 8 * 5
    per = out["per_rank_frames_per_s"]
    assert len(per) == n and all(v > 0 for v in per)
    # rank r sleeps (1 + r) x 10 ms: the job time is the slowest rank's
    assert per[0] > per[-1]
    assert out["value"] <= sum(per) + 1e-6
    assert abs(out["value"] - out["frames_total"] / (out["frames_total"] / n / per[-1])) / out["value"] < 0.05


def test_launcher_c5_shape_eight_ranks():
    """C5's shape (8 x EuRoC 752x480, one sequence per GPU) through the launcher
    with stub workers: eight ranks, eight distinct sequences, the aggregate is
    the sum of the ranks' frames over the slowest rank's wall time."""
    pytest.importorskip("torch")
    n, batch, steps = 8, 8, 3
    r = _run(["--gpus", str(n), "--config", "euroc", "--steps", str(steps), "--warmup", "1", "--batch", str(batch),
              "--stub-worker"], timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["config"]["workload"].startswith("C5")
    ranks = out["ranks"]
    assert [x["rank"] for x in ranks] == list(range(n))
    assert len({x["seed"] for x in ranks}) == n  # one distinct sequence per GPU
    assert all(x["frame"] == "752x480" and x["nfeatures"] == 1000 for x in ranks)
    assert out["frames_total"] == sum(x["frames"] for x in ranks) == n * batch * steps
    per = out["per_rank_frames_per_s"]
    assert len(per) == n and min(per) == per[-1]  # rank 7 sleeps longest
    # value = all frames / the slowest rank's time (not a sum or mean of rates)
    assert abs(out["value"] - out["frames_total"] / out["job_wall_s"]) / out["value"] < 1e-3
    assert abs(out["job_wall_s"] - batch * steps / per[-1]) / out["job_wall_s"] < 0.01
    assert out["value"] < sum(per)


def test_gpus_must_match_torchrun_world():
    pytest.importorskip("torch")
    r = _run(["--gpus", "2", "--stub-worker"], {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_launcher_refuses_to_oversubscribe():
    pytest.importorskip("torch")
    import torch
    n = torch.cuda.device_count()
    r = _run(["--gpus", str(n + 1), "--spawn", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and "oversubscribe" in (r.stderr + r.stdout)


def test_parse_defaults():
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse_args([])
    assert a.gpus == 1 and a.batch == 64 and a.pool % a.batch == 0 and a.pool * 1280 * 376 > 256 * 2 ** 20
    assert a.match_order == "init,top2,bow" and not a.match_priority
    assert bench.parse_args(["--bow-match"]).match_order == "bow,init,top2"


@pytest.mark.parametrize("order,ok", [("init,top2,bow", True), ("bow,top2,init", True), ("top2,bow", False),
                                      ("top2,top2,init", False), ("top2,bow,init,x", False)])
def test_parse_match_order(order, ok):
    sys.path.insert(0, ROOT)
    import bench
    if ok:
        assert bench.parse_args(["--match-order", order]).match_order == order
    else:
        with pytest.raises(SystemExit):
            bench.parse_args(["--match-order", order])


def test_launcher_parent_never_loads_hip():
    """visible_gpus() counts devices in a child: the launcher process, which
    spawns the per-GPU workers, must not have the HIP runtime or liborbx mapped."""
    pytest.importorskip("torch")
    code = ("import sys; sys.path.insert(0, %r); import bench; n = bench.visible_gpus(); "
            "m = open('/proc/self/maps').read(); "
            "print(n, 'libamdhip64' in m, 'liborbx' in m)") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    n, hip, orbx = r.stdout.split()
    assert int(n) >= 0 and hip == "False" and orbx == "False"


@pytest.mark.parametrize("var", ["ORBX_INIT_STOP", "ORBX_FAST_TWICE", "ORBX_FAST_PROF", "ORBX_LIB_VARIANT",
                                 "ORBX_SOMETHING_NEW"])
def test_bench_refuses_diagnostic_env(var):
    """A timed region under a switch that skips, repeats or clocks work (or an
    A/B library variant, or an undocumented variable) is refused..."""
    pytest.importorskip("torch")
    r = _run(["--gpus", "1", "--spawn", "--steps", "1", "--warmup", "0", "--stub-worker"], {var: "1"})
    assert r.returncode != 0 and "refusing" in (r.stderr + r.stdout) and var in r.stderr
    # ...unless asked for, and then the line names it
    r = _run(["--gpus", "1", "--spawn", "--steps", "1", "--warmup", "0", "--stub-worker", "--allow-diag"], {var: "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["orbx_env"] == {var: "1"}


def test_bench_allows_and_stamps_tuning_env():
    pytest.importorskip("torch")
    r = _run(["--gpus", "1", "--spawn", "--steps", "1", "--warmup", "0", "--stub-worker"], {"ORBX_PYR_PLAN": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["orbx_env"] == {"ORBX_PYR_PLAN": "1"}


def test_env_audit_unit():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.audit_env(False, {"PATH": "/bin", "ORBX_TOP2_VALU": "1"}) == {"ORBX_TOP2_VALU": "1"}
    with pytest.raises(SystemExit):
        bench.audit_env(False, {"ORBX_VOC_STOP": "1"})
    assert bench.audit_env(True, {"ORBX_VOC_STOP": "1"}) == {"ORBX_VOC_STOP": "1"}
