#!/usr/bin/env python3
"""bench.py — ORB extract + match throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): KITTI-shaped 1241x376 mono u8
frames, nFeatures=2000, 8 levels, scale 1.2, iniThFAST 20 / minThFAST 7.
One step = --batches-per-step (4) consecutive batches of B (64) frames
resident in HBM; per batch:
  * ORBextractor::operator() on all B frames (orbx_extract_batch), and
  * for every frame t, matching against frame t-1: the dense brute-force
    2000 x 2000 Hamming best/second search (orbm_hamming_top2) and the exact
    ORBmatcher::SearchForInitialization (window 100, ratio 0.9, rotation
    check) used by monocular initialisation.
Frame t-1 of the first frame of a batch is the last frame of the previous
batch (carried on device), so every batch does B extractions + B matches.
Batch k processes slot k mod (pool / B) of a resident pool of synthetic
frames larger than the 256 MB MALL (--pool, default 640 frames = 308 MB),
so level 0 streams from HBM instead of staying in the last-level cache.

Streams: the matching of batch k (a few wide workgroups per frame pair) runs
on its own stream, overlapping the extraction of batch k+1; outputs are
triple-buffered and ordered by events (see MonoPipeline.step). --serial runs
everything on one stream.

Extra legs in the same JSON line (rank 0, N = 1; skipped with --no-latency /
--no-host-stream):
  * "latency": the call Tracking makes per frame, orbx_extract on ONE host
    1241x376 image (host in, host keypoints + descriptors out; pinned
    staging, captured hipGraph) and the host SearchForInitialization call,
    median / p99 over 200 calls, beside the oracle's single-thread latency;
  * "host_stream": the same C3 pipeline fed from pinned host memory every
    step (H2D of each batch on a copy stream, keypoints / descriptors /
    matches copied back), PCIe-inclusive frames/s.

Multi-GPU: one process per GPU. `--gpus N` without a torchrun environment
spawns N worker processes (multiprocessing "spawn", before this process
touches the GPU); under torchrun (RANK set) each rank is one worker and
--gpus must equal WORLD_SIZE. Each rank selects device LOCAL_RANK before any
allocation, streams its own synthetic sequence and matches within its shard:
no data-path collective ("weak" scaling). The barrier, the max-over-ranks of
the timed region and the per-rank figures go through torch.distributed with
the gloo backend (control plane only).

Prints ONE JSON line (rank 0). Per-kernel durations are measured live with
HIP events recorded on the launch stream around every stage of every step.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/s ORB extract+match, 1241×376 mono nFeatures=2000; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
# Dense FP4 MFMA peak (the Hamming top-2 runs on v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1
# operands): 65536 MACs per 32 cycles per SIMD x 1024 SIMDs x 2.4 GHz = 10.07 PFLOP/s
# (MI355X_MICROARCH.md: FP4 = 4x the BF16 rate, dense, no sparsity)
MFMA_FP4_PEAK_TFLOPS = 10066.3
# VALU lane-op peak: 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz (the top-2 update costs 2 lane-ops per pair)
VALU_PEAK_TOPS = 78.6
STAGES = ["pyramid", "blur", "fast_grid", "quadtree", "orient_brief", "hamming_top2", "search_init"]
KERNELS = {"bow_transform": "voc_descend_kernel + voc_assemble_kernel", "pyramid": "pyr_band_kernel", "blur": "blur_kernel", "fast_grid": "fast_cells_kernel",
           "bow_match": "search_bow_kernel<256>",
           "quadtree": "quadtree_kernel", "orient_brief": "orient_brief_kernel",
           "hamming_top2": "hamming_top2_mfma_kernel", "search_init": "search_init_prep_kernel + search_init_query_kernel + search_init_resolve_kernel"}
KP, DS = 28, 32  # bytes of one orbx_kp (cv::KeyPoint) and one descriptor

CONFIGS = {
    "kitti": dict(W=1241, H=376, nfeatures=2000,
                  workload="C3: KITTI-shaped 1241x376 mono u8, nFeatures=2000, 8 levels x1.2, "
                           "extract + match vs t-1 (dense 2000x2000 Hamming top-2 + SearchForInitialization)"),
    "stereo": dict(W=1241, H=376, nfeatures=2000, stereo=True,
                   workload="C4: stereo_kitti, 2 x 1241x376 u8 per pair, nFeatures=2000 per image, 8 levels x1.2, "
                            "left/right extraction on separate HIP streams + Frame::ComputeStereoMatches"),
    "euroc": dict(W=752, H=480, nfeatures=1000,
                  workload="C5: EuRoC-shaped 752x480 mono u8, nFeatures=1000, 8 levels x1.2, "
                           "extract + match vs t-1 (dense Hamming top-2 + SearchForInitialization), "
                           "one sequence per GPU"),
    # the reference's other shipped camera settings (parity cases, not bench lines)
    "kitti14": dict(W=1226, H=370, nfeatures=2000, nlevels=10, ini=17, mn=7,
                    workload="Examples/Monocular/KITTI14.yaml: 1226x370, nFeatures=2000, 10 levels x1.2, 17/7, "
                             "extract + match vs t-1"),
    "intcatch1080": dict(W=1920, H=1080, nfeatures=2000, nlevels=3, ini=10, mn=4,
                         workload="Examples/Monocular/intcatch-1080p.yaml: 1920x1080, nFeatures=2000, 3 levels "
                                  "x1.2, 10/4, extract + match vs t-1"),
}


def ext_params(cfg):
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) of a config
    (the yaml's ORBextractor.* keys, src/Tracking.cc:123-141)."""
    return (cfg["nfeatures"], cfg.get("scale", 1.2), cfg.get("nlevels", 8), cfg.get("ini", 20), cfg.get("mn", 7))


def oracle_config(O, cfg):
    nf, sc, nl, ini, mn = ext_params(cfg)
    return O.config(nfeatures=nf, width=cfg["W"], height=cfg["H"], scale_factor=sc, nlevels=nl,
                    ini_th=ini, min_th=mn)


def level_sizes(W, H, L=8, s=1.2):
    sc = [1.0]
    for _ in range(1, L):
        sc.append(np.float32(sc[-1]) * np.float32(s))
    out = []
    for f in sc:
        inv = np.float32(1.0) / np.float32(f)
        out.append((int(np.rint(np.float32(W) * inv)), int(np.rint(np.float32(H) * inv))))
    return out


def algorithmic_bytes(W, H, nkp, L=8, s=1.2):
    """Per-frame algorithmic HBM bytes of each stage (DESIGN.md "Roofline")."""
    P = [w * h for w, h in level_sizes(W, H, L, s)]
    return {
        "pyramid": sum(P[l - 1] + P[l] for l in range(1, L)),         # read l-1, write l
        "blur": 2 * sum(P),                                            # read + write every level
        "fast_grid": sum(P),                                           # read every level once
        "pyr_fast_pass": P[0] + sum(P[:L - 1]) + sum(P[1:]) + sum(P),  # BASELINE.md B_pf
        "orient_brief": nkp * (2 * 31 * 31 + 60),                      # patch gathers + outputs
    }


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="GPUs of this node, one worker process each")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64, help="frames per batch per GPU (2 extraction launches of 32)")
    ap.add_argument("--batches-per-step", type=int, default=4,
                    help="batches per timed step (a step is 4 x 64 frames by default, so a short --steps "
                         "run still times the pipeline's steady state rather than its fill and drain)")
    ap.add_argument("--pool", type=int, default=640,
                    help="resident synthetic frames per GPU, cycled batch by batch (> the 256 MB MALL)")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="kitti")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="frame-parallel oracle workers for cpu_baseline (0 = the host's CPU share, OMP_NUM_THREADS)")
    ap.add_argument("--cpu-sample", type=int, default=200,
                    help="frames (stereo: 2 x pairs) in the CPU baseline sample, ~10 s on one core (0 = skip)")
    ap.add_argument("--no-match", action="store_true", help="extract only (C2)")
    ap.add_argument("--serial", action="store_true", help="one stream: no overlap of matching with the next extraction")
    ap.add_argument("--split", type=int, default=2, help="extraction launches (and streams) per batch")
    ap.add_argument("--priority", action="store_true",
                    help="high-priority extraction streams, low-priority matching stream")
    ap.add_argument("--match-priority", dest="match_priority", action="store_true", default=False,
                    help="matching stream(s) at high priority (A/B; default normal: with the pyramid, FAST, "
                         "quadtree, blur, orient+BRIEF stage order that is 2 %% faster on C3 and EuRoC and "
                         "equal on the other configs, DESIGN.md section 6)")
    ap.add_argument("--no-match-priority", dest="match_priority", action="store_false", default=False,
                    help="matching stream(s) at normal priority (the default)")
    ap.add_argument("--match-cus", default="",
                    help="A/B: the matching stream(s) on a compute-unit subset, 'stride:K' (every K-th CU) or "
                         "'first:N'; with --cu-exclusive the extraction streams get the other CUs")
    ap.add_argument("--cu-exclusive", action="store_true", help="with --match-cus: extraction on the complement")
    ap.add_argument("--bow", action="store_true",
                    help="also Frame::ComputeBoW every frame (synthetic ORBvoc-shaped vocabulary, k 10 L 6)")
    ap.add_argument("--bow-match", action="store_true",
                    help="also SearchByBoW of every frame against its predecessor as reference keyframe (implies --bow)")
    ap.add_argument("--match-streams", type=int, choices=[1, 2], default=1,
                    help="2: SearchForInitialization on its own stream, beside the dense top-2")
    ap.add_argument("--match-order", type=match_order, default=None,
                    help="order of the matching stages on the matching stream: a permutation of top2 (dense "
                         "Hamming top-2), bow (ComputeBoW [+ SearchByBoW], with --bow/--bow-match), init "
                         "(SearchForInitialization); default init,top2,bow (bow,init,top2 with --bow / "
                         "--bow-match: SearchForInitialization first is 7 %% faster on KITTI14, 4-7 %% on EuRoC, "
                         "but 14 %% slower with the BoW stages, DESIGN.md section 6)")
    ap.add_argument("--carry", choices=["match", "ext"], default="match",
                    help="stream that copies a batch's last frame for the next batch's first pair")
    ap.add_argument("--stage-order", default="",
                    help="the extraction stages' launch order (orbx_set_stage_order: p b f q o, e.g. pfqbo); "
                         "default: the library's, pbfqo with --bow / --bow-match")
    ap.add_argument("--no-latency", action="store_true", help="skip the single-frame latency leg")
    ap.add_argument("--no-shim-latency", action="store_true",
                    help="skip the drop-in C++ shim's per-call latency leg (a child process)")
    ap.add_argument("--no-host-stream", action="store_true", help="skip the host-streamed throughput leg")
    ap.add_argument("--host-steps", type=int, default=30, help="timed steps of the host-streamed leg")
    ap.add_argument("--h2d-mode", choices=["1d", "2d", "kernel"], default="kernel",
                    help="host-streamed leg: upload padded frames (1d DMA), unpadded rows into the padded pitch "
                         "(2d DMA rectangle: 0.13 GB/s on the box, tools/h2d_bench.py), or unpadded rows by a copy "
                         "kernel reading pinned host memory (54 GB/s)")
    ap.add_argument("--h2d-kernel-wgs", type=int, default=48,
                    help="workgroups of the --h2d-mode kernel copy (48: 80%% of the link peak in the pipeline, "
                         "16 / 32 / 64 / 96: 41 / 69 / 75 / 66%%)")
    ap.add_argument("--no-h2d-priority", dest="h2d_priority", action="store_false",
                    help="host-streamed leg: upload streams at normal priority (default high: the copy kernel's "
                         "workgroups are dispatched ahead of the extraction's)")
    ap.add_argument("--h2d-split", type=int, default=1,
                    help="host-streamed leg: the batch upload in this many parts, each on a copy stream of its own "
                         "(a multiple of the extraction halves; an extraction half waits for its own parts only)")
    ap.add_argument("--spawn", action="store_true", help="use the worker launcher even for --gpus 1")
    ap.add_argument("--split-sequence", action="store_true",
                    help="split ONE synthetic sequence (pool x N frames) into contiguous blocks, one per GPU; "
                         "each rank extracts the frame before its block itself for the boundary pair (SURVEY §8(e))")
    ap.add_argument("--share-device", action="store_true", help=argparse.SUPPRESS)  # tests: every rank on device 0
    ap.add_argument("--dump-pairs", default=None, help=argparse.SUPPRESS)  # tests: rank r saves batch 0's outputs
    ap.add_argument("--allow-diag", action="store_true",
                    help="run even with diagnostic ORBX_* variables set (phase clocks, library variants); "
                         "the line then carries them and is not a valid measurement")
    ap.add_argument("--stub-worker", action="store_true", help=argparse.SUPPRESS)  # launcher tests (CPU)
    a = ap.parse_args(argv)
    if a.match_order is None:
        a.match_order = "bow,init,top2" if (a.bow or a.bow_match) else "init,top2,bow"
    return a


# ORBX_* variables the library reads (INTEGRATION.md "Environment variables").
# Tuning: select among bit-exact code paths; allowed, and stamped into the line.
ENV_TUNING = {"ORBX_TIMING", "ORBX_EXTRACT_GRAPH", "ORBX_EXTRACT_ORDER", "ORBX_PYR_PLAN", "ORBX_QT_GENERIC",
              "ORBX_PROJ_ROUNDS", "ORBX_TOP2_VALU", "ORBX_VOC_GL", "ORBX_STEREO_GROUPS",
              "ORBX_BOW_ROUNDS", "ORBX_PYR_KEEP", "ORBX_QT_SORTED", "ORBX_QT_LDS_KB",
              "ORBX_STAGE_THREAD",
              # the C++ shim's configuration (shim/src/ORBextractor.cc); bench.py does not read them
              "ORBX_DEVICE", "ORBX_SCALE_MODE", "ORBX_PATTERN", "ORBX_HOST_PYRAMID",
              "ORBX_STEREO_THREADS"}
# Diagnostics: phase clocks synchronise after every launch, *_STOP / FAST_TWICE
# skip or repeat work (they only act in -DORBX_DIAG builds), ORBX_LIB_VARIANT
# loads an A/B build of the library. A timed region under any of them is not
# the product's: refused unless --allow-diag.
ENV_DIAG = {"ORBX_LIB_VARIANT", "ORBX_FAST_TWICE", "ORBX_INIT_STOP", "ORBX_STEREO_STOP", "ORBX_VOC_STOP",
            "ORBX_FAST_PROF", "ORBX_PYR_PROF", "ORBX_QT_PROF", "ORBX_INIT_PROF", "ORBX_BOW_PROF", "ORBX_PROJ_PROF",
            "ORBX_EXTRACT_PROF", "ORBX_PYR_PADMOD", "ORBX_STEREO_PROF", "ORBX_PLAN_INFO",
            }


def audit_env(allow_diag: bool, environ=None) -> dict:
    """The ORBX_* variables set for this run (stamped into the JSON line as
    "orbx_env"). Diagnostic or unknown ones end the run unless allow_diag."""
    environ = os.environ if environ is None else environ
    env = {k: v for k, v in sorted(environ.items()) if k.startswith("ORBX_")}
    bad = sorted(k for k in env if k not in ENV_TUNING)
    if bad and not allow_diag:
        raise SystemExit("bench.py: refusing to measure with diagnostic or unknown ORBX_* variables set: "
                         + ", ".join(f"{k}={env[k]}" for k in bad) + " (pass --allow-diag to run anyway; "
                         "the line is then stamped and is not a measurement of the product)")
    return env


def library_audit(L) -> dict:
    """The loaded liborbx build: a -DORBX_DIAG build (orbx_version says 'diag') may skip work."""
    v = L.orbx_version()
    v = v.decode() if isinstance(v, bytes) else str(v)
    return {"version": v, "diag_build": "diag" in v}


# --------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpus() -> int:
    """GPUs this node exposes, counted in a short-lived child process so that
    this (launcher) process never loads the HIP runtime before it spawns the
    workers (tests/test_bench_launcher.py checks its memory map)."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise SystemExit(f"bench.py: could not count GPUs: {r.stderr[-500:]}")
    return int(r.stdout.strip().splitlines()[-1])


def _worker_entry(argv, rank, world, port):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    worker(parse_args(argv))


def launch(args, argv) -> int:
    """One worker process per GPU (spawned before this process makes any GPU
    call); returns the first non-zero worker exit code, or 0."""
    import multiprocessing as mp
    N = args.gpus
    if not args.stub_worker and not args.share_device:
        n = visible_gpus()
        if N > n:
            raise SystemExit(f"bench.py: --gpus {N} but only {n} GPU(s) visible; refusing to oversubscribe")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker_entry, args=(argv, r, N, port), daemon=False) for r in range(N)]
    for p in procs:
        p.start()
    code = 0
    for p in procs:
        p.join()
        if p.exitcode != 0 and code == 0:
            code = p.exitcode if p.exitcode > 0 else 1
            for q in procs:  # a dead rank would leave the others blocked in the barrier
                if q.is_alive():
                    q.terminate()
    return code


def match_order(v):
    names = v.split(",")
    if sorted(names) != ["bow", "init", "top2"]:
        raise argparse.ArgumentTypeError("a permutation of top2,bow,init")
    return v


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    audit_env(args.allow_diag)  # before any worker starts
    if "RANK" not in os.environ and (args.gpus > 1 or args.spawn):
        code = launch(args, argv)
        if code:
            raise SystemExit(code)
        return
    worker(args)


def aggregate(frames_rank: int, wall_rank: float, dist, world: int) -> dict:
    """Whole-job figures: value = frames of all ranks / the slowest rank's time."""
    from orb_slam_cuda_amd import sharding
    wall = sharding.max_over_ranks(wall_rank, dist)
    frames = int(round(sharding.sum_over_ranks(float(frames_rank), dist)))
    per_rank = [frames_rank / wall_rank]
    if dist is not None:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, round(frames_rank / wall_rank, 2))
    return {"value": frames / wall, "wall": wall, "frames": frames, "per_rank": [round(v, 2) for v in per_rank]}


def worker(args):
    from orb_slam_cuda_amd import sharding
    rank, world, local = sharding.rank_info()
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    # control plane only (gloo), initialised before liborbx loads so one HIP runtime is in the process
    dist = sharding.init_control_plane()
    try:
        if args.stub_worker:
            return run_stub(args, rank, world, dist)
        from orb_slam_cuda_amd import _lib
        L = _lib.lib()
        lib_info = library_audit(L)
        if lib_info["diag_build"] and not args.allow_diag:
            raise SystemExit(f"bench.py: refusing to measure a diagnostics build of liborbx ({lib_info['version']}); "
                             "rebuild without -DORBX_DIAG or pass --allow-diag")
        args.audit = {"orbx_env": audit_env(args.allow_diag), "library": lib_info}
        ndev = _lib.device_count()
        if args.share_device:
            local = 0  # tests only: several ranks on one device
        if local >= ndev:
            raise SystemExit(f"bench.py: rank {rank} needs device {local}, only {ndev} visible")
        # the device is selected before ANY allocation, stream or event of this process
        _lib.check(L.orbx_set_device(local))
        cfg = CONFIGS[args.config]
        if cfg.get("stereo"):
            run_stereo(args, cfg, rank, world, local, dist)
        else:
            run_mono(args, cfg, rank, world, local, dist)
    finally:
        if dist is not None:
            dist.destroy_process_group()


def run_stub(args, rank, world, dist):
    """CPU stand-in for the GPU work (launcher tests): rank r 'processes'
    batch x steps frames in (1 + r) x 10 ms; everything else is the real
    control plane and reporting path."""
    from orb_slam_cuda_amd import sharding
    cfg = CONFIGS[args.config]
    # what rank r would stream: its own sequence (seed) of frames of the config's shape
    mine = {"rank": rank, "seed": sharding.sequence_seed(rank), "frame": f"{cfg['W']}x{cfg['H']}",
            "nfeatures": cfg["nfeatures"], "frames": args.batch * args.steps}
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (1 + rank))
    wall = time.perf_counter() - t0
    agg = aggregate(args.batch * args.steps, wall, dist, world)
    ranks = [mine]
    if dist is not None:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(agg["value"], 2), "unit": "frames/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "per_rank_frames_per_s": agg["per_rank"],
                          "frames_total": agg["frames"], "job_wall_s": round(agg["wall"], 6), "ranks": ranks,
                          "config": {"workload": cfg["workload"]}, "data": "stub (no GPU work)",
                          "orbx_env": audit_env(args.allow_diag)}), flush=True)


# --------------------------------------------------------------------------- mono pipeline
class MonoPipeline:
    """The C3 / C5 step: extraction of a batch on S streams, matching of the
    same batch against t-1 on the matching stream, overlapping the next
    batch's extraction. Input either from a resident device pool (default)
    or from pinned host memory (host=True: H2D per batch on a copy stream,
    results copied back on a second one)."""

    NS = 3  # output sets: batch k writes set k % 3

    def __init__(self, args, cfg, local, frames_pool, host=False, need_events=True, boundary=False, halo=None):
        import orb_slam_cuda_amd as pkg
        from orb_slam_cuda_amd import _lib
        self.args, self.cfg, self.host = args, cfg, host
        self.L, self.check, self._lib = _lib.lib(), _lib.check, _lib
        W, H, NF, B = cfg["W"], cfg["H"], cfg["nfeatures"], args.batch
        self.W, self.H, self.B = W, H, B
        self.pitch = pitch = (W + 63) & ~63
        self.fbytes = H * pitch
        npool = len(frames_pool)
        if npool % B:
            raise SystemExit("--pool must be a multiple of --batch")
        self.nbatches = npool // B
        if host:
            # 1d: the pool held at the device pitch (padded rows cross the link);
            # 2d / kernel: unpadded rows, expanded to the pitch by the copy
            self.h2d_mode = args.h2d_mode
            hp = pitch if self.h2d_mode == "1d" else W
            self.h_fbytes = H * hp
            self.h_pool = _lib.HostArray((npool, H, hp), np.uint8)
            self.h_pool.a[:, :, :W] = frames_pool
            self.d_in = [_lib.DeviceArray(B * self.fbytes) for _ in range(self.NS)]  # input ring
        else:
            self.d_pool = _lib.DeviceArray(npool * self.fbytes)
            chunk = np.zeros((B, H, pitch), np.uint8)
            for b in range(self.nbatches):
                chunk[:, :, :W] = frames_pool[b * B:(b + 1) * B]
                self.d_pool.upload(chunk, b * B * self.fbytes)
        S = args.split
        if S < 1 or B % S:
            raise SystemExit("--split must divide --batch")
        self.S, self.BS = S, B // S
        self.exts = [pkg.ORBextractor(*ext_params(cfg), W, H, device=local, max_batch=self.BS) for _ in range(S)]
        # the stages' launch order for this pipeline (results do not depend on
        # it): the library default, or "pbfqo" when the matching stream also runs
        # ComputeBoW + SearchByBoW (C3 + BoW 136.1 / 133.3 k vs 123.7 / 123.7 k
        # with the default); --stage-order overrides
        self.stage_order = args.stage_order or ("pbfqo" if (args.bow or args.bow_match) else "")
        if self.stage_order:
            for ex in self.exts:
                ex.set_stage_order(self.stage_order)
        self.cap = cap = self.exts[0].frame_capacity
        NS = self.NS
        DA = _lib.DeviceArray
        self.d_kps = [DA((B + 1) * cap * KP) for _ in range(NS)]
        self.d_desc = [DA((B + 1) * cap * DS) for _ in range(NS)]
        self.d_counts = [DA((B + 1) * 4) for _ in range(NS)]
        for d in self.d_counts:
            d.zero()
        self.matcher = pkg.ORBmatcher(0.9, True, device=local, max_pairs=B, max_kps=cap)
        self.d_bi, self.d_bd, self.d_sd, self.d_m12 = ([DA(B * cap * 4) for _ in range(NS)] for _ in range(4))
        self.d_nm = [DA(B * 4) for _ in range(NS)]
        if host:
            HA = _lib.HostArray
            self.h_kps = [HA(B * cap * KP, np.uint8) for _ in range(NS)]
            self.h_desc = [HA(B * cap * DS, np.uint8) for _ in range(NS)]
            self.h_counts = [HA(B, np.int32) for _ in range(NS)]
            self.h_m12 = [HA(B * cap, np.int32) for _ in range(NS)]
            self.h_nm = [HA(B, np.int32) for _ in range(NS)]
            hp = 1 if args.h2d_priority else None
            self.s_h2d, self.s_d2h = _lib.Stream(hp), _lib.Stream()
            # --h2d-split N: the upload in N parts on N copy streams (half h waits for its own parts)
            nparts = args.h2d_split if not args.serial else 1
            if nparts < 1 or (nparts > 1 and (nparts % S or B % nparts)):
                raise SystemExit(f"bench.py: --h2d-split {nparts} must divide the batch and be a multiple of --split")
            self.s_h2ds = [self.s_h2d] + [_lib.Stream(hp) for _ in range(nparts - 1)]
        prio = 1 if args.priority else None
        mmask = emask = None
        if args.match_cus and not args.serial:
            mmask, emask = cu_masks(args.match_cus, args.cu_exclusive)
        self.s_exts = [_lib.Stream(prio, emask) for _ in range(S)]
        self.s_ext = self.s_exts[0]
        # the host-streamed leg keeps normal priority: there the high-priority
        # matcher starves the copy streams (32.6 k vs 46.1 k frames/s)
        mprio = 0 if args.priority else (1 if args.match_priority and not host else None)
        self.s_match = _lib.Stream(mprio, mmask) if not args.serial else self.s_ext
        self.two_match = (args.match_streams == 2 and not args.serial and not args.no_match
                          and args.carry == "match" and not host)
        self.s_init = _lib.Stream(mprio, mmask) if self.two_match else self.s_match
        self.bounds = _lib.GridBounds(0.0, float(W), 0.0, float(H))
        self.voc = None
        self.bow_match = args.bow_match and not host
        if (args.bow or args.bow_match) and not host:
            from orb_slam_cuda_amd.synth import synthetic_vocabulary
            self.voc = pkg.ORBVocabulary.from_arrays(synthetic_vocabulary(10, 6, seed=1), device=local)
            # BoW of slots 0..B (slot 0 = frame t-1 of the batch's first frame) when
            # SearchByBoW matches every frame against its predecessor as the reference keyframe
            NB1 = B + 1
            self.d_bw, self.d_bn, self.d_fn, self.d_fi, self.d_fnn = (DA(NB1 * cap * 4), DA(NB1 * 4),
                                                                      DA(NB1 * cap * 4), DA(NB1 * cap * 4),
                                                                      DA(NB1 * 4))
            self.d_bv = DA(NB1 * cap * 8)
            self.d_fo = DA(NB1 * (cap + 1) * 4)
            self.d_vw = (DA(NB1 * cap * 4), DA(NB1 * cap * 4), DA(NB1 * cap * 8))
            if self.bow_match:
                self.bow_matcher = pkg.ORBmatcher(0.7, True, device=local, max_pairs=B, max_kps=cap)
                self.d_bow_out, self.d_bow_nm = DA(B * cap * 4), DA(B * 4)
        self.need_events = need_events
        self.ev = {}
        # --split-sequence: the first batch of every pass over the pool gets its
        # slot 0 (frame t-1 of the block's first frame) by extracting the frame
        # before the block (`halo`) on the matching stream, or an empty frame for
        # the sequence's first block, instead of the carry of the pool's last frame
        self.boundary = boundary and not host
        if self.boundary:
            self.halo_ext = pkg.ORBextractor(*ext_params(cfg), W, H, device=local, max_batch=1)
            self.d_halo = None
            if halo is not None:
                hb = np.zeros((H, pitch), np.uint8)
                hb[:, :W] = halo
                self.d_halo = DA(self.fbytes)
                self.d_halo.upload(hb)
            self.d_zero = DA(16)
            self.d_zero.zero()

    def _event(self, name, k):
        e = self.ev.get((name, k))
        if e is None:
            e = self.ev[(name, k)] = self._lib.Event()
        return e

    def alloc_events(self, total):
        E = self._lib.Event
        n_ev = 13  # 6 extraction stage marks + 3 matching marks + 2 BoW marks + init start + BoW match end
        self.evsets = [[E() for _ in range(n_ev)] for _ in range(total)] if self.need_events else None
        self.ev_ext = [E() for _ in range(total)]
        self.ev_done = [E() for _ in range(total)]
        self.ev_done2 = [E() for _ in range(total)]
        self.ev_carry = [E() for _ in range(total)]
        self.ev_part = [[E() for _ in range(self.S)] for _ in range(total)]
        if self.host:
            self.ev_in = [[E() for _ in self.s_h2ds] for _ in range(total)]
            self.ev_out = [E() for _ in range(total)]

    def frames_ptr(self, k):
        if self.host:
            return self.d_in[k % self.NS].ptr
        return self.d_pool.ptr + (k % self.nbatches) * self.B * self.fbytes

    def step(self, k):
        """Batch k: extraction on the extraction streams; carry copy and
        matching of the same batch on s_match, overlapping the extraction of
        batch k+1 (--serial: one stream). Extraction k waits for matching k-3
        (the last reader of set k % 3); matching k waits for extraction k."""
        a, L, check = self.args, self.L, self.check
        vp = C.c_void_p
        B, BS, cap, NS = self.B, self.BS, self.cap, self.NS
        b, nb = k % NS, (k + 1) % NS
        evs = self.evsets[k] if self.evsets is not None else None
        if self.host:
            # H2D of batch k into input slot k % 3, after extraction k-3 read it
            src = self.h_pool.ptr + (k % self.nbatches) * B * self.h_fbytes
            parts = len(self.s_h2ds)
            for i, sh in enumerate(self.s_h2ds):
                if k >= NS:
                    sh.wait(self.ev_ext[k - NS])
                lo, hi = i * B // parts, (i + 1) * B // parts
                dst = vp(self.d_in[k % NS].ptr + lo * self.fbytes)
                hsrc = vp(src + lo * self.h_fbytes)
                if self.h2d_mode == "1d":
                    check(L.orbx_memcpy_htod_async(dst, hsrc, (hi - lo) * self.fbytes, sh.s))
                elif self.h2d_mode == "2d":
                    check(L.orbx_memcpy2d_htod_async(dst, self.pitch, hsrc, self.W, self.W, (hi - lo) * self.H, sh.s))
                else:
                    check(L.orbx_copy2d_kernel_async(dst, self.pitch, hsrc, self.W, self.W, (hi - lo) * self.H,
                                                     a.h2d_kernel_wgs, sh.s))
                self.ev_in[k][i].record(sh)
        fp = self.frames_ptr(k)
        for h, (ex, se) in enumerate(zip(self.exts, self.s_exts)):
            if h == 0 and evs is not None:
                arr = (C.c_void_p * 6)(*[e.e.value for e in evs[:6]])
                check(L.orbx_set_stage_events(ex.handle, arr))
            sv = se if not a.serial else self.s_ext
            if self.host:
                nparts = len(self.s_h2ds)
                per = nparts // self.S
                for i in range(h * per, (h + 1) * per) if nparts > 1 else (0,):
                    sv.wait(self.ev_in[k][i])  # the parts holding half h's frames
            if not a.serial and k >= NS:
                sv.wait(self.ev_done[k - NS])  # matching k-3 was the last reader of set k % 3
                if self.two_match:
                    sv.wait(self.ev_done2[k - NS])
                if self.host:
                    sv.wait(self.ev_out[k - NS])  # and the read-back of batch k-3
            check(L.orbx_extract_batch(ex.handle, vp(fp + h * BS * self.fbytes), BS, self.fbytes, self.pitch,
                                       vp(self.d_kps[b].ptr + (1 + h * BS) * cap * KP),
                                       vp(self.d_desc[b].ptr + (1 + h * BS) * cap * DS),
                                       vp(self.d_counts[b].ptr + 4 * (1 + h * BS)), sv.s))
            if h > 0 and not a.serial:
                self.ev_part[k][h].record(se)
                self.s_ext.wait(self.ev_part[k][h])

        def carry(st):
            check(L.orbx_memcpy_dtod_async(vp(self.d_kps[nb].ptr), vp(self.d_kps[b].ptr + B * cap * KP), cap * KP, st.s))
            check(L.orbx_memcpy_dtod_async(vp(self.d_desc[nb].ptr), vp(self.d_desc[b].ptr + B * cap * DS), cap * DS,
                                           st.s))
            check(L.orbx_memcpy_dtod_async(vp(self.d_counts[nb].ptr), vp(self.d_counts[b].ptr + B * 4), 4, st.s))

        s_match, s_init = self.s_match, self.s_init
        if self.boundary and k == 0:
            self.first_slot(0, s_match)  # batch 0's slot 0, ahead of its matching on this stream
        if self.boundary and (k + 1) % self.nbatches == 0:
            pass  # the next batch starts a pass over the pool: its slot 0 is the boundary frame (below)
        elif a.carry == "ext" or a.serial:
            # slot 0 of set (k+1) % 3 was last read by matching k-2
            if k >= 2 and not a.serial:
                self.s_ext.wait(self.ev_done[k - 2])
            carry(self.s_ext)
        self.ev_ext[k].record(self.s_ext)
        if not a.serial:
            s_match.wait(self.ev_ext[k])
        if self.boundary and (k + 1) % self.nbatches == 0:
            if self.two_match and k >= 2:
                s_match.wait(self.ev_done2[k - 2])
            self.first_slot(nb, s_match)  # in order after matching k-2, the last reader of set (k+1) % 3
            self.ev_carry[k].record(s_match)
        elif a.carry == "match" and not a.serial:
            if self.two_match and k >= 2:
                s_match.wait(self.ev_done2[k - 2])  # SearchForInitialization k-2 also read set (k+1) % 3
            carry(s_match)  # in order after matching k-2, the last reader of set (k+1) % 3
            self.ev_carry[k].record(s_match)
        def bow():
            if self.voc is not None:
                evs[9].record(s_match)
                # Frame::ComputeBoW (src/Frame.cc:394-401, levelsup 4) of the batch's frames
                # (slots 1..B; with --bow-match also slot 0, the reference keyframe of slot 1)
                s0 = 0 if self.bow_match else 1
                check(L.orbv_transform_batch(self.voc.handle, vp(self.d_desc[b].ptr + s0 * cap * DS), cap * DS,
                                             vp(self.d_counts[b].ptr + 4 * s0), B + 1 - s0, cap, 4, vp(self.d_bw.ptr),
                                             vp(self.d_bv.ptr), vp(self.d_bn.ptr), vp(self.d_fn.ptr), vp(self.d_fo.ptr),
                                             vp(self.d_fi.ptr), vp(self.d_fnn.ptr), vp(self.d_vw[0].ptr),
                                             vp(self.d_vw[1].ptr), vp(self.d_vw[2].ptr), s_match.s), vocabulary=True)
                evs[10].record(s_match)
                if self.bow_match:
                    # SearchByBoW(KF, F) of frame t against frame t-1 as the reference keyframe, every
                    # keyframe feature with a MapPoint (Tracking::TrackReferenceKeyFrame, ratio 0.7,
                    # src/Tracking.cc:839-842), all B pairs in one launch
                    ofs = lambda d, k, pitch, size: vp(d.ptr + k * pitch * size)
                    sides = []
                    for side in (0, 1):
                        sides += [ofs(self.d_kps[b], side, cap, KP), ofs(self.d_desc[b], side, cap, DS),
                                  ofs(self.d_counts[b], side, 1, 4), None, ofs(self.d_fn, side, cap, 4),
                                  ofs(self.d_fo, side, cap + 1, 4), ofs(self.d_fi, side, cap, 4),
                                  ofs(self.d_fnn, side, 1, 4)]
                    check(L.orbm_search_by_bow_batch(self.bow_matcher.handle, B, cap, cap, *sides, C.c_float(0.7), 1, 0,
                                                     vp(self.d_bow_out.ptr), vp(self.d_bow_nm.ptr), s_match.s),
                          matcher=True)
                    evs[12].record(s_match)
        def top2():
            if evs is not None:
                evs[6].record(s_match)
            if not a.no_match:
                # query = frame t (slots 1..B), candidates = frame t-1 (slots 0..B-1)
                check(L.orbm_hamming_top2(self.matcher.handle, vp(self.d_desc[b].ptr + cap * DS), cap * DS,
                                          vp(self.d_counts[b].ptr + 4), cap, vp(self.d_desc[b].ptr), cap * DS,
                                          vp(self.d_counts[b].ptr), B, vp(self.d_bi[b].ptr), vp(self.d_bd[b].ptr),
                                          vp(self.d_sd[b].ptr), s_match.s), matcher=True)
                if evs is not None:
                    evs[7].record(s_match)
        def init():
            if not a.no_match:
                if self.two_match:  # after batch k's extraction and the carry into its slot 0 (step k-1)
                    s_init.wait(self.ev_ext[k])
                    if k >= 1:
                        s_init.wait(self.ev_carry[k - 1])
                if evs is not None:
                    evs[11].record(s_init)
                check(L.orbm_search_for_initialization_batch(
                    self.matcher.handle, vp(self.d_kps[b].ptr), vp(self.d_desc[b].ptr), vp(self.d_counts[b].ptr),
                    vp(self.d_kps[b].ptr + cap * KP), vp(self.d_desc[b].ptr + cap * DS), vp(self.d_counts[b].ptr + 4),
                    cap, B, self.bounds, None, 100, C.c_float(0.9), 1, vp(self.d_m12[b].ptr), vp(self.d_nm[b].ptr),
                    s_init.s), matcher=True)
            if evs is not None:
                evs[8].record(s_init)
        stages = {"bow": bow, "top2": top2, "init": init}
        for name in a.match_order.split(","):
            stages[name]()
        self.ev_done[k].record(s_match)
        if self.two_match:
            self.ev_done2[k].record(s_init)
        if self.host:
            # read back batch k's keypoints, descriptors, counts and matches
            d2h = self.s_d2h
            d2h.wait(self.ev_done[k])
            cp = lambda dst, src, n: check(L.orbx_memcpy_dtoh_async(vp(dst), vp(src), n, d2h.s))
            cp(self.h_kps[b].ptr, self.d_kps[b].ptr + cap * KP, B * cap * KP)
            cp(self.h_desc[b].ptr, self.d_desc[b].ptr + cap * DS, B * cap * DS)
            cp(self.h_counts[b].ptr, self.d_counts[b].ptr + 4, B * 4)
            if not a.no_match:
                cp(self.h_m12[b].ptr, self.d_m12[b].ptr, B * cap * 4)
                cp(self.h_nm[b].ptr, self.d_nm[b].ptr, B * 4)
            self.ev_out[k].record(d2h)

    def first_slot(self, b, st):
        """Slot 0 of output set b for a block's first batch: the boundary frame's
        keypoints, descriptors and count (extracted here), or count 0."""
        vp = C.c_void_p
        if self.d_halo is None:
            self.check(self.L.orbx_memcpy_dtod_async(vp(self.d_counts[b].ptr), vp(self.d_zero.ptr), 4, st.s))
            return
        self.check(self.L.orbx_extract_batch(self.halo_ext.handle, vp(self.d_halo.ptr), 1, self.fbytes, self.pitch,
                                             vp(self.d_kps[b].ptr), vp(self.d_desc[b].ptr), vp(self.d_counts[b].ptr),
                                             st.s))

    def sync_all(self):
        for se in self.s_exts:
            se.synchronize()
        self.s_match.synchronize()
        self.s_init.synchronize()
        if self.host:
            for sh in self.s_h2ds:
                sh.synchronize()
            self.s_d2h.synchronize()

    def run(self, warmup, steps, dist):
        total = warmup + steps
        self.alloc_events(total)
        for k in range(warmup):
            self.step(k)
        self.sync_all()
        if dist is not None:
            dist.barrier()
        self.sync_all()
        t0 = time.perf_counter()
        for k in range(warmup, total):
            self.step(k)
        t_issue = time.perf_counter()
        self.sync_all()
        t1 = time.perf_counter()
        if dist is not None:
            dist.barrier()
        self.total = total
        return t1 - t0, t_issue - t0

    def check_status(self):
        bad = {f"extractor{i}": e.status() for i, e in enumerate(self.exts)}
        bad["matcher"] = self.matcher.status()
        if getattr(self, "bow_match", False):
            bad["bow_matcher"] = self.bow_matcher.status()
        bad = {k: v for k, v in bad.items() if v}
        if bad:
            raise RuntimeError(f"device status words set after the timed region: {bad}")

    def last_set(self):
        return (self.total - 1) % self.NS


def run_mono(args, cfg, rank, world, local, dist):
    from orb_slam_cuda_amd import sharding
    from orb_slam_cuda_amd.synth import SynthSequence, SynthStream
    W, H, NF, B = cfg["W"], cfg["H"], cfg["nfeatures"], args.batch
    pool = max(B, (args.pool // B) * B)
    halo = None
    if args.split_sequence:
        # ONE sequence of pool x world frames; this rank's pool is its block
        stream = SynthStream(sharding.sequence_seed(0), W, H)
        block, prev = sharding.split_sequence(pool * world, rank, world)
        frames = stream.frames(block)
        halo = stream.frame(prev) if prev is not None else None
    else:
        frames = SynthSequence(sharding.sequence_seed(rank), W, H).frames(pool)
    pipe = MonoPipeline(args, cfg, local, frames, boundary=args.split_sequence, halo=halo)
    SUB = max(1, args.batches_per_step)
    wall_rank, issue = pipe.run(args.warmup * SUB, args.steps * SUB, dist)
    agg = aggregate(B * SUB * args.steps, wall_rank, dist, world)
    pipe.check_status()
    if args.dump_pairs:
        dump_batch0(args, pipe, rank, block if args.split_sequence else None, prev if args.split_sequence else None)
    BS, S, cap = pipe.BS, pipe.S, pipe.cap
    timed = pipe.evsets[args.warmup * SUB:]
    ev_ms = timed[0][0].elapsed_ms(timed[-1][8])
    from orb_slam_cuda_amd import _lib as _stage_lib
    names = STAGES
    ext_stages = names[:5]
    launch_order = _stage_lib.stage_order(pipe.exts[0].handle)  # stage event i + 1 closes launch_order[i]
    STAGES_RUN = ext_stages + (["hamming_top2", "search_init"] if not args.no_match else []) \
        + (["bow_transform"] if (args.bow or args.bow_match) else []) + (["bow_match"] if args.bow_match else [])
    # per-stage average durations over the timed steps (ms per launch-group, BS frames),
    # each bracketed by events on the stream its kernels run on
    st = {s: 0.0 for s in STAGES_RUN}
    for evs in timed:
        for i, s in enumerate(launch_order):
            st[s] += evs[i].elapsed_ms(evs[i + 1])
        if args.bow or args.bow_match:
            st["bow_transform"] += evs[9].elapsed_ms(evs[10])
        if args.bow_match:
            st["bow_match"] += evs[10].elapsed_ms(evs[12])
        if not args.no_match:
            st["hamming_top2"] += evs[6].elapsed_ms(evs[7])
            st["search_init"] += evs[11].elapsed_ms(evs[8])
    st = {s: v / len(timed) for s, v in st.items()}  # per batch (per launch group)
    ls = pipe.last_set()
    nm = pipe.d_nm[ls].download(B, np.int32)
    cnt = pipe.d_counts[ls].download(B + 1, np.int32).astype(np.int64)
    nkp_mean = float(cnt[1:].mean())
    # quadtree tie-rule exposure over the last batch (orbx_get_tie_stats)
    ties = np.concatenate([e.tie_stats(0, BS) for e in pipe.exts])  # (B, L, 3)
    tie = {"events_per_frame": round(float(ties[:, :, 0].sum(1).mean()), 2),
           "kept_keypoints_per_frame": round(float(ties[:, :, 2].sum(1).mean()), 1),
           "fraction_of_kept": round(float(ties[:, :, 2].sum() / max(1, cnt[1:].sum())), 4),
           "levels_with_event_frac": round(float((ties[:, :, 0] > 0).mean()), 3),
           "frames": int(len(ties))}
    ab = algorithmic_bytes(W, H, nkp_mean, ext_params(cfg)[2], ext_params(cfg)[1])
    extract_ms = sum(st[s] for s in ext_stages)
    dominant = max(STAGES_RUN, key=lambda s: st[s])
    # roofline of the pyramid+FAST pass: the kernels that run it
    pf_ms = st["pyramid"] + st["fast_grid"]
    pf_gbs = ab["pyr_fast_pass"] * BS / (pf_ms * 1e-3) / 1e9
    hbm_stages = {"pyramid": ab["pyramid"], "blur": ab["blur"], "fast_grid": ab["fast_grid"],
                  "orient_brief": ab["orient_brief"]}
    # the roofline kernel: FAST, the longest extraction kernel alone (its event
    # time in the pipelined run matches its rocprofv3 average)
    rk = "fast_grid"
    traffic = pmc_bytes(KERNELS[rk])
    ach = hbm_stages[rk] * BS / (st[rk] * 1e-3) / 1e9
    roof = {"kernel": KERNELS[rk], "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": "profiles/pmc_traffic.json: committed FETCH_SIZE/WRITE_SIZE passes (tools/pmc_passes.sh),"
                              " not measured in this run",
            "algorithmic_bytes_per_launch": int(hbm_stages[rk] * BS),
            "avg_launch_ms": round(st[rk], 4)}
    # the same kernel run alone (--serial): its committed rocprofv3 average, so
    # the pipelined event time's share of waiting for CUs beside the other
    # streams (which grows as the pipeline overlaps more) can be told apart
    alone = serial_avg_ms(KERNELS[rk], BS)
    if alone:
        roof["alone"] = {"avg_launch_ms": round(alone[0], 4),
                         "achieved": round(hbm_stages[rk] * BS / (alone[0] * 1e-3) / 1e9, 1),
                         "frac": round(hbm_stages[rk] * BS / (alone[0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "source": alone[1] + " (committed --serial rocprofv3 summary, not measured in this run)"}
    # the same kernel against VALU issue (it is latency / issue bound, not HBM bound):
    # its committed SQ_INSTS_VALU per launch over this run's launch time
    vi = sq_valu(KERNELS[rk])
    if vi and BS == SQ_LAUNCH_FRAMES:
        roof["valu_issue"] = {"wave_instr_per_launch": int(vi), "achieved_T_per_s": round(vi / (st[rk] * 1e-3) / 1e12, 4),
                              "peak_T_per_s": VALU_ISSUE_PEAK_T, "frac": round(vi / (st[rk] * 1e-3) / 1e12 / VALU_ISSUE_PEAK_T, 4),
                              "source": "profiles/sq_valu.json: committed SQ_INSTS_VALU pass (tools/pmc_sq.sh, serial "
                                        "run), not measured in this run; the time is this run's"}
    # the dense matcher runs on the matrix cores: algorithmic work = one 256-element +-1 dot
    # product per (query, candidate) pair = 512 FLOP, against the dense FP4 MFMA peak; the
    # per-pair top-2 update (v_min + v_med3) is reported against the VALU lane-op peak
    match_roof = None
    if not args.no_match and st["hamming_top2"] > 0:
        pairs = int((cnt[1:] * cnt[:-1]).sum())
        sec = st["hamming_top2"] * 1e-3
        tf = 512.0 * pairs / sec / 1e12
        match_roof = {"kernel": KERNELS["hamming_top2"], "bound": "mfma", "unit": "TFLOP/s",
                      "achieved": round(tf, 1), "peak": MFMA_FP4_PEAK_TFLOPS, "frac": round(tf / MFMA_FP4_PEAK_TFLOPS, 4),
                      "dtype": "fp4 e2m1 (+-1 bits, exact)", "top2_valu_frac": round(2.0 * pairs / sec / 1e12 / VALU_PEAK_TOPS, 4),
                      "traffic": pmc_bytes(KERNELS["hamming_top2"]),
                      "pairs_per_launch": pairs, "pairs_per_s": round(pairs / sec, 1),
                      "avg_launch_ms": round(st["hamming_top2"], 4)}
    bow_nm = (round(float(pipe.d_bow_nm.download(B, np.int32).mean()), 1) if args.bow_match else None)
    # release the timed pipeline (its streams hold hardware queues) before the extra legs
    pipe.sync_all()
    del pipe, timed
    import gc
    gc.collect()
    lat = host = cpu = cpu1 = tie_rule = None
    solo = world == 1
    shim_lat = shim_match_lat = None
    if rank == 0 and solo and not args.no_latency:
        lat = latency_leg(cfg, local, frames[:32], args.no_match)
        if not args.no_shim_latency and (W, H, NF) == (1241, 376, 2000) and ext_params(cfg)[2] == 8:
            shim_lat = shim_latency_leg(frames[:32], W, H, local)
            if not args.no_match:
                shim_match_lat = shim_matcher_latency_leg(local)
    if rank == 0 and solo and not args.no_host_stream and args.host_steps > 0:
        host = host_stream_leg(args, cfg, local, frames)
    if rank == 0 and solo and args.cpu_sample > 0:
        sample = frames if args.cpu_sample <= len(frames) else seq_cpu(rank, W, H, args.cpu_sample)
        cpu1 = cpu_baseline(sample, cfg, args.cpu_sample, args.no_match)
        nt = args.cpu_threads if args.cpu_threads > 0 else cpu_threads_default()
        cpu = cpu_baseline(sample, cfg, args.cpu_sample, args.no_match, nt) if nt > 1 else cpu1
        if lat is not None:
            lat["cpu_oracle"] = cpu_latency(frames[:220], cfg, args.no_match)
        tie_rule = cpu_tie_rule_study(frames[:8], cfg)

    if rank == 0:
        workload = (cfg["workload"] if not args.no_match
                    else "C2" + cfg["workload"].split(", extract")[0][2:] + ", extract only"
                    if cfg["workload"].startswith("C3") else cfg["workload"].split(", extract")[0] + ", extract only")
        if args.split_sequence:
            workload += f"; ONE sequence of {pool * world} frames split into {world} contiguous blocks"
        out = {
            "metric": METRIC, "value": round(agg["value"], 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(agg["wall"] / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded shapes + noise sequence, orb_slam_cuda_amd/synth.py), "
                    f"{pool} resident frames per GPU cycled batch by batch",
            "config": {"workload": workload + (" + Frame::ComputeBoW (synthetic k10 L6 vocabulary)" if (args.bow or args.bow_match) else "")
                                   + (" + SearchByBoW(KF t-1, F t)" if args.bow_match else ""),
                       "frame": f"{W}x{H}", "nfeatures": NF, "nlevels": ext_params(cfg)[2],
                       "scale_factor": ext_params(cfg)[1], "fast_thresholds": list(ext_params(cfg)[3:]),
                       "frames_per_step_per_gpu": B * SUB, "batches_per_step": SUB, "frames_per_batch": B,
                       "resident_pool_frames": pool,
                       "parallelism": (f"sequence split x{world} (contiguous blocks, boundary frame re-extracted per rank)"
                                       if args.split_sequence else f"frame-sharded x{world}") + ", one process per GPU, no collectives",
                       "streams": 1 if args.serial else S + 1, "frames_per_extract_launch": BS,
                       "match_stream_priority": ("low" if args.priority else "high" if args.match_priority
                                                 else "normal"),
                       "stage_order": "".join(c[0] if c != "fast_grid" else "f" for c in launch_order),
                       "match_order": args.match_order},
            "per_rank_frames_per_s": agg["per_rank"],
            "roofline": roof,
            "match_roofline": match_roof,
            "cpu_baseline": cpu,
            "cpu_baseline_1thread": cpu1,
            "latency": lat,
            "shim_latency": shim_lat,
            "shim_matcher_latency": shim_match_lat,
            "host_stream": host,
            "quadtree_tie_straddle": tie,
            "tie_rule_disagreement": tie_rule,
            "pyr_fast_pass_hbm_gbs": round(pf_gbs, 1),
            "dominant_kernel": KERNELS[dominant],
            "dominant_kernel_basis": "HIP-event stage time of the pipelined step (a stage's events also hold its "
                                     "workgroups' wait for compute units beside the other streams)",
            "rocprof_ranking": rocprof_ranking(),
            "stage_ms_per_batch": {s: round(v, 4) for s, v in st.items()},
            "extract_only_frames_per_s": round(BS / (extract_ms * 1e-3), 1),
            "host_issue_ms_per_step": round(issue / args.steps * 1e3, 4), "event_ms_per_step": round(ev_ms / args.steps, 4),
            "keypoints_per_frame": round(nkp_mean, 1),
            "init_matches_per_pair": round(float(nm.mean()), 1),
            "bow_matches_per_pair": bow_nm,
            **args.audit,
        }
        print(json.dumps(out), flush=True)


def dump_batch0(args, pipe, rank, block, prev):
    """Tests only (--dump-pairs DIR): batch 0's outputs of this rank (the run
    must be one batch long so that output set 0 still holds them)."""
    import orb_slam_cuda_amd as pkg
    B, cap = pipe.B, pipe.cap
    if pipe.total != 1:
        raise SystemExit("--dump-pairs needs exactly one batch (--steps 1 --warmup 0 --batches-per-step 1)")
    os.makedirs(args.dump_pairs, exist_ok=True)
    np.savez(os.path.join(args.dump_pairs, f"rank{rank}.npz"),
             counts=pipe.d_counts[0].download(B + 1, np.int32),
             kps=pipe.d_kps[0].download((B + 1) * cap, pkg.KP_DTYPE).reshape(B + 1, cap),
             desc=pipe.d_desc[0].download((B + 1, cap, 32), np.uint8),
             m12=pipe.d_m12[0].download((B, cap), np.int32), nm=pipe.d_nm[0].download(B, np.int32),
             bi=pipe.d_bi[0].download((B, cap), np.int32), bd=pipe.d_bd[0].download((B, cap), np.int32),
             sd=pipe.d_sd[0].download((B, cap), np.int32),
             block=np.array([block.start, block.stop] if block is not None else [-1, -1]),
             prev=np.array([-1 if prev is None else prev]))


SQ_LAUNCH_FRAMES = 32   # frames per extraction launch of the committed SQ counter run
VALU_ISSUE_PEAK_T = 1.2288  # wave64 VALU instructions/s: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles


def cu_masks(spec, exclusive, ncu=None):
    """CU masks (lists of u32 words) for --match-cus: the matching stream's and
    (exclusive) the extraction streams' complement, or None for the latter."""
    ncu = ncu or 256  # MI355X: 8 XCDs x 32 CUs
    kind, _, val = spec.partition(":")
    k = int(val)
    sel = [(i % k == 0) if kind == "stride" else (i < k) for i in range(ncu)]
    words = lambda bits: [sum(1 << b for b in range(32) if w * 32 + b < ncu and bits[w * 32 + b])
                          for w in range((ncu + 31) // 32)]
    return words(sel), (words([not x for x in sel]) if exclusive else None)


def rocprof_ranking(top=6):
    """Kernels of the newest committed pipelined rocprofv3 summary
    (profiles/rNN_kernel_stats.csv, the default C3 command) by total time:
    the ranking beside the HIP-event one (dominant_kernel)."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_kernel_stats.csv")))
    if not files:
        return None
    rows = list(csv.DictReader(open(files[-1])))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    return {"source": os.path.relpath(files[-1], ROOT) + " (committed, not measured in this run)",
            "by_total_time": [{"kernel": r["Name"].split("(")[0].replace("void ", "").replace("orbx::", ""),
                               "avg_us": round(float(r["AverageNs"]) / 1e3, 1), "pct": float(r["Percentage"])}
                              for r in rows[:top]]}


def serial_avg_ms(kernel, launch_frames):
    """(average ms, file) of `kernel` in the newest committed --serial rocprofv3
    summary of the default C3 command (profiles/rNN_serial_kernel_stats.csv),
    for launches of SQ_LAUNCH_FRAMES frames only."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_serial_kernel_stats.csv")))
    if not files or launch_frames != SQ_LAUNCH_FRAMES:
        return None
    for r in csv.DictReader(open(files[-1])):
        if r["Name"].split("(")[0].replace("void ", "").replace("orbx::", "").split("<")[0] == kernel.split("<")[0]:
            return float(r["AverageNs"]) / 1e6, os.path.relpath(files[-1], ROOT)
    return None


def sq_valu(kernel):
    """VALU wave-instructions per launch of `kernel` from the committed SQ counters (profiles/)."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "sq_valu.json")))
    except Exception:
        return None
    want = kernel.split(" ")[0]
    return next((v.get("valu_per_launch") for k, v in d.items() if k.split("<")[0] == want), None)


def pmc_bytes(kernel):
    """HBM-side bytes per launch of `kernel` from the committed PMC passes (profiles/)."""
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        pmc = json.load(open(pmc_path))
    except Exception:
        return None
    want = kernel.split(" ")[0]  # profile keys carry template arguments ("fast_cells_kernel<44, false>")
    return next((v.get("bytes_per_launch") for k, v in pmc.items() if k.split("<")[0] == want), None)


def host_stream_leg(args, cfg, local, frames):
    """The C3 pipeline fed from pinned host memory: every batch crosses PCIe
    (H2D on a copy stream, overlapped with the previous batch's compute) and
    its keypoints, descriptors, counts and matches come back (D2H on a second
    copy stream). PCIe-inclusive throughput; never `value`."""
    link = link_peak(cfg, args.batch)
    pipe = MonoPipeline(args, cfg, local, frames, host=True, need_events=False)
    wall, issue = pipe.run(min(args.warmup, 10), args.host_steps, None)
    pipe.check_status()
    B, cap = pipe.B, pipe.cap
    h2d = B * pipe.h_fbytes
    d2h = B * (cap * (KP + DS) + 4) + (0 if args.no_match else B * (cap + 1) * 4)
    h2d_rate = h2d * args.host_steps / wall / 1e9
    return {"value": round(B * args.host_steps / wall, 2), "unit": "frames/s", "steps": args.host_steps,
            "ms_per_step": round(wall / args.host_steps * 1e3, 4),
            "pcie_gb_per_s": round((h2d + d2h) * args.host_steps / wall / 1e9, 2),
            "h2d_gb_per_s": round(h2d_rate, 2), "link": link,
            "h2d_frac_of_link_peak": round(h2d_rate / link["h2d_peak_GBps"], 3) if link.get("h2d_peak_GBps") else None,
            "h2d_mode": args.h2d_mode, "h2d_bytes_per_step": h2d, "d2h_bytes_per_step": d2h,
            "host_issue_ms_per_step": round(issue / args.host_steps * 1e3, 4),
            "h2d_streams": len(pipe.s_h2ds), "h2d_priority": bool(args.h2d_priority),
            "what": f"pool of {len(frames)} frames in pinned host memory, batch uploaded per step, "
                    "keypoints + descriptors + counts" + ("" if args.no_match else " + matches") + " read back"}


def link_peak(cfg, B, reps=20):
    """The box's pinned host<->device copy rates alone (hipMemcpyAsync of one
    padded batch from / to pinned memory, 1 and 2 streams): the ceiling the
    host-streamed leg is compared with."""
    from orb_slam_cuda_amd import _lib
    L = _lib.lib()
    vp = C.c_void_p
    W, H = cfg["W"], cfg["H"]
    nb = B * H * ((W + 63) & ~63)
    h = _lib.HostArray(nb, np.uint8)
    d = _lib.DeviceArray(nb)
    ss = [_lib.Stream(), _lib.Stream()]
    out = {"bytes": nb}
    for name, kind in (("h2d", 0), ("d2h", 1)):
        best = 0.0
        for ns in (1, 2):
            def once():
                for i in range(ns):
                    lo, hi = i * nb // ns, (i + 1) * nb // ns
                    if kind == 0:
                        _lib.check(L.orbx_memcpy_htod_async(vp(d.ptr + lo), vp(h.ptr + lo), hi - lo, ss[i].s))
                    else:
                        _lib.check(L.orbx_memcpy_dtoh_async(vp(h.ptr + lo), vp(d.ptr + lo), hi - lo, ss[i].s))
            once()
            for st in ss:
                st.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                once()
            for st in ss:
                st.synchronize()
            rate = nb * reps / (time.perf_counter() - t0) / 1e9
            out[f"{name}_{ns}stream_GBps"] = round(rate, 2)
            best = max(best, rate)
        out[f"{name}_peak_GBps"] = round(best, 2)
    return out


def latency_leg(cfg, local, frames, no_match, n=200, warm=20):
    """orbx_extract (the synchronous single-image call the reference's
    Tracking makes, src/Frame.cc:246-252) and the host SearchForInitialization,
    median / p99 over n calls after warm calls."""
    import orb_slam_cuda_amd as pkg
    from orb_slam_cuda_amd import _lib
    W, H, NF = cfg["W"], cfg["H"], cfg["nfeatures"]
    L = _lib.lib()
    ext = pkg.ORBextractor(*ext_params(cfg), W, H, device=local)
    cap = ext.frame_capacity
    imgs = [np.ascontiguousarray(f) for f in frames]
    kps = [np.empty(cap, pkg.KP_DTYPE) for _ in imgs]
    desc = [np.empty((cap, 32), np.uint8) for _ in imgs]
    ns = [0] * len(imgs)
    n_c = C.c_int(0)

    def one(i):
        j = i % len(imgs)
        _lib.check(L.orbx_extract(ext.handle, _lib.ptr(imgs[j]), W, H, W, _lib.ptr(kps[j]), cap, _lib.ptr(desc[j]),
                                  C.byref(n_c)))
        ns[j] = n_c.value

    for i in range(warm):
        one(i)
    t = []
    for i in range(n):
        t0 = time.perf_counter()
        one(i)
        t.append(time.perf_counter() - t0)
    t = np.array(t) * 1e3
    out = {"extract_ms": {"median": round(float(np.median(t)), 4), "p99": round(float(np.percentile(t, 99)), 4),
                          "calls": n},
           "what": f"orbx_extract, one host {W}x{H} u8 image in, host keypoints + descriptors out "
                   "(pinned staging, H2D + 5 kernels + D2H as one replayed hipGraph, one sync)"}
    if not no_match:
        m = pkg.ORBmatcher(0.9, True, device=local, max_kps=cap)
        b = _lib.GridBounds(0.0, float(W), 0.0, float(H))
        m12 = np.empty(cap, np.int32)
        nm = C.c_int(0)
        ts = []
        for i in range(warm + n):
            j = i % (len(imgs) - 1)
            k1, d1, k2, d2 = kps[j][:ns[j]], desc[j][:ns[j]], kps[j + 1][:ns[j + 1]], desc[j + 1][:ns[j + 1]]
            prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1), np.float32)
            t0 = time.perf_counter()
            _lib.check(L.orbm_search_for_initialization(m.handle, _lib.ptr(k1), _lib.ptr(d1), len(k1), _lib.ptr(k2),
                                                        _lib.ptr(d2), len(k2), b, _lib.ptr(prev), 100, C.c_float(0.9),
                                                        1, _lib.ptr(m12), C.byref(nm)), matcher=True)
            if i >= warm:
                ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        out["search_init_ms"] = {"median": round(float(np.median(ts)), 4),
                                 "p99": round(float(np.percentile(ts, 99)), 4), "calls": n}
    return out


SHIM_DRIVER = os.path.join(ROOT, "shim", "build", "orbx_shim_driver")


def shim_latency_leg(frames, W, H, local, n=200, warm=20):
    """The drop-in C++ classes as Tracking calls them, per frame: a fresh child
    process (shim/build/orbx_shim_driver --latency) times orbx_extract alone,
    ORBextractor::operator() (src/Frame.cc:246-252; with and without the pinned
    host mvImagePyramid) and the stereo Frame constructor (two extraction
    threads + ComputeStereoMatches, src/Frame.cc:60-128) on the host clock,
    median / p99 over n calls after warm ones. KITTI-shaped mono frames; the
    stereo pairs are synth.stereo_pair's."""
    import subprocess
    import tempfile
    from orb_slam_cuda_amd.synth import stereo_pair
    if not os.path.exists(SHIM_DRIVER):
        return {"error": f"{SHIM_DRIVER} not built (python __graft_entry__.py builds it)"}
    nf = len(frames)
    pairs = [stereo_pair(1000 + i, W, H) for i in range(nf)]
    with tempfile.TemporaryDirectory() as d:
        paths = [os.path.join(d, x) for x in ("mono.u8", "left.u8", "right.u8")]
        np.ascontiguousarray(np.stack(frames), np.uint8).tofile(paths[0])
        np.ascontiguousarray(np.stack([p[0] for p in pairs]), np.uint8).tofile(paths[1])
        np.ascontiguousarray(np.stack([p[1] for p in pairs]), np.uint8).tofile(paths[2])
        env = dict(os.environ, ORBX_DEVICE=str(local))
        try:
            r = subprocess.run([SHIM_DRIVER, "--latency", *paths, str(nf), str(W), str(H), str(n), str(warm)],
                               capture_output=True, text=True, timeout=300, env=env)
        except subprocess.TimeoutExpired:
            return {"error": "shim driver timed out (300 s)"}
    if r.returncode != 0:
        return {"error": f"shim driver rc {r.returncode}: {r.stderr.strip()[-300:]}"}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    base = out["orbx_extract_ms"]["median"]
    out["operator_over_orbx_extract"] = round(out["operator_ms"]["median"] / base, 3)
    out["stereo_frame_over_operator"] = round(out["stereo_frame_ms"]["median"] / out["operator_ms"]["median"], 3)
    out["what"] = ("child process, host clock per call: orbx_extract (C-ABI, host buffers); "
                   "ORBextractor::operator() as shipped (operator_ms: no host mvImagePyramid, the default) and "
                   "with the opt-in pinned host copy (operator_ms_host_pyramid, ORBX_HOST_PYRAMID=1); "
                   "stereo Frame = two operator() threads + ComputeStereoMatches on the device outputs")
    return out


def shim_matcher_latency_leg(local, n=100, warm=10, cpu_reps=20):
    """The drop-in ORBmatcher methods per host call as Tracking and LocalMapping
    make them: SearchByProjection(F, local map points)
    (src/Tracking.cc:1277), SearchByProjection(CurrentFrame, LastFrame)
    (:962), SearchByBoW(KF, F) (:842, 1465), SearchForTriangulation
    (src/LocalMapping.cc:301) and Fuse (:525, 550), each through the compiled
    shim on reference-typed Frames / KeyFrames / MapPoints at KITTI sizes
    (2000 keypoints, 2000-3000 map points; tests/shimscene.py builds the
    scenes, shim/host/scene.cc --scene-latency times the call alone with the
    state rebuilt outside the clock), and beside each the single-thread CPU
    restatement (oracle/) on the same inputs, timed in this process after the
    timed region (the oracle is the CPU baseline here, never the product)."""
    import subprocess
    import tempfile
    import time
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import shimscene
    from oracle import oracle as O
    if not os.path.exists(SHIM_DRIVER):
        return {"error": f"{SHIM_DRIVER} not built (python __graft_entry__.py builds it)"}
    calls = [("search_by_projection_local_map", "local_map", "src/Tracking.cc:1277"),
             ("search_by_projection_last_frame", "last_frame", "src/Tracking.cc:962"),
             ("search_by_bow_kf_f", "bow", "src/Tracking.cc:842"),
             ("search_for_triangulation", "triangulation", "src/LocalMapping.cc:301"),
             ("fuse", "fuse", "src/LocalMapping.cc:525")]
    out = {}
    env = dict(os.environ, ORBX_DEVICE=str(local))
    with tempfile.TemporaryDirectory() as d:
        for key, builder, site in calls:
            recs, want = getattr(shimscene, builder)(O, 1)
            cpu_fn = shimscene.LAST_CPU[0]
            path = os.path.join(d, key + ".bin")
            shimscene.write_scene(path, recs)
            try:
                r = subprocess.run([SHIM_DRIVER, "--scene-latency", path, str(n), str(warm)], capture_output=True,
                                   text=True, timeout=300, env=env)
            except subprocess.TimeoutExpired:
                out[key] = {"error": "shim driver timed out"}
                continue
            if r.returncode != 0:
                out[key] = {"error": f"rc {r.returncode}: {r.stderr.strip()[-200:]}"}
                continue
            g = json.loads(r.stdout.strip().splitlines()[-1])
            cpu_fn()
            ts = []
            for _ in range(cpu_reps):
                t0 = time.perf_counter()
                cpu_fn()
                ts.append((time.perf_counter() - t0) * 1e3)
            cpu_ms = float(np.median(ts))
            out[key] = {"site": site, "shim_ms": {"median": round(g["median_ms"], 4), "p99": round(g["p99_ms"], 4)},
                        "cpu_oracle_1thread_ms": round(cpu_ms, 4),
                        "cpu_over_shim": round(cpu_ms / g["median_ms"], 2) if g["median_ms"] > 0 else None,
                        "matches": int(g["matches"]), "matches_expected": int(want[0])}
    out["what"] = ("host clock per call through the drop-in shim (upload, launch, one stream wait, download; the "
                   "Frame/KeyFrame state rebuilt outside the clock) vs the single-thread oracle on the same scene "
                   f"(median of {cpu_reps}; ctypes call overhead included); KITTI-sized synthetic scenes")
    return out


def cpu_tie_rule_study(frames, cfg):
    """How far the product's quadtree tie rule (node creation order) is from
    the reference's (heap address, src/ORBextractor.cc:1041), measured on the
    CPU with the oracle's layout-identical pointer-order quadtree
    (orc_tie_sequence), and how far the pointer order is
    from itself under another heap history. Runs with the CPU baseline, after
    the timed region; the oracle is the checker here, not the product."""
    from oracle import oracle as O
    oc = oracle_config(O, cfg)
    d01, k01 = O.tie_sequence(oc, frames, O.TIE_LATER_FIRST, O.TIE_POINTER)
    d11, k11 = O.tie_sequence(oc, frames, O.TIE_POINTER, O.TIE_POINTER)
    return {"frames": int(len(frames)),
            "creation_vs_pointer": {"levels_list_differs_frac": round(float(d01.mean()), 3),
                                    "levels_kept_set_differs_frac": round(float((k01 > 0).mean()), 3),
                                    "keypoints_kept_by_one_rule_per_frame": round(float(k01.sum(1).mean()), 2)},
            "pointer_vs_pointer_other_heap_history": {"levels_list_differs_frac": round(float(d11.mean()), 3),
                                                      "levels_kept_set_differs_frac": round(float((k11 > 0).mean()), 3),
                                                      "keypoints_kept_by_one_run_per_frame": round(float(k11.sum(1).mean()), 2)},
            "source": "oracle tie-rule study on the host CPU (checker), consecutive frames of the timed sequence"}


def cpu_model():
    """The host CPU's model name (report it beside the CPU baseline)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_latency(frames, cfg, no_match, warm=20):
    """The oracle's single-thread latency of the same calls: median over the
    frames after `warm` warm-up frames (>= 200 frames)."""
    from oracle import oracle as O
    W, H, NF = cfg["W"], cfg["H"], cfg["nfeatures"]
    oc = oracle_config(O, cfg)
    te, ts, prev = [], [], None
    for fr in frames:
        t0 = time.perf_counter()
        kp, desc = O.extract(oc, fr)
        te.append(time.perf_counter() - t0)
        if prev is not None and not no_match:
            pk, pd = prev
            t0 = time.perf_counter()
            O.search_for_initialization(pk, pd, kp, desc, (0, W, 0, H), np.stack([pk["x"], pk["y"]], 1), 100, 0.9, True)
            ts.append(time.perf_counter() - t0)
        prev = (kp, desc)
    w = min(warm, max(0, len(te) - 1))
    te, ts = te[w:], ts[w:]
    out = {"extract_ms_median": round(float(np.median(te)) * 1e3, 3), "frames": len(te), "warmup": w, "cores": 1,
           "kind": "port"}
    if ts:
        out["search_init_ms_median"] = round(float(np.median(ts)) * 1e3, 3)
    return out


STEREO_METRIC = "stereo pairs/s ORB extract (left+right) + ComputeStereoMatches, 2x1241x376 nFeatures=2000"
MB, MBF = 0.54, 0.54 * 718.856  # KITTI stereo baseline (m) and baseline x fx


def run_stereo(args, cfg, rank, world, local, dist):
    """C4: per step B rectified pairs resident in HBM; left frames extracted on
    one stream and right frames on another (two ORBextractor handles, as
    Frame's mpORBextractorLeft / mpORBextractorRight), then ComputeStereoMatches
    of the B pairs on the left stream once both are done. Two handle sets
    (each with its own matcher) alternate between steps so that the stereo
    matching of step k (which reads step k's pyramids) overlaps the
    extraction of step k+1."""
    import orb_slam_cuda_amd as pkg
    from orb_slam_cuda_amd import _lib, sharding
    from orb_slam_cuda_amd.synth import stereo_pair

    L = _lib.lib()
    check = _lib.check
    W, H, NF, B = cfg["W"], cfg["H"], cfg["nfeatures"], args.batch
    pitch = (W + 63) & ~63
    base = sharding.sequence_seed(rank)
    pairs = [stereo_pair(base + i, W, H) for i in range(B)]
    host = np.zeros((2, B, H, pitch), np.uint8)
    for i, (a, b) in enumerate(pairs):
        host[0, i, :, :W] = a
        host[1, i, :, :W] = b
    d_frames = _lib.DeviceArray(host.nbytes)
    d_frames.upload(host)
    fb = B * H * pitch  # bytes of one side's frames
    NSET = 2
    sets = []
    s_one = _lib.Stream() if args.serial else None  # --serial: every launch on one stream
    for _ in range(NSET):
        eL = pkg.ORBextractor(*ext_params(cfg), W, H, device=local, max_batch=B)
        eR = pkg.ORBextractor(*ext_params(cfg), W, H, device=local, max_batch=B)
        if args.stage_order:
            eL.set_stage_order(args.stage_order)
            eR.set_stage_order(args.stage_order)
        cap = eL.frame_capacity
        sL = s_one or _lib.Stream()
        sets.append(dict(eL=eL, eR=eR, sL=sL, sR=s_one or _lib.Stream(),
                         m=pkg.ORBmatcher(device=local, max_pairs=B, max_kps=cap),
                         kps=_lib.DeviceArray(2 * B * cap * KP), desc=_lib.DeviceArray(2 * B * cap * DS),
                         n=_lib.DeviceArray(2 * B * 4), u=_lib.DeviceArray(B * cap * 4),
                         d=_lib.DeviceArray(B * cap * 4), kept=_lib.DeviceArray(B * 4)))
    cap = sets[0]["eL"].frame_capacity
    vp = lambda a: C.c_void_p(a)
    total = args.warmup + args.steps
    # per step: 6 extraction stage marks (left stream) + stereo start/end + right-done + done
    evs = [[_lib.Event() for _ in range(10)] for _ in range(total)]

    def step(k):
        st = sets[k % NSET]
        ev = evs[k]
        if k >= NSET:
            st["sR"].wait(evs[k - NSET][9])  # stereo k-2 (left stream) read this set's right pyramid
        arr = (C.c_void_p * 6)(*[e.e.value for e in ev[:6]])
        check(L.orbx_set_stage_events(st["eL"].handle, arr))
        for side, (ex, s) in enumerate(((st["eL"], st["sL"]), (st["eR"], st["sR"]))):
            check(L.orbx_extract_batch(ex.handle, vp(d_frames.ptr + side * fb), B, H * pitch, pitch,
                                       vp(st["kps"].ptr + side * B * cap * KP),
                                       vp(st["desc"].ptr + side * B * cap * DS), vp(st["n"].ptr + side * B * 4), s.s))
        ev[8].record(st["sR"])
        st["sL"].wait(ev[8])
        ev[6].record(st["sL"])
        check(L.orbm_compute_stereo_matches_batch(
            st["m"].handle, st["eL"].handle, 0, st["eR"].handle, 0, vp(st["kps"].ptr), vp(st["desc"].ptr),
            vp(st["n"].ptr), vp(st["kps"].ptr + B * cap * KP), vp(st["desc"].ptr + B * cap * DS),
            vp(st["n"].ptr + B * 4), cap, B, C.c_float(MB), C.c_float(MBF), vp(st["u"].ptr), vp(st["d"].ptr),
            vp(st["kept"].ptr), st["sL"].s), matcher=True)
        ev[7].record(st["sL"])
        ev[9].record(st["sL"])

    def sync_all():
        for st in sets:
            st["sL"].synchronize()
            st["sR"].synchronize()

    for k in range(args.warmup):
        step(k)
    sync_all()
    if dist is not None:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    for k in range(args.warmup, total):
        step(k)
    sync_all()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    agg = aggregate(B * args.steps, t1 - t0, dist, world)
    for st in sets:
        for h in (st["eL"], st["eR"]):
            if h.status():
                raise RuntimeError("extractor device status word set")
        if st["m"].status():
            raise RuntimeError("matcher device status word set")
    timed = evs[args.warmup:]
    from orb_slam_cuda_amd import _lib as _stage_lib
    launch_order = _stage_lib.stage_order(sets[0]["eL"].handle)  # stage event i + 1 closes launch_order[i]
    stages = STAGES[:5] + ["stereo"]
    sm = {s: 0.0 for s in stages}
    for ev in timed:
        for i, s in enumerate(launch_order):
            sm[s] += ev[i].elapsed_ms(ev[i + 1])
        sm["stereo"] += ev[6].elapsed_ms(ev[7])
    sm = {s: v / args.steps for s, v in sm.items()}
    last = sets[(total - 1) % NSET]
    kept = last["kept"].download(B, np.int32)
    nkp = last["n"].download(2 * B, np.int32)
    ab = algorithmic_bytes(W, H, float(nkp.mean()))
    hbm_stages = {"pyramid": ab["pyramid"], "blur": ab["blur"], "fast_grid": ab["fast_grid"],
                  "orient_brief": ab["orient_brief"]}
    rk = "fast_grid"
    ach = hbm_stages[rk] * B / (sm[rk] * 1e-3) / 1e9
    roof = {"kernel": KERNELS[rk], "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_bytes(KERNELS[rk]),
            "algorithmic_bytes_per_launch": int(hbm_stages[rk] * B), "avg_launch_ms": round(sm[rk], 4)}
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline_stereo(pairs, cfg, max(1, args.cpu_sample // 2))
    if rank == 0:
        out = {
            "metric": STEREO_METRIC, "value": round(agg["value"], 2), "unit": "stereo pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(agg["wall"] / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic rectified pairs (orb_slam_cuda_amd/synth.py stereo_pair)",
            "config": {"workload": cfg["workload"], "frame": f"2x{W}x{H}", "nfeatures": NF, "nlevels": ext_params(cfg)[2],
                       "scale_factor": 1.2, "pairs_per_step_per_gpu": B,
                       "parallelism": f"pair-sharded x{world}, one process per GPU, no collectives",
                       "streams": 1 if args.serial else 2 * NSET,
                       "mb": MB, "mbf": MBF},
            "per_rank_pairs_per_s": agg["per_rank"],
            "roofline": roof,
            "cpu_baseline": cpu,
            "stage_ms_per_step": {s: round(v, 4) for s, v in sm.items()},
            "keypoints_per_image": round(float(nkp.mean()), 1),
            "stereo_matches_per_pair": round(float(kept.mean()), 1),
            **args.audit,
        }
        print(json.dumps(out), flush=True)


def cpu_baseline_stereo(pairs, cfg, n):
    """The CPU oracle on a bounded sample of pairs: extract left + right, pyramids, ComputeStereoMatches."""
    from oracle import oracle as O
    W, H, NF = cfg["W"], cfg["H"], cfg["nfeatures"]
    oc = oracle_config(O, cfg)
    li = O.level_info(oc)
    t0 = time.perf_counter()
    for i in range(n):
        a, b = pairs[i % len(pairs)]
        kl, dl = O.extract(oc, a)
        kr, dr = O.extract(oc, b)
        O.compute_stereo_matches(kl, dl, kr, dr, O.pyramid(oc, a), O.pyramid(oc, b), li["scale"], li["inv_scale"],
                                 MB, np.float32(MBF))
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "stereo pairs/s", "cores": 1, "kind": "port",
            "sample": f"{n} synthetic pairs (cycling the step's {len(pairs)}), oracle extract left + right + ComputeStereoMatches "
                      f"(pyramids rebuilt for the SAD), single thread, {dt:.1f} s"}


def seq_cpu(rank, W, H, n):
    """The first n frames of the rank's synthetic sequence (the timed batch is its first B)."""
    from orb_slam_cuda_amd import sharding
    from orb_slam_cuda_amd.synth import SynthSequence
    return SynthSequence(sharding.sequence_seed(rank), W, H).frames(n)


def _cpu_run(O, oc, frames, W, no_match):
    """Oracle extract (+ dense top-2 + SearchForInitialization vs the previous frame) over consecutive frames."""
    prev = None
    for fr in frames:
        kp, desc = O.extract(oc, fr)
        if prev is not None and not no_match:
            pk, pd = prev
            O.hamming_top2(desc, pd)
            O.search_for_initialization(pk, pd, kp, desc, (0, W, 0, fr.shape[0]), np.stack([pk["x"], pk["y"]], 1),
                                        100, 0.9, True)
        prev = (kp, desc)


def cpu_threads_default():
    """The host cores this job may use (the GPU box exports OMP_NUM_THREADS = its CPU share)."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, int(env)) if env.isdigit() else min(8, os.cpu_count() or 1)


def cpu_baseline(frames, cfg, n, no_match, threads=1):
    """The CPU oracle (restatement of the reference CPU path) on a bounded sample.

    threads == 1: one thread over n consecutive frames.
    threads > 1: independent frame-parallel workers, one per core, each over its
    own run of n consecutive frames, aggregate frames/s over the wall clock
    (SURVEY 8(d) (ii)); the oracle's C calls release the GIL.
    """
    from oracle import oracle as O
    W, H, NF = cfg["W"], cfg["H"], cfg["nfeatures"]
    oc = oracle_config(O, cfg)
    n = min(n, len(frames))
    what = " + dense top-2 + SearchForInitialization vs t-1"
    if threads <= 1:
        t0 = time.perf_counter()
        _cpu_run(O, oc, frames[:n], W, no_match)
        dt = time.perf_counter() - t0
        return {"value": round(n / dt, 3), "unit": "frames/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
                "sample": f"{n} consecutive frames of the same synthetic sequence, oracle extract"
                          + ("" if no_match else what) + f", single thread, {dt:.1f} s"}
    from concurrent.futures import ThreadPoolExecutor
    # every worker runs as many frames as the single-thread sample (about
    # 10 s of CPU work each, so the aggregate is not a sub-second blip)
    per = max(2, n)
    chunks = [frames[(k * 37) % max(1, len(frames) - per):][:per] for k in range(threads)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda c: _cpu_run(O, oc, c, W, no_match), chunks))
    dt = time.perf_counter() - t0
    tot = sum(len(c) for c in chunks)
    return {"value": round(tot / dt, 3), "unit": "frames/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{threads} frame-parallel oracle workers x {per} consecutive frames of the synthetic sequence, "
                      "oracle extract" + ("" if no_match else what) + f", {dt:.1f} s wall"}


if __name__ == "__main__":
    main()
