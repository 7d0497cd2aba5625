#!/usr/bin/env python3
"""bench.py — ORB extract + match throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): KITTI-shaped 1241x376 mono u8
frames, nFeatures=2000, 8 levels, scale 1.2, iniThFAST 20 / minThFAST 7.
One step = one batch of B frames resident in HBM:
  * ORBextractor::operator() on all B frames (orbx_extract_batch), and
  * for every frame t, matching against frame t-1: the dense brute-force
    2000 x 2000 Hamming best/second search (orbm_hamming_top2) and the exact
    ORBmatcher::SearchForInitialization (window 100, ratio 0.9, rotation
    check) used by monocular initialisation.
Frame t-1 of the first frame of a batch is the last frame of the previous
batch (carried on device), so every step does B extractions + B matches.

Two streams: the matching of batch k (a few wide workgroups per frame pair)
runs on its own stream, overlapping the extraction of batch k+1; outputs are
triple-buffered and ordered by events (see step()). --serial runs everything
on one stream.

Multi-GPU: one process per GPU, frames sharded by rank (each rank streams its
own synthetic sequence), no data-path collective ("weak" scaling). The
barrier and the max-over-ranks of the timed region go through
torch.distributed with the gloo backend (control plane only).

Prints ONE JSON line (rank 0). Per-kernel durations are measured live with
HIP events recorded on the launch stream around every stage of every step.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
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
           "quadtree": "quadtree_kernel", "orient_brief": "orient_brief_kernel",
           "hamming_top2": "hamming_top2_mfma_kernel", "search_init": "search_init_kernel"}

CONFIGS = {
    "kitti": dict(W=1241, H=376, nfeatures=2000,
                  workload="C3: KITTI-shaped 1241x376 mono u8, nFeatures=2000, 8 levels x1.2, "
                           "extract + match vs t-1 (dense 2000x2000 Hamming top-2 + SearchForInitialization)"),
    "stereo": dict(W=1241, H=376, nfeatures=2000, stereo=True,
                   workload="C4: stereo_kitti, 2 x 1241x376 u8 per pair, nFeatures=2000 per image, 8 levels x1.2, "
                            "left/right extraction on separate HIP streams + Frame::ComputeStereoMatches"),
    "euroc": dict(W=752, H=480, nfeatures=1000,
                  workload="C5: EuRoC-shaped 752x480 mono u8, nFeatures=1000, 8 levels x1.2, "
                           "extract + match vs t-1 (dense Hamming top-2 + SearchForInitialization)"),
}


def level_sizes(W, H, L=8, s=1.2):
    sc = [1.0]
    for _ in range(1, L):
        sc.append(np.float32(sc[-1]) * np.float32(s))
    out = []
    for f in sc:
        inv = np.float32(1.0) / np.float32(f)
        out.append((int(np.rint(np.float32(W) * inv)), int(np.rint(np.float32(H) * inv))))
    return out


def algorithmic_bytes(W, H, nkp):
    """Per-frame algorithmic HBM bytes of each stage (DESIGN.md "Roofline")."""
    P = [w * h for w, h in level_sizes(W, H)]
    return {
        "pyramid": sum(P[l - 1] + P[l] for l in range(1, 8)),         # read l-1, write l
        "blur": 2 * sum(P),                                            # read + write every level
        "fast_grid": sum(P),                                           # read every level once
        "pyr_fast_pass": P[0] + sum(P[:7]) + sum(P[1:]) + sum(P),      # BASELINE.md B_pf
        "orient_brief": nkp * (2 * 31 * 31 + 60),                      # patch gathers + outputs
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64, help="frames per step per GPU")
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
    ap.add_argument("--bow", action="store_true",
                    help="also Frame::ComputeBoW every frame (synthetic ORBvoc-shaped vocabulary, k 10 L 6)")
    ap.add_argument("--match-streams", type=int, choices=[1, 2], default=1,
                    help="2: SearchForInitialization on its own stream, beside the dense top-2")
    ap.add_argument("--carry", choices=["match", "ext"], default="match",
                    help="stream that copies a batch's last frame for the next batch's first pair")
    args = ap.parse_args()

    from orb_slam_cuda_amd import sharding
    rank, world, local = sharding.rank_info()
    # control plane only (gloo); initialised before liborbx loads so one HIP runtime is in the process
    dist = sharding.init_control_plane()

    import orb_slam_cuda_amd as pkg
    from orb_slam_cuda_amd import _lib
    from orb_slam_cuda_amd.synth import SynthSequence

    L = _lib.lib()
    cfg = CONFIGS[args.config]
    if cfg.get("stereo"):
        return run_stereo(args, cfg, rank, world, local, dist)
    W, H, NF, B = cfg["W"], cfg["H"], cfg["nfeatures"], args.batch
    pitch = (W + 63) & ~63

    seq = SynthSequence(sharding.sequence_seed(rank), W, H)
    frames = seq.frames(B)
    host = np.zeros((B, H, pitch), np.uint8)
    host[:, :, :W] = frames
    d_frames = _lib.DeviceArray(host.nbytes)
    check = _lib.check
    check(L.orbx_set_device(local))
    d_frames.upload(host)

    S = args.split
    if S < 1 or B % S:
        raise SystemExit("--split must divide --batch")
    BS = B // S  # frames per extraction launch
    exts = [pkg.ORBextractor(NF, 1.2, 8, 20, 7, W, H, device=local, max_batch=BS) for _ in range(S)]
    ext = exts[0]
    cap = ext.frame_capacity
    KP, DS = 28, 32
    # three output sets: batch k writes set k % 3, slots 1..B, and its last
    # frame is copied into slot 0 of set (k+1) % 3 (frame t-1 of the next
    # batch's first frame).
    NS = 3
    d_kps = [_lib.DeviceArray((B + 1) * cap * KP) for _ in range(NS)]
    d_desc = [_lib.DeviceArray((B + 1) * cap * DS) for _ in range(NS)]
    d_counts = [_lib.DeviceArray((B + 1) * 4) for _ in range(NS)]
    for d in d_counts:
        d.zero()
    matcher = pkg.ORBmatcher(0.9, True, device=local, max_pairs=B, max_kps=cap)
    d_bi, d_bd, d_sd = (_lib.DeviceArray(B * cap * 4) for _ in range(3))
    d_m12 = _lib.DeviceArray(B * cap * 4)
    d_nm = _lib.DeviceArray(B * 4)
    # the extraction stream may ask the dispatcher for priority (--priority):
    # it is the critical path, matching fills the compute units it leaves idle
    prio = 1 if args.priority else None
    s_exts = [_lib.Stream(prio) for _ in range(S)]
    s_ext = s_exts[0]
    s_match = _lib.Stream(0 if args.priority else None) if not args.serial else s_ext
    two_match = args.match_streams == 2 and not args.serial and not args.no_match and args.carry == "match"
    s_init = _lib.Stream(0 if args.priority else None) if two_match else s_match
    bounds = _lib.GridBounds(0.0, float(W), 0.0, float(H))
    vp = lambda a: C.c_void_p(a)
    n_ev = 12  # 6 extraction stage marks (extract stream) + 3 matching marks + 2 BoW marks (match stream) + init start
    voc = None
    if args.bow:
        from orb_slam_cuda_amd.synth import synthetic_vocabulary
        voc = pkg.ORBVocabulary.from_arrays(synthetic_vocabulary(10, 6, seed=1), device=local)
        d_bw, d_bn, d_fn, d_fi, d_fnn = (_lib.DeviceArray(B * cap * 4), _lib.DeviceArray(B * 4),
                                         _lib.DeviceArray(B * cap * 4), _lib.DeviceArray(B * cap * 4),
                                         _lib.DeviceArray(B * 4))
        d_bv = _lib.DeviceArray(B * cap * 8)
        d_fo = _lib.DeviceArray(B * (cap + 1) * 4)
        d_vw = (_lib.DeviceArray(B * cap * 4), _lib.DeviceArray(B * cap * 4), _lib.DeviceArray(B * cap * 8))

    def step(k, evs, ev_ext, ev_done):
        """Batch k: extraction on s_ext; carry copy and matching of the same
        batch on s_match, overlapping the extraction of batch k+1 (--serial:
        one stream, no overlap). Extraction k waits for matching k-3 (the
        last reader of set k % 3); matching k waits for extraction k."""
        b, nb = k % NS, (k + 1) % NS
        # the batch is cut into S contiguous parts, one extractor and stream each
        for h, (ex, se) in enumerate(zip(exts, s_exts)):
            if h == 0:
                arr = (C.c_void_p * 6)(*[e.e.value for e in evs[:6]])
                check(L.orbx_set_stage_events(ex.handle, arr))
            if not args.serial and k >= 3:
                se.wait(ev_done[k - 3])  # matching k-3 was the last reader of set k % 3
                if two_match:
                    se.wait(ev_done2[k - 3])
            sv = se if not args.serial else s_ext
            check(L.orbx_extract_batch(ex.handle, vp(d_frames.ptr + h * BS * H * pitch), BS, H * pitch, pitch,
                                       vp(d_kps[b].ptr + (1 + h * BS) * cap * KP),
                                       vp(d_desc[b].ptr + (1 + h * BS) * cap * DS),
                                       vp(d_counts[b].ptr + 4 * (1 + h * BS)), sv.s))
            if h > 0 and not args.serial:
                ev_part[k][h].record(se)
                s_ext.wait(ev_part[k][h])
        def carry(st):
            check(L.orbx_memcpy_dtod_async(vp(d_kps[nb].ptr), vp(d_kps[b].ptr + B * cap * KP), cap * KP, st.s))
            check(L.orbx_memcpy_dtod_async(vp(d_desc[nb].ptr), vp(d_desc[b].ptr + B * cap * DS), cap * DS, st.s))
            check(L.orbx_memcpy_dtod_async(vp(d_counts[nb].ptr), vp(d_counts[b].ptr + B * 4), 4, st.s))

        if args.carry == "ext" or args.serial:
            # slot 0 of set (k+1) % 3 was last read by matching k-2
            if k >= 2 and not args.serial:
                s_ext.wait(ev_done[k - 2])
            carry(s_ext)
        ev_ext[k].record(s_ext)
        if not args.serial:
            s_match.wait(ev_ext[k])
        if args.carry == "match" and not args.serial:
            if two_match and k >= 2:
                s_match.wait(ev_done2[k - 2])  # SearchForInitialization k-2 also read set (k+1) % 3
            carry(s_match)  # in order after matching k-2, the last reader of set (k+1) % 3
            ev_carry[k].record(s_match)
        if voc is not None:
            evs[9].record(s_match)
            # Frame::ComputeBoW of the batch's frames (slots 1..B), levelsup 4 (src/Frame.cc:398)
            check(L.orbv_transform_batch(voc.handle, vp(d_desc[b].ptr + cap * DS), cap * DS, vp(d_counts[b].ptr + 4),
                                         B, cap, 4, vp(d_bw.ptr), vp(d_bv.ptr), vp(d_bn.ptr), vp(d_fn.ptr),
                                         vp(d_fo.ptr), vp(d_fi.ptr), vp(d_fnn.ptr), vp(d_vw[0].ptr), vp(d_vw[1].ptr),
                                         vp(d_vw[2].ptr), s_match.s), vocabulary=True)
            evs[10].record(s_match)
        evs[6].record(s_match)
        if not args.no_match:
            # query = frame t (slots 1..B), candidates = frame t-1 (slots 0..B-1)
            check(L.orbm_hamming_top2(matcher.handle, vp(d_desc[b].ptr + cap * DS), cap * DS,
                                      vp(d_counts[b].ptr + 4), cap, vp(d_desc[b].ptr), cap * DS,
                                      vp(d_counts[b].ptr), B, vp(d_bi.ptr), vp(d_bd.ptr), vp(d_sd.ptr),
                                      s_match.s), matcher=True)
            evs[7].record(s_match)
            if two_match:  # after batch k's extraction and the carry into its slot 0 (step k-1)
                s_init.wait(ev_ext[k])
                if k >= 1:
                    s_init.wait(ev_carry[k - 1])
            evs[11].record(s_init)
            check(L.orbm_search_for_initialization_batch(
                matcher.handle, vp(d_kps[b].ptr), vp(d_desc[b].ptr), vp(d_counts[b].ptr),
                vp(d_kps[b].ptr + cap * KP), vp(d_desc[b].ptr + cap * DS), vp(d_counts[b].ptr + 4), cap, B,
                bounds, None, 100, C.c_float(0.9), 1, vp(d_m12.ptr), vp(d_nm.ptr), s_init.s), matcher=True)
        evs[8].record(s_init)
        ev_done[k].record(s_match)
        if two_match:
            ev_done2[k].record(s_init)

    total_steps = args.warmup + args.steps
    evsets = [[_lib.Event() for _ in range(n_ev)] for _ in range(total_steps)]
    ev_ext = [_lib.Event() for _ in range(total_steps)]
    ev_done = [_lib.Event() for _ in range(total_steps)]
    ev_done2 = [_lib.Event() for _ in range(total_steps)]
    ev_carry = [_lib.Event() for _ in range(total_steps)]
    ev_part = [[_lib.Event() for _ in range(S)] for _ in range(total_steps)]
    def sync_all():
        for se in s_exts:
            se.synchronize()
        s_match.synchronize()
        s_init.synchronize()

    for k in range(args.warmup):
        step(k, evsets[k], ev_ext, ev_done)
    sync_all()
    if dist is not None:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    for k in range(args.warmup, total_steps):
        step(k, evsets[k], ev_ext, ev_done)
    t_issue = time.perf_counter()  # host time to enqueue the timed steps (launch-bound if close to wall)
    sync_all()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    wall = sharding.max_over_ranks(t1 - t0, dist)
    timed = evsets[args.warmup:]
    ev_ms = timed[0][0].elapsed_ms(timed[-1][8])
    STAGES_RUN = STAGES + (["bow_transform"] if args.bow else [])

    # per-stage average durations over the timed steps (ms per launch-group, B frames),
    # each bracketed by events on the stream its kernels run on
    st = {s: 0.0 for s in STAGES_RUN}
    for evs in timed:
        for i, s in enumerate(STAGES[:5]):
            st[s] += evs[i].elapsed_ms(evs[i + 1])
        if args.bow:
            st["bow_transform"] += evs[9].elapsed_ms(evs[10])
        if not args.no_match:
            st["hamming_top2"] += evs[6].elapsed_ms(evs[7])
            st["search_init"] += evs[11].elapsed_ms(evs[8])
    st = {s: v / args.steps for s, v in st.items()}

    nm = d_nm.download(B, np.int32)
    nkp_mean = float(d_counts[(total_steps - 1) % NS].download(B + 1, np.int32)[1:].mean())
    frames_total = B * args.steps * world
    value = frames_total / wall
    ab = algorithmic_bytes(W, H, nkp_mean)
    extract_ms = sum(st[s] for s in STAGES[:5])
    dominant = max(STAGES_RUN, key=lambda s: st[s])
    # roofline of the pyramid+FAST pass and of the dominant kernel
    pf_ms = st["pyramid"] + st["fast_grid"]
    pf_gbs = ab["pyr_fast_pass"] * BS / (pf_ms * 1e-3) / 1e9
    roof = None
    hbm_stages = {"pyramid": ab["pyramid"], "blur": ab["blur"], "fast_grid": ab["fast_grid"],
                  "orient_brief": ab["orient_brief"]}
    # the roofline kernel is FAST: the longest extraction kernel when each runs
    # alone (profiles/r01_serial_kernel_stats.csv) and the one whose event time
    # in this pipelined run matches its rocprofv3 average; the event pairs of
    # the pyramid and the blur also hold their wait for compute units that the
    # other streams occupy, which a by-time pick would report as their duration
    rk = "fast_grid"
    def pmc_bytes(kernel):
        """HBM-side bytes per launch of `kernel` from the committed PMC passes (profiles/)."""
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        try:
            pmc = json.load(open(pmc_path))
        except Exception:
            return None
        want = kernel.split(" ")[0]  # profile keys carry template arguments ("fast_cells_kernel<44>")
        return next((v.get("bytes_per_launch") for k, v in pmc.items() if k.split("<")[0] == want), None)

    traffic = pmc_bytes(KERNELS[rk])
    ach = hbm_stages[rk] * BS / (st[rk] * 1e-3) / 1e9
    roof = {"kernel": KERNELS[rk], "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": int(hbm_stages[rk] * BS),
            "avg_launch_ms": round(st[rk], 4)}

    # the dense matcher runs on the matrix cores: algorithmic work = one 256-element +-1 dot
    # product per (query, candidate) pair = 512 FLOP, against the dense FP4 MFMA peak; the
    # per-pair top-2 update (v_min + v_med3) is reported against the VALU lane-op peak
    match_roof = None
    if not args.no_match and st["hamming_top2"] > 0:
        cnt = d_counts[(total_steps - 1) % NS].download(B + 1, np.int32).astype(np.int64)
        pairs = int((cnt[1:] * cnt[:-1]).sum())
        sec = st["hamming_top2"] * 1e-3
        tf = 512.0 * pairs / sec / 1e12
        match_roof = {"kernel": KERNELS["hamming_top2"], "bound": "mfma", "unit": "TFLOP/s",
                      "achieved": round(tf, 1), "peak": MFMA_FP4_PEAK_TFLOPS, "frac": round(tf / MFMA_FP4_PEAK_TFLOPS, 4),
                      "dtype": "fp4 e2m1 (+-1 bits, exact)", "top2_valu_frac": round(2.0 * pairs / sec / 1e12 / VALU_PEAK_TOPS, 4),
                      "traffic": pmc_bytes(KERNELS["hamming_top2"]),
                      "pairs_per_launch": pairs, "pairs_per_s": round(pairs / sec, 1),
                      "avg_launch_ms": round(st["hamming_top2"], 4)}

    cpu = cpu1 = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        sample = frames if args.cpu_sample <= len(frames) else seq_cpu(rank, W, H, args.cpu_sample)
        cpu1 = cpu_baseline(sample, cfg, args.cpu_sample, args.no_match)
        nt = args.cpu_threads if args.cpu_threads > 0 else cpu_threads_default()
        cpu = cpu_baseline(sample, cfg, args.cpu_sample, args.no_match, nt) if nt > 1 else cpu1

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded shapes + noise sequence, orb_slam_cuda_amd/synth.py)",
            "config": {"workload": (cfg["workload"] if not args.no_match else cfg["workload"].split(", extract")[0] + ", extract only")
                                   + (" + Frame::ComputeBoW (synthetic k10 L6 vocabulary)" if args.bow else ""),
                       "frame": f"{W}x{H}", "nfeatures": NF, "nlevels": 8, "scale_factor": 1.2,
                       "frames_per_step_per_gpu": B, "parallelism": f"frame-sharded x{world}, no collectives",
                       "streams": 1 if args.serial else S + 1, "frames_per_extract_launch": BS},
            "roofline": roof,
            "match_roofline": match_roof,
            "cpu_baseline": cpu,
            "cpu_baseline_1thread": cpu1,
            "pyr_fast_pass_hbm_gbs": round(pf_gbs, 1),
            "dominant_kernel": KERNELS[dominant],
            "stage_ms_per_step": {s: round(v, 4) for s, v in st.items()},
            "extract_only_frames_per_s": round(BS / (extract_ms * 1e-3), 1),
            "host_issue_ms_per_step": round((t_issue - t0) / args.steps * 1e3, 4), "event_ms_per_step": round(ev_ms / args.steps, 4),
            "keypoints_per_frame": round(nkp_mean, 1),
            "init_matches_per_pair": round(float(nm[1:].mean()), 1),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


STEREO_METRIC = "stereo pairs/s ORB extract (left+right) + ComputeStereoMatches, 2x1241x376 nFeatures=2000"
MB, MBF = 0.54, 0.54 * 718.856  # KITTI stereo baseline (m) and baseline x fx


def run_stereo(args, cfg, rank, world, local, dist):
    """C4: per step B rectified pairs resident in HBM; left frames extracted on
    one stream and right frames on another (two ORBextractor handles, as
    Frame's mpORBextractorLeft / mpORBextractorRight), then ComputeStereoMatches
    of the B pairs on the left stream once both are done. Two handle sets
    alternate between steps so that the stereo matching of step k (which reads
    step k's pyramids) overlaps the extraction of step k+1."""
    import orb_slam_cuda_amd as pkg
    from orb_slam_cuda_amd import _lib, sharding
    from orb_slam_cuda_amd.synth import stereo_pair

    L = _lib.lib()
    check = _lib.check
    W, H, NF, B = cfg["W"], cfg["H"], cfg["nfeatures"], args.batch
    pitch = (W + 63) & ~63
    check(L.orbx_set_device(local))
    base = sharding.sequence_seed(rank)
    pairs = [stereo_pair(base + i, W, H) for i in range(B)]
    host = np.zeros((2, B, H, pitch), np.uint8)
    for i, (a, b) in enumerate(pairs):
        host[0, i, :, :W] = a
        host[1, i, :, :W] = b
    d_frames = _lib.DeviceArray(host.nbytes)
    d_frames.upload(host)
    fb = B * H * pitch  # bytes of one side's frames
    KP, DS, NSET = 28, 32, 2
    sets = []
    s_one = _lib.Stream() if args.serial else None  # --serial: every launch on one stream
    for _ in range(NSET):
        eL = pkg.ORBextractor(NF, 1.2, 8, 20, 7, W, H, device=local, max_batch=B)
        eR = pkg.ORBextractor(NF, 1.2, 8, 20, 7, W, H, device=local, max_batch=B)
        cap = eL.frame_capacity
        sL = s_one or _lib.Stream()
        sets.append(dict(eL=eL, eR=eR, sL=sL, sR=s_one or _lib.Stream(),
                         kps=_lib.DeviceArray(2 * B * cap * KP), desc=_lib.DeviceArray(2 * B * cap * DS),
                         n=_lib.DeviceArray(2 * B * 4), u=_lib.DeviceArray(B * cap * 4),
                         d=_lib.DeviceArray(B * cap * 4), kept=_lib.DeviceArray(B * 4)))
    cap = sets[0]["eL"].frame_capacity
    matcher = pkg.ORBmatcher(device=local, max_pairs=B, max_kps=cap)
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
            matcher.handle, st["eL"].handle, 0, st["eR"].handle, 0, vp(st["kps"].ptr), vp(st["desc"].ptr),
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
    wall = sharding.max_over_ranks(t1 - t0, dist)
    timed = evs[args.warmup:]
    stages = STAGES[:5] + ["stereo"]
    sm = {s: 0.0 for s in stages}
    for ev in timed:
        for i, s in enumerate(STAGES[:5]):
            sm[s] += ev[i].elapsed_ms(ev[i + 1])
        sm["stereo"] += ev[6].elapsed_ms(ev[7])
    sm = {s: v / args.steps for s, v in sm.items()}
    last = sets[(total - 1) % NSET]
    kept = last["kept"].download(B, np.int32)
    nkp = last["n"].download(2 * B, np.int32)
    value = B * args.steps * world / wall
    ab = algorithmic_bytes(W, H, float(nkp.mean()))
    hbm_stages = {"pyramid": ab["pyramid"], "blur": ab["blur"], "fast_grid": ab["fast_grid"],
                  "orient_brief": ab["orient_brief"]}
    rk = max(hbm_stages, key=lambda s: sm[s])
    ach = hbm_stages[rk] * B / (sm[rk] * 1e-3) / 1e9
    roof = {"kernel": KERNELS[rk], "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "algorithmic_bytes_per_launch": int(hbm_stages[rk] * B), "avg_launch_ms": round(sm[rk], 4)}
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline_stereo(pairs, cfg, max(1, args.cpu_sample // 2))
    if rank == 0:
        out = {
            "metric": STEREO_METRIC, "value": round(value, 2), "unit": "stereo pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic rectified pairs (orb_slam_cuda_amd/synth.py stereo_pair)",
            "config": {"workload": cfg["workload"], "frame": f"2x{W}x{H}", "nfeatures": NF, "nlevels": 8,
                       "scale_factor": 1.2, "pairs_per_step_per_gpu": B,
                       "parallelism": f"pair-sharded x{world}, no collectives",
                       "streams": 1 if args.serial else 2 * NSET,
                       "mb": MB, "mbf": MBF},
            "roofline": roof,
            "cpu_baseline": cpu,
            "stage_ms_per_step": {s: round(v, 4) for s, v in sm.items()},
            "keypoints_per_image": round(float(nkp.mean()), 1),
            "stereo_matches_per_pair": round(float(kept.mean()), 1),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline_stereo(pairs, cfg, n):
    """The CPU oracle on a bounded sample of pairs: extract left + right, pyramids, ComputeStereoMatches."""
    from oracle import oracle as O
    W, H, NF = cfg["W"], cfg["H"], cfg["nfeatures"]
    oc = O.config(nfeatures=NF, width=W, height=H)
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
    own run of n // threads consecutive frames, aggregate frames/s over the wall
    clock; the oracle's C calls release the GIL.
    """
    from oracle import oracle as O
    W, H, NF = cfg["W"], cfg["H"], cfg["nfeatures"]
    oc = O.config(nfeatures=NF, width=W, height=H)
    n = min(n, len(frames))
    what = " + dense top-2 + SearchForInitialization vs t-1"
    if threads <= 1:
        t0 = time.perf_counter()
        _cpu_run(O, oc, frames[:n], W, no_match)
        dt = time.perf_counter() - t0
        return {"value": round(n / dt, 3), "unit": "frames/s", "cores": 1, "kind": "port",
                "sample": f"{n} consecutive frames of the same synthetic sequence, oracle extract"
                          + ("" if no_match else what) + f", single thread, {dt:.1f} s"}
    from concurrent.futures import ThreadPoolExecutor
    per = max(2, n // threads)
    chunks = [frames[(k * per) % max(1, len(frames) - per):][:per] for k in range(threads)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda c: _cpu_run(O, oc, c, W, no_match), chunks))
    dt = time.perf_counter() - t0
    tot = sum(len(c) for c in chunks)
    return {"value": round(tot / dt, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{threads} frame-parallel oracle workers x {per} consecutive frames of the synthetic sequence, "
                      "oracle extract" + ("" if no_match else what) + f", {dt:.1f} s wall"}


if __name__ == "__main__":
    main()
