"""Overlap accounting of a pipelined rocprofv3 kernel trace.

    python tools/trace_overlap.py gpurun_out/x/trace/run_kernel_trace.csv [--skip 0.3]

Takes the kernels of the bench's pipeline (extraction chain: pyramid, blur,
FAST, quadtree, orient+BRIEF; matching chain: Hamming top-2,
SearchForInitialization prep/query/resolve), drops the first `skip` fraction
of the trace (warm-up), and sweeps the start/end timestamps: the time with no
pipeline kernel running (idle), with only extraction kernels, only matching
kernels, both, and the time-weighted number of concurrent kernels. Per
kernel: launches, mean duration in the pipeline, and the share of its
duration during which another pipeline kernel was running.
"""
import argparse
import csv
from collections import defaultdict

EXTRACT = ("pyr_band_kernel", "blur_kernel", "fast_cells_kernel", "quadtree_kernel", "orient_brief_kernel")
MATCH = ("hamming_top2_mfma_kernel", "search_init_prep_kernel", "search_init_query_kernel",
         "search_init_resolve_kernel")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("orbx::", "")
    return n.split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=float, default=0.3)
    a = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(a.trace)):
        n = short(r["Kernel_Name"])
        if n in EXTRACT or n in MATCH:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r.get("Stream_Id", "")))
    ks.sort()
    ks = ks[int(len(ks) * a.skip):]
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    ev = []
    for i, (s, e, n, _) in enumerate(ks):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    last = t0
    acc = defaultdict(float)
    conc = defaultdict(float)
    overl = defaultdict(float)
    for t, d, i in ev:
        dt = t - last
        if dt > 0:
            ex = any(ks[j][2] in EXTRACT for j in active)
            ma = any(ks[j][2] in MATCH for j in active)
            acc["both" if ex and ma else "extract only" if ex else "match only" if ma else "idle"] += dt
            conc[len(active)] += dt
            if len(active) > 1:
                for j in active:
                    overl[j] += dt
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    span = t1 - t0
    print(f"window {span / 1e3:.1f} us, {len(ks)} kernels")
    for k in ("idle", "extract only", "match only", "both"):
        print(f"  {k:13s} {acc[k] / 1e3:10.1f} us  {acc[k] / span:6.1%}")
    print("  concurrency (time-weighted):", ", ".join(f"{c}: {v / span:.1%}" for c, v in sorted(conc.items())))
    per = defaultdict(list)
    ov = defaultdict(float)
    for i, (s, e, n, _) in enumerate(ks):
        per[n].append(e - s)
        ov[n] += overl[i]
    print(f"  {'kernel':28s} {'launches':>8s} {'mean us':>9s} {'sum us':>10s} {'overlapped':>10s}")
    for n in EXTRACT + MATCH:
        if n in per:
            d = per[n]
            print(f"  {n:28s} {len(d):8d} {sum(d) / len(d) / 1e3:9.1f} {sum(d) / 1e3:10.1f} {ov[n] / sum(d):10.1%}")


if __name__ == "__main__":
    main()
