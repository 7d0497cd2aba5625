"""Device timeline of single-frame orbx_extract calls from a rocprofv3 trace
(--kernel-trace --memory-copy-trace --output-format csv of tools/latency_prof.py):
per call, the H2D copy, the five kernels, the D2H copies and the gaps between
them; medians over the calls after the first `skip`.
  python tools/single_timeline.py DIR/run_kernel_trace.csv DIR/run_memory_copy_trace.csv [skip]"""
import csv
import sys
from collections import defaultdict

import numpy as np


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("orbx::", "")
    return n.split("<")[0]


def main():
    kt, mt = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    ev = []
    for r in csv.DictReader(open(kt)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    for r in csv.DictReader(open(mt)):
        d = r.get("Direction", r.get("Operation", ""))
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "H2D" if "HOST_TO_DEVICE" in d.upper() else
                   "D2H" if "DEVICE_TO_HOST" in d.upper() else d))
    ev.sort()
    # graph memcpy nodes run as blit kernels (__amd_rocclr_copyBuffer): a call
    # starts at the copy right before a pyramid launch (the H2D of its image)
    calls, cur = [], None
    for i, e in enumerate(ev):
        if e[2].startswith("__amd_rocclr_copy") and i + 1 < len(ev) and ev[i + 1][2] == "pyr_band_kernel":
            if cur:
                calls.append(cur)
            cur = [(e[0], e[1], "H2D copy")]
        elif cur is not None:
            cur.append((e[0], e[1], "D2H copy" if e[2].startswith("__amd_rocclr_copy") else e[2]))
    if cur:
        calls.append(cur)
    calls = calls[skip:]
    seg = defaultdict(list)
    for c in calls:
        t0 = c[0][0]
        prev_end = None
        names = defaultdict(int)
        for s, e, n in c:
            k = n if names[n] == 0 else f"{n}#{names[n]}"
            names[n] += 1
            if prev_end is not None:
                seg[f"gap before {k}"].append((s - prev_end) / 1e3)
            seg[k].append((e - s) / 1e3)
            prev_end = max(prev_end or 0, e)
        seg["total (first start -> last end)"].append((prev_end - t0) / 1e3)
    print(f"{len(calls)} calls; medians (us):")
    for k, v in seg.items():
        print(f"  {k:45s} {np.median(v):8.1f}")


if __name__ == "__main__":
    main()
