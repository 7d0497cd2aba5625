"""Per-call device timeline of synchronous calls from a rocprofv3 trace
(--kernel-trace [--memory-copy-trace] --output-format csv): the events are
split into calls at device-idle gaps longer than --gap us, and for each event
position of a call the median start (relative to the call's first event),
duration and stream are printed; calls whose event sequence differs from the
most common one are skipped.
  python tools/call_timeline.py DIR/run_kernel_trace.csv [--copies DIR/run_memory_copy_trace.csv] [--gap 20] [--skip 30]"""
import argparse
import csv
from collections import Counter

import numpy as np


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("orbx::", "")
    n = n.split("<")[0]
    return "copy (blit)" if n.startswith("__amd_rocclr_copy") else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--copies")
    ap.add_argument("--gap", type=float, default=20.0)
    ap.add_argument("--skip", type=int, default=30)
    a = ap.parse_args()
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Stream_Id", ""))
          for r in csv.DictReader(open(a.trace))]
    if a.copies:
        for r in csv.DictReader(open(a.copies)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "sdma " + r["Direction"].replace("MEMORY_COPY_", ""),
                       r.get("Stream_Id", "")))
    ev.sort()
    calls, cur, end = [], [], 0
    for e in ev:
        if cur and e[0] - end > a.gap * 1e3:
            calls.append(cur)
            cur = []
        end = max(end, e[1]) if cur else e[1]
        cur.append(e)
    if cur:
        calls.append(cur)
    calls = calls[a.skip:]
    sig = Counter(tuple(e[2] for e in c) for c in calls)
    common, n = sig.most_common(1)[0]
    calls = [c for c in calls if tuple(e[2] for e in c) == common]
    print(f"{len(calls)} calls with the common sequence of {len(common)} events (of {sum(sig.values())}); medians, us:")
    print(f"  {'event':32s} {'stream':>6s} {'start':>8s} {'dur':>8s} {'end':>8s}")
    for i, name in enumerate(common):
        st = np.median([(c[i][0] - c[0][0]) / 1e3 for c in calls])
        du = np.median([(c[i][1] - c[i][0]) / 1e3 for c in calls])
        en = np.median([(c[i][1] - c[0][0]) / 1e3 for c in calls])
        print(f"  {name:32s} {calls[0][i][3]:>6s} {st:8.1f} {du:8.1f} {en:8.1f}")
    tot = [(max(e[1] for e in c) - c[0][0]) / 1e3 for c in calls]
    print(f"  call span (first start -> last end): median {np.median(tot):.1f} us")


if __name__ == "__main__":
    main()
