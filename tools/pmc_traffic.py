"""HBM-side traffic per kernel launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Usage: python tools/pmc_traffic.py OUT.json FETCH_DIR WRITE_DIR

Counters are collected in separate passes (FETCH_SIZE and WRITE_SIZE do not fit
one TCC pass) with --kernel-trace only. Both are reported in KiB per dispatch.
gfx950 correction (MI355X_MICROARCH.md, "HBM"): FETCH_SIZE reports half of
the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as
is. Infinity-Cache (MALL) hits are counted by these memory-side counters, so
the figure is "bytes that left L2", an upper bound on HBM bytes.
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            per[(r["Kernel_Name"].split("(")[0].split("::")[-1], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in per.items():
            acc[k].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    out, fdir, wdir = sys.argv[1:4]
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd"):
            continue
        f = 2.0 * fetch.get(k, 0.0) * 1024.0
        w = write.get(k, 0.0) * 1024.0
        res[k] = {"fetch_bytes_per_launch": round(f), "write_bytes_per_launch": round(w),
                  "bytes_per_launch": round(f + w),
                  "correction": "FETCH_SIZE x2 (gfx950 half-count), WRITE_SIZE x1; KiB -> B"}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:28s} {v['bytes_per_launch'] / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
