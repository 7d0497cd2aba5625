"""Summarise rocprofv3 --pmc CSVs: per kernel, mean counter value per dispatch."""
import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/pass*_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(float)
    for r in rows:
        key = (r["Kernel_Name"].split("(")[0], r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
    for (k, disp, c), v in per.items():
        acc[k][c].append(v)
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.1f}   (n={len(v)})")
