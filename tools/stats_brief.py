"""Short per-kernel summary of a rocprofv3 --stats kernel_stats.csv: name, calls, average us."""
import csv
import sys

for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        name = r["Name"].split("(")[0].replace("orbx::", "")
        print("  %-28s %5s calls  avg %8.1f us" % (name, r["Calls"], float(r["AverageNs"]) / 1e3))
