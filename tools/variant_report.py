"""Summarise gpurun_out/var/ (tools/variant_sweep.sh)."""
import glob
import json
import os
import sys

names = sys.argv[1:] or sorted({os.path.basename(p).split(".")[0] for p in glob.glob("gpurun_out/var/*.json")})
for v in names:
    try:
        t = open("gpurun_out/var/%s.test.log" % v).read().strip().splitlines()[-1]
        s = json.load(open("gpurun_out/var/%s.serial.json" % v))
        b = [json.load(open("gpurun_out/var/%s.b%d.json" % (v, i)))["value"] for i in (1, 2)]
    except (OSError, ValueError, IndexError) as e:
        print(v, "incomplete:", e)
        continue
    st = " ".join("%s=%.1f" % (k[:6], 1000 * x) for k, x in s["stage_ms_per_batch"].items())
    print("%-8s %-22s serial %7.0f  pipe %7.0f %7.0f  | %s" % (v, t[:22], s["value"], b[0], b[1], st))
