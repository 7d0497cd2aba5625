"""Per-kernel VALU / LDS wave-instructions per launch from a tools/pmc_sq.sh
summary (profiles/r02_sq_counters_serial.txt) -> JSON that bench.py reads for
the VALU-issue figure next to its HBM roofline.
Usage: python tools/sq_valu.py SUMMARY.txt OUT.json"""
import json
import sys

out, cur = {}, None
for line in open(sys.argv[1]):
    if not line.startswith(" "):
        cur = line.strip().split("(")[0].replace("void ", "").replace("orbx::", "")
        out[cur] = {}
        continue
    parts = line.split()
    if len(parts) >= 2 and parts[0].startswith(("SQ_", "GRBM_")):
        out[cur][parts[0]] = float(parts[1])
res = {k: {"valu_per_launch": v.get("SQ_INSTS_VALU"), "lds_per_launch": v.get("SQ_INSTS_LDS"),
           "salu_per_launch": v.get("SQ_INSTS_SALU"), "waves_per_launch": v.get("SQ_WAVES")}
       for k, v in out.items() if "SQ_INSTS_VALU" in v and "rocclr" not in k}
json.dump(res, open(sys.argv[2], "w"), indent=1, sort_keys=True)
print(json.dumps(res, indent=1, sort_keys=True))
