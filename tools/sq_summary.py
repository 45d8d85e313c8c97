#!/usr/bin/env python3
"""Per-wave SQ counter summary for the largest k_play launches (rocprofv3
csv).  SQ_*_CYCLES count quad-cycles (MI355X_MICROARCH.md constants table)."""
import csv
import sys
from collections import defaultdict

rows = defaultdict(dict)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        rows[(path, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[(path, r["Dispatch_Id"])]["grid"] = int(r["Grid_Size"])
agg = defaultdict(list)
for (path, _), v in rows.items():
    big = max(x["grid"] for (p, _), x in rows.items() if p == path)
    if v["grid"] == big:
        for k, x in v.items():
            agg[k].append(x)
mean = {k: sum(v) / len(v) for k, v in agg.items()}
w = mean.get("SQ_WAVES", 1.0)
out = {k: round(v / w, 1) for k, v in mean.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
if "SQ_WAVE_CYCLES" in mean:
    wc = mean["SQ_WAVE_CYCLES"]
    out["cycles_per_wave"] = round(4 * wc / w)
    for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
        out[k + "_frac"] = round(mean[k] / wc, 3)
print(out)
