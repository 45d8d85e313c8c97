#!/usr/bin/env python3
"""Per-kernel SQ summary (rocprofv3 --pmc csv files): totals over every
dispatch of each kernel name, per-wave means and the wave-cycle split.
SQ_*_CYCLES count quad-cycles (MI355X_MICROARCH.md constants table)."""
import csv
import json
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add((path, r["Dispatch_Id"]))
out = {}
for name, c in tot.items():
    w = c.get("SQ_WAVES", 0.0) or 1.0
    d = {k: v for k, v in c.items()}
    d["dispatches_per_pass"] = len(disp[name]) / max(1, len(sys.argv) - 1)
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if k in c:
                d[k + "_frac"] = round(c[k] / wc, 3)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        if k in c:
            d[k + "_per_wave"] = round(c[k] / w, 1)
    out[name] = d
print(json.dumps(out, indent=1))
