#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM
traffic for one kernel, with the gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): counters are in KB;
FETCH_SIZE reads 1/2 of the bytes of wide coalesced streams, so it is
doubled (an upper estimate for narrower accesses); WRITE_SIZE is exact for
16-B-per-lane stores.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV KERNEL_SUBSTR OUT_JSON [note]
"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path, kernel, counter):
    vals = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    note = sys.argv[5] if len(sys.argv) > 5 else ""
    f = per_dispatch(fetch_csv, kernel, "FETCH_SIZE")
    w = per_dispatch(write_csv, kernel, "WRITE_SIZE")
    f_kb, w_kb = sum(f) / len(f), sum(w) / len(w)
    rec = {
        "kernel": kernel,
        "dispatches": {"fetch": len(f), "write": len(w)},
        "fetch_size_kb_raw": f_kb,
        "write_size_kb_raw": w_kb,
        "fetch_bytes_corrected": 2.0 * f_kb * 1024.0,
        "write_bytes": w_kb * 1024.0,
        "traffic_bytes_per_launch": 2.0 * f_kb * 1024.0 + w_kb * 1024.0,
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream under-count), KB -> bytes x1024",
        "note": note,
    }
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
