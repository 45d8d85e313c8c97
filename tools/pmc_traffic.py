#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-bench-step HBM
traffic, with the gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md
(HBM section): counters are in KB; FETCH_SIZE reads 1/2 of the bytes of wide
coalesced streams, so it is doubled (an upper estimate for narrower
accesses); WRITE_SIZE is exact for 16-B-per-lane stores.

KERNELS is one or more kernel-name substrings separated by '|'.  Each gets its
mean traffic per dispatch and its dispatch count; the FIRST kernel is the play
launch that defines a bench step, and every other kernel is priced per step by
its measured dispatches per play dispatch (the K-group pipeline runs one
steady twist, k_mt_ahead<false, per K play launches).  A kernel whose name
matches `k_mt_ahead<true` (the pipeline's start-up twist, once per pipeline
start, not per step) is recorded but left out of the step traffic.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV KERNELS OUT_JSON [note]
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
    fetch_csv, write_csv, kernels, out = sys.argv[1:5]
    note = sys.argv[5] if len(sys.argv) > 5 else ""
    rec = {"kernels": {}, "correction": "FETCH_SIZE x2 (gfx950 wide-stream under-count), KB -> bytes x1024",
           "note": note}
    tot = 0.0
    names = kernels.split("|")
    plays = None
    for k in names:
        f = per_dispatch(fetch_csv, k, "FETCH_SIZE")
        w = per_dispatch(write_csv, k, "WRITE_SIZE")
        if not f or not w:  # a kernel this path does not launch
            continue
        f_kb, w_kb = sum(f) / len(f), sum(w) / len(w)
        b = 2.0 * f_kb * 1024.0 + w_kb * 1024.0
        rec["kernels"][k] = {"dispatches": {"fetch": len(f), "write": len(w)}, "fetch_size_kb_raw": f_kb,
                             "write_size_kb_raw": w_kb, "fetch_bytes_corrected": 2.0 * f_kb * 1024.0,
                             "write_bytes": w_kb * 1024.0, "traffic_bytes_per_dispatch": b}
        if plays is None:
            plays = len(f)
        ratio = len(f) / plays
        rec["kernels"][k]["dispatches_per_play_launch"] = ratio
        if "k_mt_ahead<true" in k:
            rec["kernels"][k]["in_step_traffic"] = False
            continue
        tot += b * ratio
    rec["play_dispatches"] = plays
    rec["step_traffic_bytes"] = tot
    rec["step_traffic_rule"] = ("sum over kernels of traffic_bytes_per_dispatch x dispatches_per_play_launch "
                                "(the start-up twist k_mt_ahead<true excluded)")
    rec["traffic_bytes_per_launch"] = tot
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
