#!/usr/bin/env python3
"""Kernel busy time vs span of a rocprofv3 kernel trace (last N seconds of it):
how much of the wall the GPU spends between kernels.  usage: busy_span.py trace.csv [tail_s]"""
import csv
import sys

ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
tail = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
end = max(k[1] for k in ks)
ks = [k for k in ks if k[0] >= end - tail * 1e9]
span = (ks[-1][1] - ks[0][0]) / 1e6
busy, cur_s, cur_e = 0.0, None, None
for s, e, _ in ks:  # union of intervals
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += (cur_e - cur_s) / 1e6
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += (cur_e - cur_s) / 1e6
by = {}
for s, e, n in ks:
    k = n.split("(")[0][:60]
    by[k] = by.get(k, 0.0) + (e - s) / 1e6
print(f"span {span:.1f} ms, busy {busy:.1f} ms ({100 * busy / span:.0f} %), kernels {len(ks)}")
for k, v in sorted(by.items(), key=lambda kv: -kv[1])[:8]:
    print(f"  {v:8.1f} ms  {k}")
