#!/usr/bin/env python3
"""Step timeline of the pipelined bench from a rocprofv3 --kernel-trace csv:
per step, k_play and k_mt_ahead start/end relative to the previous k_play's
end (shows the cross-stream hand-off gaps).  Usage: trace_gaps.py kernel_trace.csv | run_results.db | <dir>"""
import csv
import sys

def load(path):
    """(start, end, name) of every kernel: a kernel_trace.csv, or a rocpd
    database (run_results.db, or the directory holding it)"""
    if path.endswith(".csv"):
        return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
    import os
    import sqlite3

    db = sqlite3.connect(path if path.endswith(".db") else os.path.join(path, "run_results.db"))
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else [c for c in cols if "name" in c.lower()][0]
    return [(int(a), int(b), n) for a, b, n in db.execute(f"select start, end, {name} from kernels")]


ks = [k for k in load(sys.argv[1]) if "k_play" in k[2] or "k_mt_ahead" in k[2]]
ks.sort()
plays = [k for k in ks if "k_play" in k[2]]
aheads = [k for k in ks if "k_mt_ahead<false" in k[2]]
print("plays", len(plays), "aheads", len(aheads))
gaps, durs, adurs, periods = [], [], [], []
for a, b in zip(plays[-60:-1], plays[-59:]):
    gaps.append((b[0] - a[1]) / 1e3)
    durs.append((a[1] - a[0]) / 1e3)
    periods.append((b[0] - a[0]) / 1e3)
for a in aheads[-60:]:
    adurs.append((a[1] - a[0]) / 1e3)
m = lambda v: sum(v) / max(len(v), 1)
print(f"k_play dur {m(durs):.1f} us, gap to next k_play {m(gaps):.1f} us, period {m(periods):.1f} us, k_mt_ahead dur {m(adurs):.1f} us")
# relation: ahead start/end vs play windows
for a, b in zip(plays[-6:-1], plays[-5:]):
    inside = [x for x in aheads if a[0] - 200000 <= x[0] <= b[0]]
    s = " ".join(f"ahead[{(x[0]-a[0])/1e3:.1f},{(x[1]-a[0])/1e3:.1f}]" for x in inside)
    print(f"play[0,{(a[1]-a[0])/1e3:.1f}] next play at {(b[0]-a[0])/1e3:.1f}  {s}")
