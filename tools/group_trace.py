#!/usr/bin/env python3
"""Per-position timeline of the K-group pipelined headline step from a
rocprofv3 --kernel-trace csv (diagnostics): k_play launches are numbered in
issue order; the one a steady twist (k_mt_ahead<false, ..>) starts beside is
position 0 of its group.  Prints, per position in the group, the mean k_play
duration and the mean gap from the previous k_play's end to its start, and
the twist's duration and its start relative to its play launch.

usage: group_trace.py kernel_trace.csv [K]
"""
import csv
import json
import sys
from statistics import mean


def main():
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(sys.argv[1]))]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows.sort()
    plays = [r for r in rows if "k_play" in r[2]]
    twists = [r for r in rows if "k_mt_ahead<false" in r[2]]
    # a twist belongs to the last play launch that started before it
    owner = {}
    for t in twists:
        i = max((k for k, p in enumerate(plays) if p[0] <= t[0]), default=None)
        if i is not None:
            owner[i] = t
    if not owner:
        print(json.dumps({"plays": len(plays), "twists": len(twists)}))
        return
    first = sorted(owner)
    pos = {}
    for i in range(len(plays)):
        starts = [f for f in first if f <= i]
        if starts and i - starts[-1] < K:
            pos[i] = i - starts[-1]
    # skip the first two groups (warmup / pipeline start)
    skip = first[min(2, len(first) - 1)]
    by = {k: {"dur_us": [], "gap_us": []} for k in range(K)}
    tw = {"dur_us": [], "start_after_play_us": [], "end_after_play_end_us": []}
    for i in range(max(skip, 1), len(plays)):
        if i not in pos:
            continue
        p, prev = plays[i], plays[i - 1]
        by[pos[i]]["dur_us"].append((p[1] - p[0]) / 1e3)
        by[pos[i]]["gap_us"].append((p[0] - prev[1]) / 1e3)
        if i in owner:
            t = owner[i]
            tw["dur_us"].append((t[1] - t[0]) / 1e3)
            tw["start_after_play_us"].append((t[0] - p[0]) / 1e3)
            tw["end_after_play_end_us"].append((t[1] - p[1]) / 1e3)
    out = {"plays": len(plays), "steady_twists": len(twists), "K": K, "groups_used": len(tw["dur_us"]),
           "by_position": {k: {m: round(mean(v), 2) if v else None for m, v in d.items()} | {"n": len(d["dur_us"])}
                           for k, d in by.items()},
           "twist": {m: round(mean(v), 2) if v else None for m, v in tw.items()}}
    allp = [d for k in by for d in by[k]["dur_us"]]
    allg = [d for k in by for d in by[k]["gap_us"]]
    if allp:
        out["period_us"] = round(mean(allp) + mean(allg), 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
