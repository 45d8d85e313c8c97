"""Per-kernel summary (calls, total, mean) of a rocprofv3 SQLite trace under
gpurun_out/<tag>/prof; writes gpurun_out/<tag>/kernel_stats.csv."""
import csv
import glob
import sqlite3
import sys

tag = sys.argv[1]
dbs = glob.glob(f"gpurun_out/{tag}/prof/**/*.db", recursive=True)
if not dbs:  # summarised on the GPU box already
    sys.exit(print(open(f"gpurun_out/{tag}/kernel_stats.csv").read()[:3000]))
db = dbs[0]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) from kernels "
                 "group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
with open(f"gpurun_out/{tag}/kernel_stats.csv", "w") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100 * r[2] / tot, 2)])
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{r[1]:7d} {r[2] / 1e6:9.2f} ms {r[3] / 1e3:9.2f} us {100 * r[2] / tot:5.1f}%  {r[0][:100]}")
