"""Per-kernel summary (CSV) of a rocprofv3 --kernel-trace database
(<dir>/run_results.db, rocpd SQLite): name, calls, average / min / max
duration (us), total (ms), share of the traced kernel time.

usage: python tools/db_kstats.py gpurun_out/<tag>/<prof dir> [out.csv]
"""
import csv
import sqlite3
import sys
from pathlib import Path


def kernel_rows(db_path):
    db = sqlite3.connect(str(db_path))
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else [c for c in cols if "name" in c.lower()][0]
    q = (f"select {name}, count(*), avg(end - start), min(end - start), max(end - start), sum(end - start) "
         f"from kernels group by {name} order by 6 desc")
    rows = list(db.execute(q))
    total = sum(r[5] for r in rows) or 1
    return [(n, c, a / 1e3, lo / 1e3, hi / 1e3, s / 1e6, 100.0 * s / total) for n, c, a, lo, hi, s in rows]


def main():
    src = Path(sys.argv[1])
    db = src if src.suffix == ".db" else src / "run_results.db"
    rows = kernel_rows(db)
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["kernel", "calls", "avg_us", "min_us", "max_us", "total_ms", "percent"])
    for r in rows:
        w.writerow([r[0], r[1]] + [f"{x:.3f}" for x in r[2:]])


if __name__ == "__main__":
    main()
