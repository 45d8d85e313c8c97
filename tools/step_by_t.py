"""Mean duration of each config-4 rollout kernel by rollout length n and
rollout step t (position after the rollout's k_puct_deal; n_cur = n - t)
from a rocprofv3 kernel-trace database.
usage: python tools/step_by_t.py <prof dir | run_results.db>"""
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    db = sqlite3.connect(path if path.endswith(".db") else os.path.join(path, "run_results.db"))
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else [c for c in cols if "name" in c.lower()][0]
    ks = sorted(db.execute(f"select start, end, {name} from kernels"))
    acc = defaultdict(list)  # (kind, n, t) -> durations; n = rollout steps of the rollout
    cur = []

    def flush():
        n = sum(1 for k, _ in cur if k == "mlp")
        t = {"mlp": -1}
        for k, d in cur:
            if k == "mlp":
                t["mlp"] += 1
            acc[(k, n, t["mlp"])].append(d)

    for a, b, n in ks:
        if "k_puct_deal" in n:
            flush()
            cur = []
        elif "k_puct_mlp_seats" in n:
            cur.append(("mlp", (b - a) / 1e3))
        elif "k_puct_step" in n:
            cur.append(("step", (b - a) / 1e3))
    flush()
    for (k, n, t), v in sorted(acc.items()):
        if n:
            print(f"{k} n={n} t={t} n_cur={n - t} calls={len(v)} mean_us={sum(v) / len(v):.1f}")


if __name__ == "__main__":
    main()
