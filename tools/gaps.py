"""Timeline of the pipelined numpy rollout from a rocprofv3 kernel trace
(tools/trace_head.sh): per k_play launch, the gap before it, the k_mt_ahead
running beside it (start offset, end relative to k_play's end)."""
import glob
import sqlite3
import sys

import numpy as np

db = glob.glob(f"gpurun_out/{sys.argv[1]}/prof/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
play = [(s, e) for n, s, e in rows if n.startswith("void k_play<")]
ahead = [(s, e) for n, s, e in rows if n.startswith("void k_mt_ahead<false")]
play, ahead = np.array(play[-60:], dtype=np.int64), np.array(ahead, dtype=np.int64)
print("launches", len(play), "play us", np.mean(play[:, 1] - play[:, 0]) / 1e3)
gaps = (play[1:, 0] - play[:-1, 1]) / 1e3
per = (play[1:, 0] - play[:-1, 0]) / 1e3
print("period us mean %.1f median %.1f | gap mean %.1f median %.1f" % (per.mean(), np.median(per), gaps.mean(), np.median(gaps)))
# the twist beside play launch i: the one that starts inside it
out = []
for s, e in play[:-1]:
    k = np.searchsorted(ahead[:, 0], s)
    if k < len(ahead):
        a0, a1 = ahead[k]
        out.append(((a0 - s) / 1e3, (a1 - a0) / 1e3, (a1 - e) / 1e3))
out = np.array(out)
print("ahead: start after play start %.1f us, duration %.1f us, end after play end %.1f us (median %.1f)"
      % (out[:, 0].mean(), out[:, 1].mean(), out[:, 2].mean(), np.median(out[:, 2])))
for i in range(5):
    print(" ", play[i + 10, 0] - play[10, 0], play[i + 10, 1] - play[10, 0], out[i + 10])
