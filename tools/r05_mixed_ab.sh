#!/bin/bash
# run.py league leg (config 5, training on): whole-rollout PUCT kernel vs launch per step
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-mixed_ab}
mkdir -p $OUT
for rep in 1 2; do
  for ro in 1 0; do
    nm=mixed_ro${ro}_$rep
    SECHS_PUCT_ROLLOUTS=$ro timeout -k 10 400 python bench.py --only mixed > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
    python - $OUT/$nm.json $ro <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["extra_config5_run_py_league"]
ph = d.get("phases") or {}
top = sorted(((k, v) for k, v in ph.items() if isinstance(v, (int, float))), key=lambda kv: -kv[1])[:4]
print("rollouts-kernel", sys.argv[2], "s/round %.3f" % d.get("s_per_round", 0), "games/s %.0f" % d.get("games_per_s", 0), top)
PY
  done
done
echo done
