#!/bin/bash
# r04: the whole GPU suite, smoke(), two default bench runs (league spread), on the final tree
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_final}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; fatal $rc pytest
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; fatal $rc smoke
for rep in 1 2; do
  timeout -k 10 400 python bench.py > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err
  rc=$?; fatal $rc bench
  python tools/ab_line.py head $OUT/bench_$rep.json bench rep=$rep
  python - $OUT/bench_$rep.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("extra_config4_puct", "extra_config5_run_py_league", "extra_config5_tournament", "extra_config3_mcs"):
    x = r.get(k) or {}
    print(k, x.get("value"), x.get("unit"), x.get("s_per_round"), x.get("games_per_s"))
PY
done
echo done
