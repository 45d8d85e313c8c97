#!/bin/bash
# One GPU-box pass for a development round: the GPU test suite (or a -k
# subset), the headline bench without the slow legs, and optional extra bench
# legs.  Each GPU step has its own time limit; a crash / abort / timeout
# (rc >= 124) ends the script, a plain test failure (rc 1) does not.
#   gpurun -- bash tools/gpu_round.sh <tag> [pytest -k expr] [bench --only legs]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cur}
K=${2:-}
LEGS=${3:-}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
if [ "$K" != "none" ]; then
  if [ -n "$K" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/gpu_tests.log 2>&1
  else
    timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  fi
  rc=$?; tail -25 $OUT/gpu_tests.log; fatal $rc pytest
fi
timeout -k 10 300 python bench.py --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin > $OUT/bench_head.json 2> $OUT/bench_head.err
rc=$?; tail -3 $OUT/bench_head.err; fatal $rc bench_head
python - $OUT/bench_head.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("HEAD", round(r["value"] / 1e9, 3), "G/s ms", round(r["ms_per_step"], 4), "k_play", round(r["roofline"]["kernel_ms"] * 1e3, 1),
      "us ahead", round((r["roofline"]["concurrent"] or {}).get("kernel_ms", 0) * 1e3, 1), "us philox",
      round(r.get("extra_config2_philox", {}).get("value", 0) / 1e9, 3))
PY
if [ -n "$LEGS" ]; then
  timeout -k 10 600 python bench.py --only $LEGS ${BENCH_ARGS:-} > $OUT/bench_legs.json 2> $OUT/bench_legs.err
  rc=$?; tail -3 $OUT/bench_legs.err; cat $OUT/bench_legs.json | cut -c1-3000; fatal $rc bench_legs
fi
echo done
