#!/bin/bash
# Whole GPU suite + smoke on the product library, then the PUCT A/B of a
# variant build against it.  gpurun -- bash tools/final_ab.sh <tag> <variant.so>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VAR=$2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in prod var; do
    unset SECHS_LIB; [ $v = var ] && export SECHS_LIB=$R/$VAR
    timeout -k 10 400 python bench.py --only puct,mixed > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -3 $OUT/ab_$v.err; exit 1; }
    python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'puct', round(r['extra_config4_puct']['value']/1e6,1), 'M league s/round', round(r['extra_config5_run_py_league']['s_per_round'],3))" $OUT/ab_$v.json $v
  done
done
echo done
