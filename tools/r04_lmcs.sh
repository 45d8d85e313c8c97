#!/bin/bash
# r04: league MCS kernel (wave decisions inlined) -- MCS + league GPU tests, run.py league leg, kernel stats
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_lmcs}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mcs.py tests/test_gpu_league.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; fatal $rc pytest
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python bench.py --only mixed > $OUT/mixed.json 2> $OUT/mixed.err
rc=$?; fatal $rc mixed
python tools/ab_line.py mixed $OUT/mixed.json | cut -c1-400
timeout -k 10 200 python bench.py --only dropin > $OUT/dropin.json 2> $OUT/dropin.err
rc=$?; fatal $rc dropin
python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(r['extra_dropin_search'])" $OUT/dropin.json | cut -c1-300
echo done
