#!/bin/bash
# r04: ACER split-K weight gradients -- GPU ACER/league tests, learn() profile, run.py league leg (split-K on / off)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_acer2}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_acer.py tests/test_gpu_league.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; fatal $rc pytest
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python tools/acer_profile.py > $OUT/prof.txt 2>&1
rc=$?; fatal $rc acerprof
grep "learn()" $OUT/prof.txt
for k in 1 0; do
  SECHS_ACER_SPLITK=$k timeout -k 10 400 python bench.py --only mixed > $OUT/mixed_$k.json 2> $OUT/mixed_$k.err
  rc=$?; fatal $rc mixed
  echo "splitk=$k"; python tools/ab_line.py mixed $OUT/mixed_$k.json | cut -c1-400
done
echo done
