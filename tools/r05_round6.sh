#!/bin/bash
# three-phase whole-round twists in k_mt_ahead: env parity (round default, K = 2 / 3), timing
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-round6}
mkdir -p $OUT
P="timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread"
$P > $OUT/pytest_k1.log 2>&1; rc=$?; tail -2 $OUT/pytest_k1.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=2 $P -k "pipelined or oracle or round or quad" > $OUT/pytest_k2.log 2>&1; rc=$?; tail -2 $OUT/pytest_k2.log; [ $rc -ne 0 ] && exit $rc
run() { env "$@" timeout -k 10 120 python tools/fused_diag.py >> $OUT/diag.jsonl 2>> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }; tail -1 $OUT/diag.jsonl | cut -c1-330; }
for rep in 1 2; do
  run FD_QUAD=0 FD_EVERY=1 FD_ROUND=0
  run FD_QUAD=0 FD_EVERY=1 FD_ROUND=1
  run FD_QUAD=0 FD_EVERY=2 FD_ROUND=1
  run FD_QUAD=0 FD_EVERY=1 FD_ROUND=1 SECHS_PIPE_SERIAL=1
  run FD_QUAD=0 FD_EVERY=1 FD_ROUND=0 SECHS_PIPE_SERIAL=1
done
echo done
