#!/bin/bash
# SN_OPT_TWIST_EVERY groups: env parity suite at K = 1 (default), 2, 3 (whole-round and exact-lead twists),
# then timing (tools/fused_diag.py) per K / round.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-groups}
mkdir -p $OUT
P="timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread"
$P > $OUT/pytest_k1.log 2>&1; rc=$?; tail -2 $OUT/pytest_k1.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=3 $P > $OUT/pytest_k3.log 2>&1; rc=$?; tail -2 $OUT/pytest_k3.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=2 $P -k "pipelined or oracle or round or quad" > $OUT/pytest_k2.log 2>&1; rc=$?; tail -2 $OUT/pytest_k2.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=2 SECHS_TEST_TWIST_ROUND=0 $P -k "pipelined or oracle or round or quad" > $OUT/pytest_k2r0.log 2>&1; rc=$?; tail -2 $OUT/pytest_k2r0.log; [ $rc -ne 0 ] && exit $rc
run() { env "$@" timeout -k 10 120 python tools/fused_diag.py >> $OUT/diag.jsonl 2>> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }; tail -1 $OUT/diag.jsonl | cut -c1-330; }
for rep in 1 2; do
  run FD_QUAD=0 FD_EVERY=1 FD_ROUND=0
  run FD_QUAD=0 FD_EVERY=2 FD_ROUND=0
  run FD_QUAD=0 FD_EVERY=3 FD_ROUND=0
  run FD_QUAD=0 FD_EVERY=2 FD_ROUND=1
  run FD_QUAD=1 FD_EVERY=3 FD_ROUND=0
done
echo done
