#!/bin/bash
# SN_OPT_PIPE_DEPTH bring-up: env parity tests with SECHS_TEST_PIPE_DEPTH=2
# (whole-round and exact-lead twists), then timing (tools/fused_diag.py).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-depth}
mkdir -p $OUT
SECHS_TEST_PIPE_DEPTH=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_d2.log 2>&1
rc=$?; tail -3 $OUT/pytest_d2.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_PIPE_DEPTH=2 SECHS_TEST_TWIST_ROUND=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread -k "pipelined or oracle or round or quad" > $OUT/pytest_d2r0.log 2>&1
rc=$?; tail -3 $OUT/pytest_d2r0.log; [ $rc -ne 0 ] && exit $rc
run() { env "$@" timeout -k 10 120 python tools/fused_diag.py >> $OUT/diag.jsonl 2>> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }; tail -1 $OUT/diag.jsonl | cut -c1-400; }
for rep in 1 2; do
  run FD_QUAD=0 FD_DEPTH=1 FD_ROUND=0
  run FD_QUAD=0 FD_DEPTH=2 FD_ROUND=0
  run FD_QUAD=0 FD_DEPTH=2 FD_ROUND=1
  run FD_QUAD=1 FD_DEPTH=2 FD_ROUND=0
done
echo done
