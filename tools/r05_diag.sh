#!/bin/bash
# fused-twist timing diagnostics (tools/fused_diag.py), no parity
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-diag}
mkdir -p $OUT
run() { env "$@" timeout -k 10 120 python tools/fused_diag.py >> $OUT/diag.jsonl 2>> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }; tail -1 $OUT/diag.jsonl; }
for rep in 1 2; do
  run FD_QUAD=0 FD_FUSED=0 SECHS_PIPE_SERIAL=1
  run FD_QUAD=1 FD_FUSED=0 SECHS_PIPE_SERIAL=1
  run FD_QUAD=1 FD_FUSED=1
  run FD_QUAD=1 FD_FUSED=1 SECHS_QUAD_DBG=8
  run FD_QUAD=1 FD_FUSED=1 SECHS_QUAD_DBG=16
  run FD_QUAD=1 FD_FUSED=1 SECHS_QUAD_DBG=12
done
echo done
