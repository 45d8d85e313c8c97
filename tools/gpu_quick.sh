#!/bin/bash
# Quick GPU pass while iterating on a kernel: GPU tests (optionally -k), then
# the k_play time breakdown.  gpurun -- bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-quick}
mkdir -p $OUT
K=${2:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python tools/breakdown.py > $OUT/breakdown.log 2>&1 || { tail -20 $OUT/breakdown.log; exit 1; }
cat $OUT/breakdown.log
