#!/bin/bash
# GPU iteration pass: GPU tests, then the profiled headline leg.
#   gpurun -- bash tools/gpu_iter.sh <tag> [numpy|philox]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-iter}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/prof_play.sh ${1:-iter} ${2:-numpy}
