#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-puct_wall}
mkdir -p $OUT
timeout -k 10 300 python -u tools/puct_wall.py > $OUT/wall.log 2>&1; rc=$?; head -60 $OUT/wall.log; exit $rc
