#!/bin/bash
# One GPU-box pass: GPU parity tests, the default bench line, and a rocprofv3
# kernel-trace summary of the same bench command.  Every GPU step has its own
# time limit and the chain stops at the first failure.
#   gpurun -- bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cur}
K=${2:-}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
fi
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
head -5 $OUT/prof/run_kernel_stats.csv | cut -c1-200
echo done
