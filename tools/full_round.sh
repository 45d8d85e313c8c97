#!/bin/bash
# Round-end validation on one GPU box: the whole GPU suite, smoke(), the
# default bench line (all legs), rocprof kernel stats of the headline.
#   gpurun -- bash tools/full_round.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-full}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -2 $OUT/bench.err; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --steps 50 --warmup 10 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; [ $rc -ne 0 ] && { echo "prof rc=$rc"; exit $rc; }
echo done
