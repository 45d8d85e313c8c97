#!/bin/bash
# rocprof kernel stats of one bench leg (default: the drop-in search path).
#   gpurun -- bash tools/prof_dropin.sh <tag> [leg]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dropin}
LEG=${2:-dropin}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --only $LEG > $OUT/leg.json 2> $OUT/leg.err
rc=$?; tail -3 $OUT/leg.err; cut -c1-3000 $OUT/leg.json; [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
cd $R && python3 tools/kstats.py $TAG 20 && rm -rf $OUT/prof
echo done
