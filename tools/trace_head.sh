#!/bin/bash
# Kernel-trace timeline of the headline bench (numpy pipeline): per-launch
# start/end of k_play and k_mt_ahead, for the gap analysis (tools/gaps.py).
#   gpurun -- bash tools/trace_head.sh <tag> [extra bench args]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-trace}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --no-philox --steps 50 --warmup 10 "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -2 $OUT/bench.err; [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
echo done
