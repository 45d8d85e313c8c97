#!/bin/bash
# config-4 kernel traces: whole-rollout kernel vs launch per step (durations per launch)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-puct_trace}
mkdir -p $OUT
cd /tmp
for ro in 1 0; do
  SECHS_PUCT_ROLLOUTS=$ro timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ro$ro -o run -- python3 $R/bench.py --only puct --puct-games 8192 > $OUT/ro$ro.log 2>&1 || { tail $OUT/ro$ro.log; exit 1; }
  head -8 $OUT/ro$ro/run_kernel_stats.csv | cut -c1-160
done
echo done
