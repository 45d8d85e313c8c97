#!/bin/bash
# config-4 bench (graph replay) kernel trace: GPU busy vs span over the timed game
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-puct_span}
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 $R/bench.py --only puct > $OUT/tr.log 2>&1 || { tail $OUT/tr.log; exit 1; }
python3 $R/tools/busy_span.py $OUT/tr/run_kernel_trace.csv 0.6
echo done
