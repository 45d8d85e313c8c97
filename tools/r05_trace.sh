#!/bin/bash
# kernel-trace timelines of the headline step (play / twist overlap, gaps) per twist cadence K
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-trace}
mkdir -p $OUT
cd /tmp
for k in 1 4; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_k$k -o run -- python3 $R/bench.py --only headline --steps 30 --warmup 5 --twist-round 0 --twist-every $k > $OUT/tr_k$k.log 2>&1 || { tail $OUT/tr_k$k.log; exit 1; }
  f=$(ls $OUT/tr_k$k/*kernel_trace.csv $OUT/tr_k$k/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/trace_gaps.py $f > $OUT/gaps_k$k.txt; head -12 $OUT/gaps_k$k.txt
done
echo done
