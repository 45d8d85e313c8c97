#!/bin/bash
# kernel-trace timelines of the headline step (play / twist overlap, gaps) per pipeline option set
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-trace}
mkdir -p $OUT
cd /tmp
for d in 1 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_d$d -o run -- python3 $R/bench.py --only headline --steps 30 --warmup 5 --twist-round 0 --pipe-depth $d > $OUT/tr_d$d.log 2>&1 || { tail $OUT/tr_d$d.log; exit 1; }
  f=$(ls $OUT/tr_d$d/*kernel_trace.csv $OUT/tr_d$d/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/trace_gaps.py $f > $OUT/gaps_d$d.txt; head -12 $OUT/gaps_d$d.txt
done
echo done
