#!/bin/bash
# r04 profile pass of the final kernels: headline kernel trace (+ gap analysis),
# PMC traffic (numpy + philox), SQ counters of the config-3/4 kernels.
#   gpurun -- bash tools/r04_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 $R/bench.py --steps 100 --warmup 3 --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --no-philox"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
python3 $R/tools/trace_gaps.py $OUT/kt/run_kernel_trace.csv > $OUT/gaps.txt 2>&1; cat $OUT/gaps.txt
cd $R
timeout -k 10 400 bash tools/pmc_config2.sh $TAG > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
tail -3 $OUT/pmc.log
timeout -k 10 600 bash tools/sq_extras.sh $TAG > $OUT/sqx.log 2>&1 || { tail $OUT/sqx.log; exit 1; }
tail -30 $OUT/sqx.log
echo done
