#!/bin/bash
# r04: kernel trace of the run.py league leg on the final tree (summarised on the box, database removed)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_league_prof}
mkdir -p $OUT
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/bench.py --only mixed > $OUT/kt.log 2>&1)
rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/db_kstats.py $OUT/kt $OUT/league_kernel_stats.csv && head -12 $OUT/league_kernel_stats.csv | cut -c1-160
find $R/gpurun_out -name "*.db" -size +1M -delete
echo done
