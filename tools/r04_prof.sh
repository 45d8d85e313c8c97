#!/bin/bash
# r04 profiles of the final tree: headline kernel trace, PMC traffic (tools/pmc_config2.sh),
# SQ counters of configs 3/4 (tools/sq_extras.sh), kernel trace of one run.py league leg.
# Databases are summarised on the box (tools/db_kstats.py) and removed: gpurun_out/ must stay < 64 MiB.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_prof}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
shrink() { find $R/gpurun_out -name "*.db" -size +1M -delete; find $R/gpurun_out -name "*kernel_trace.csv" -size +1M -delete; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_head -o run -- python3 bench.py --only headline --steps 20 > $OUT/kt_head.log 2>&1
rc=$?; echo "kt_head rc=$rc"; fatal $rc kt_head
[ $rc -ne 0 ] && { tail -5 $OUT/kt_head.log; exit 1; }
python3 tools/db_kstats.py $OUT/kt_head $OUT/kt_head_kernel_stats.csv && python3 tools/trace_gaps.py $OUT/kt_head > $OUT/kt_head_gaps.txt 2>&1; shrink
timeout -k 10 600 bash tools/pmc_config2.sh r04 > $OUT/pmc.log 2>&1
rc=$?; tail -2 $OUT/pmc.log; fatal $rc pmc
[ $rc -ne 0 ] && exit 1
shrink
timeout -k 10 900 bash tools/sq_extras.sh r04 > $OUT/sqx.log 2>&1
rc=$?; echo "sqx rc=$rc"; tail -8 $OUT/sqx.log; fatal $rc sqx
for f in $R/gpurun_out/sqx_r04/*.log; do echo "== $f"; tail -4 $f; done
shrink
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/kt_league -o run -- python3 bench.py --only mixed > $OUT/kt_league.log 2>&1
rc=$?; echo "kt_league rc=$rc"; fatal $rc kt_league
python3 tools/db_kstats.py $OUT/kt_league $OUT/kt_league_kernel_stats.csv; shrink
du -sh $R/gpurun_out
echo done
