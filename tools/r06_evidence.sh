#!/bin/bash
# r06: full-size long parity against the oracle (decode-ahead default path, 65 536 games x 300 env-steps,
# numpy and philox, with and without obs), the default headline bench repeated (box spread), and the
# run.py league leg's kernel trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_evidence}
mkdir -p $O
cd $R
timeout -k 10 600 python tools/dev_parity.py 65536 300 > $O/parity.log 2>&1; rc=$?; cat $O/parity.log | grep parity; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --only headline > $O/head_$rep.json 2> $O/head_$rep.err || { tail $O/head_$rep.err; exit 1; }
  python tools/ab_line.py head $O/head_$rep.json rep=$rep
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/league -o run -- python3 $R/bench.py --only mixed > $O/league.log 2>&1 || { tail $O/league.log; exit 1; }
cd $R
head -12 $O/league/run_kernel_stats.csv | cut -c1-140
echo done
