#!/bin/bash
# r04 iteration: PUCT + ACER + league GPU tests, config-4 leg x2 (+ kernel stats), run.py league leg (phases)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_it}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_puct.py tests/test_gpu_acer.py tests/test_gpu_league.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; fatal $rc pytest
[ $rc -ne 0 ] && exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --only puct > $OUT/puct_$rep.json 2> $OUT/puct_$rep.err
  rc=$?; fatal $rc puct
  python tools/ab_line.py puct $OUT/puct_$rep.json rep=$rep
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_puct -o run -- python3 $R/bench.py --only puct > $OUT/prof_puct.log 2>&1)
rc=$?; echo "rocprof puct rc=$rc"; fatal $rc rocprof_puct
python3 tools/db_kstats.py $OUT/prof_puct $OUT/puct_kernel_stats.csv
python3 tools/step_by_t.py $OUT/prof_puct > $OUT/puct_by_t.txt; cat $OUT/puct_by_t.txt
find $R/gpurun_out -name "*.db" -size +1M -delete
timeout -k 10 400 python bench.py --only mixed > $OUT/mixed.json 2> $OUT/mixed.err
rc=$?; fatal $rc mixed
python tools/ab_line.py mixed $OUT/mixed.json
echo done
