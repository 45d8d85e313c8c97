#!/bin/bash
# r04: rollout-MLP kernel iteration -- PUCT parity tests, config-4 leg x2, its kernel trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_mlp}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_puct.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_puct.log 2>&1
rc=$?; tail -2 $OUT/tests_puct.log; fatal $rc pytest_puct
[ $rc -ne 0 ] && exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --only puct > $OUT/puct_$rep.json 2> $OUT/puct_$rep.err
  rc=$?; fatal $rc puct
  python tools/ab_line.py puct $OUT/puct_$rep.json rep=$rep
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_puct -o run -- python3 $R/bench.py --only puct > $OUT/prof_puct.log 2>&1)
rc=$?; echo "rocprof puct rc=$rc"; fatal $rc rocprof_puct
python3 tools/db_kstats.py $OUT/prof_puct $OUT/puct_kernel_stats.csv && head -4 $OUT/puct_kernel_stats.csv | cut -c1-60,180-260
find $R/gpurun_out -name "*.db" -size +1M -delete
echo done
