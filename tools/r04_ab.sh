#!/bin/bash
# r04: pipe hand-off modes A/B (0 events, 1 CP wait on a block count, 2 poll + event marker),
# (historical A/B: the SN_OPT_PIPE_FLAGS modes it selects were measured slower and removed from the
#  library -- DESIGN.md §4; SECHS_PIPE_FLAGS is ignored by the current build)
# persistent one-kernel PUCT MLP vs the GEMM form, rest of the GPU suite, league phases
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_ab}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_env.log 2>&1
rc=$?; tail -4 $OUT/tests_env.log; fatal $rc pytest_env
[ $rc -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_puct.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_puct.log 2>&1
rc=$?; tail -4 $OUT/tests_puct.log; fatal $rc pytest_puct
[ $rc -ne 0 ] && exit 1
for rep in 1 2; do
  for f in 0 2 1; do
    SECHS_PIPE_FLAGS=$f timeout -k 10 200 python bench.py --only headline > $OUT/head_f${f}_$rep.json 2> $OUT/head_f${f}_$rep.err
    rc=$?; fatal $rc head
    python tools/ab_line.py head $OUT/head_f${f}_$rep.json flags=$f rep=$rep
  done
done
for l1 in seats gemm; do
  SECHS_MLP_LAYER1=$l1 timeout -k 10 300 python bench.py --only puct > $OUT/puct_$l1.json 2> $OUT/puct_$l1.err
  rc=$?; fatal $rc puct
  python tools/ab_line.py puct $OUT/puct_$l1.json layer1=$l1
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_puct -o run -- python3 $R/bench.py --only puct > $OUT/prof_puct.log 2>&1)
rc=$?; echo "rocprof puct rc=$rc"; fatal $rc rocprof_puct
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_env.py --deselect tests/test_gpu_puct.py > $OUT/tests_rest.log 2>&1
rc=$?; tail -4 $OUT/tests_rest.log; fatal $rc pytest_rest
timeout -k 10 400 python bench.py --only mixed > $OUT/mixed.json 2> $OUT/mixed.err
rc=$?; fatal $rc mixed
python tools/ab_line.py mixed $OUT/mixed.json
echo done
