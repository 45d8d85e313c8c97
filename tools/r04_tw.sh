#!/bin/bash
# r04: the in-launch pipeline (SN_OPT_PIPE_FLAGS = 3, k_play_tw) -- parity, then headline A/B vs events (0)
# (historical A/B: the SN_OPT_PIPE_FLAGS modes it selects were measured slower and removed from the
#  library -- DESIGN.md §4; SECHS_PIPE_FLAGS is ignored by the current build)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_tw}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread -k "pipe" > $OUT/tests_pipe.log 2>&1
rc=$?; tail -2 $OUT/tests_pipe.log; fatal $rc pytest_pipe
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_league.py -x -q --timeout 120 --timeout-method thread -k "slots_replay" > $OUT/tests_league.log 2>&1
rc=$?; tail -2 $OUT/tests_league.log; fatal $rc pytest_league
[ $rc -ne 0 ] && exit 1
for rep in 1 2 3; do
  for f in 0 3; do
    SECHS_PIPE_FLAGS=$f timeout -k 10 200 python bench.py --only headline > $OUT/head_f${f}_$rep.json 2> $OUT/head_f${f}_$rep.err
    rc=$?; fatal $rc head
    python tools/ab_line.py head $OUT/head_f${f}_$rep.json flags=$f rep=$rep
  done
done
(cd /tmp && SECHS_PIPE_FLAGS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_head3 -o run -- python3 $R/bench.py --only headline --steps 20 > $OUT/prof_head3.log 2>&1)
rc=$?; echo "rocprof head3 rc=$rc"; fatal $rc rocprof_head3
echo done
