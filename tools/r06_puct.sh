#!/bin/bash
# config-4 iteration: PUCT GPU tests, the k_puct_rollouts phase split, interleaved config-4 bench legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_puct}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_puct.py -x -q --timeout 240 --timeout-method thread -k "rollouts or mlp or league_puct or batched_deal or seat_parallel or statistics" > $OUT/pytest_puct.log 2>&1
rc=$?; tail -2 $OUT/pytest_puct.log; [ $rc -ne 0 ] && exit $rc
SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_prof.so timeout -k 10 300 python tools/puct_phase_prof.py 8192 > $OUT/phase_puct.json || exit 1
cat $OUT/phase_puct.json
for rep in 1 2; do
  timeout -k 10 200 python bench.py --only puct > $OUT/puct_$rep.json 2> $OUT/puct_$rep.err || { tail $OUT/puct_$rep.err; exit 1; }
  python tools/ab_line.py puct $OUT/puct_$rep.json rep=$rep
done
