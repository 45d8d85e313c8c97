#!/bin/bash
# run.py league leg A/B: the league's PUCT engines with whole-rollout kernels (SECHS_PUCT_ROLLOUTS=1) or the
# launch-per-step loop (default), interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_mixed}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for ro in 0 1; do
    SECHS_PUCT_ROLLOUTS=$ro timeout -k 10 300 python bench.py --only mixed > $OUT/m_${ro}_$rep.json 2> $OUT/m_${ro}_$rep.err || { tail $OUT/m_${ro}_$rep.err; exit 1; }
    echo "rollouts=$ro rep=$rep"; python tools/ab_line.py mixed $OUT/m_${ro}_$rep.json
  done
done
