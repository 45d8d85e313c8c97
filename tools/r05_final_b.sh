#!/bin/bash
# r05_final.sh, then config 4 with the whole-rollout kernel (SECHS_PUCT_ROLLOUTS=1) beside the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/r05_final.sh ${1:-r05_final} || exit $?
OUT=$R/gpurun_out/${1:-r05_final}
cd $R
for ro in 1 0; do
  SECHS_PUCT_ROLLOUTS=$ro timeout -k 10 300 python bench.py --only puct > $OUT/puct_ro$ro.json 2> $OUT/puct_ro$ro.err || { tail $OUT/puct_ro$ro.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/puct_ro$ro.json'))['extra_config4_puct'];print('config4 rollouts-kernel $ro: %.3e playout env-steps/s, %.1f TFLOP/s'%(d['value'],d['policy_tflops']))"
done
echo done_b
