#!/bin/bash
# whole-rollout kernel, layer 1 per candidate on MFMA: PUCT equality + config-4 A/B vs the seats form
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-mf}
mkdir -p $OUT
SECHS_TEST_MF_ROLLOUTS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_puct.py -x -v --timeout 250 --timeout-method thread -k "fused_rollouts or league_puct or statistics_match_reference" > $OUT/pytest_puct.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" $OUT/pytest_puct.log | tail -8; [ $rc -ne 0 ] && exit $rc
for l1 in mfma seats; do
  SECHS_MLP_LAYER1=$l1 timeout -k 10 300 python bench.py --only puct > $OUT/puct_$l1.json 2> $OUT/puct_$l1.err || { tail $OUT/puct_$l1.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/puct_$l1.json'))['extra_config4_puct'];print('config4 $l1: %.3e playout env-steps/s, %.1f TFLOP/s'%(d['value'],d['policy_tflops']))"
done
echo done
