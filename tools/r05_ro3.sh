#!/bin/bash
# whole-rollout kernel, 32-seat groups (two waves per SIMD): PUCT equality + config-4 A/B
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ro3}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_puct.py -x -v --timeout 200 --timeout-method thread -k "fused_rollouts or league_puct" > $OUT/pytest_puct.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" $OUT/pytest_puct.log | tail -8; [ $rc -ne 0 ] && exit $rc
for ro in 1 0; do
  SECHS_PUCT_ROLLOUTS=$ro timeout -k 10 300 python bench.py --only puct > $OUT/puct_ro$ro.json 2> $OUT/puct_ro$ro.err || { tail $OUT/puct_ro$ro.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/puct_ro$ro.json'))['extra_config4_puct'];print('config4 rollouts-kernel $ro: %.3e playout env-steps/s, %.1f TFLOP/s'%(d['value'],d['policy_tflops']))"
done
echo done
