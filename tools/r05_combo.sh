#!/bin/bash
# ring 64-B chunks + whole-rollout PUCT kernel: parity (env suite at K = 2 / K = 1 exact-lead, PUCT equality),
# then the headline A/B (defaults vs the r04 pipeline) and config 4 (whole-rollout kernel vs launch per step)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-combo}
mkdir -p $OUT
P="timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread"
$P > $OUT/pytest_def.log 2>&1; rc=$?; tail -2 $OUT/pytest_def.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=1 SECHS_TEST_TWIST_ROUND=0 $P -k "pipelined or oracle or round or quad" > $OUT/pytest_k1r0.log 2>&1; rc=$?; tail -2 $OUT/pytest_k1r0.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_puct.py -x -v --timeout 200 --timeout-method thread -k "fused_rollouts or batched_deal or league_puct or seat_parallel" > $OUT/pytest_puct.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" $OUT/pytest_puct.log | tail -8; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for cfg in "2 1" "1 0"; do
    set -- $cfg
    nm=h_k$1_r$2_$rep
    timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --twist-every $1 --twist-round $2 > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$nm.json'));r=d['roofline'];print('every $1 round $2: %.3e env-steps/s, ms/step %.4f, play %.4f, ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
  done
done
for ro in 1 0; do
  SECHS_PUCT_ROLLOUTS=$ro timeout -k 10 300 python bench.py --only puct > $OUT/puct_ro$ro.json 2> $OUT/puct_ro$ro.err || { tail $OUT/puct_ro$ro.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/puct_ro$ro.json'))['extra_config4_puct'];print('config4 rollouts-kernel $ro: %.3e playout env-steps/s, %.1f TFLOP/s'%(d['value'],d['policy_tflops']))"
done
echo done
