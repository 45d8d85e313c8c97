#!/bin/bash
# pipeline bring-up: env GPU tests (parity, round boundaries, exports,
# overruns, quad equality, debug library) under the default options, the env
# parity tests again with SN_OPT_TWIST_EVERY 2 (SECHS_TEST_TWIST_EVERY), the
# new PUCT / drop-in pins, then an interleaved headline A/B.
#   gpurun -- bash tools/round_check.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-round}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_env.log 2>&1
rc=$?; tail -3 $OUT/pytest_env.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread -k "pipelined or oracle or round or quad" > $OUT/pytest_env_k2.log 2>&1
rc=$?; tail -3 $OUT/pytest_env_k2.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=2 SECHS_TEST_TWIST_ROUND=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread -k "pipelined or oracle or round or quad" > $OUT/pytest_env_k2r0.log 2>&1
rc=$?; tail -3 $OUT/pytest_env_k2r0.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_puct.py tests/test_gpu_dropin.py -k "trace or fp32_reference_net or in_law or reference_training_loss or module_forward" > $OUT/pytest_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|F14|Error" $OUT/pytest_new.log | tail -12; [ $rc -ge 124 ] && exit $rc
for rep in 1 2; do
  for cfg in "1 1 0" "1 2 0" "0 1 0" "1 2 1" "1 1 1"; do
    set -- $cfg
    nm=b_r$1_k$2_q$3_$rep
    timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --twist-round $1 --twist-every $2 --play-quad $3 > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$nm.json'));r=d['roofline'];print('round $1 every $2 quad $3: %.3e env-steps/s, ms/step %.4f, play %.4f, ahead %.4f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
  done
done
for l1 in mfma seats; do
  SECHS_MLP_LAYER1=$l1 timeout -k 10 300 python bench.py --only puct > $OUT/puct_$l1.json 2> $OUT/puct_$l1.err || { tail $OUT/puct_$l1.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/puct_$l1.json'))['extra_config4_puct'];print('config4 $l1: %.3e playout env-steps/s, %.1f TFLOP/s'%(d['value'],d['policy_tflops']))"
done
echo done
