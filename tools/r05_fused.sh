#!/bin/bash
# SN_OPT_PIPE_FUSED bring-up: the quad equality test (fused / quad / one-lane),
# the env parity tests with SECHS_TEST_PIPE_FUSED=1, then a headline A/B.
#   gpurun -- bash tools/r05_fused.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-fused}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread -k "quad" > $OUT/pytest_quad.log 2>&1
rc=$?; tail -3 $OUT/pytest_quad.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_PIPE_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_env_fused.log 2>&1
rc=$?; tail -3 $OUT/pytest_env_fused.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for cfg in "0 0" "1 0" "1 1"; do
    set -- $cfg
    nm=b_f$1_s$2_$rep
    SECHS_PIPE_SERIAL=$2 timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --twist-round 0 --pipe-fused $1 > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$nm.json'));r=d['roofline'];print('fused $1 serial $2: %.3e env-steps/s, ms/step %.4f, play %.4f, ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
  done
done
echo done
