#!/bin/bash
# k_pipe_code (one wave per game) parity, then a same-box interleaved headline A/B:
# r05 defaults (K = 2, whole rounds) vs the r04 pipeline (K = 1, exact-lead twists)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ab2}
mkdir -p $OUT
P="timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread"
$P > $OUT/pytest_def.log 2>&1; rc=$?; tail -2 $OUT/pytest_def.log; [ $rc -ne 0 ] && exit $rc
SECHS_TEST_TWIST_EVERY=4 SECHS_TEST_TWIST_ROUND=0 $P -k "pipelined or oracle or round or quad" > $OUT/pytest_k4r0.log 2>&1; rc=$?; tail -2 $OUT/pytest_k4r0.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for cfg in "2 1" "1 0" "3 1"; do
    set -- $cfg
    nm=h_k$1_r$2_$rep
    timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --twist-every $1 --twist-round $2 > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$nm.json'));r=d['roofline'];print('every $1 round $2: %.3e env-steps/s, ms/step %.4f, play %.4f, ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
  done
done
echo done
