#!/bin/bash
# r05_final.sh (K = 4 default), then K = 5 parity and a K = 4 / 5 same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/r05_final.sh r05_final3 || exit $?
OUT=$R/gpurun_out/r05_final3
cd $R
SECHS_TEST_TWIST_EVERY=5 timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_k5.log 2>&1; rc=$?; tail -2 $OUT/pytest_k5.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for k in 4 5; do
    nm=k${k}_$rep
    timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --twist-every $k > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$nm.json'));r=d['roofline'];print('K $k: %.3e env-steps/s, ms/step %.4f, play %.4f'%(d['value'],d['ms_per_step'],r['kernel_ms']))"
  done
done
echo done3
