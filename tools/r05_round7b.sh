#!/bin/bash
# K-group pipeline with whole-round twists up to K = 4 (ring 4096): parity, timing; batched PUCT deal
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-round7}
mkdir -p $OUT
P="timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_puct.py -x -q --timeout 200 --timeout-method thread -k "batched_deal or seat_parallel or league_puct" > $OUT/pytest_puct.log 2>&1; rc=$?; tail -2 $OUT/pytest_puct.log; [ $rc -ne 0 ] && exit $rc
run() { env "$@" timeout -k 10 120 python tools/fused_diag.py >> $OUT/diag.jsonl 2>> $OUT/diag.err || { tail $OUT/diag.err; exit 1; }; tail -1 $OUT/diag.jsonl | cut -c1-330; }
for rep in 1 2; do
  run FD_QUAD=0 FD_EVERY=1 FD_ROUND=1
  run FD_QUAD=0 FD_EVERY=2 FD_ROUND=1
  run FD_QUAD=0 FD_EVERY=3 FD_ROUND=1
  run FD_QUAD=0 FD_EVERY=4 FD_ROUND=1
  run FD_QUAD=1 FD_EVERY=2 FD_ROUND=1
done
for rb in 16 0; do
  SECHS_PUCT_DEAL_BATCH=$rb timeout -k 10 300 python bench.py --only puct > $OUT/puct_rb$rb.json 2> $OUT/puct_rb$rb.err || { tail $OUT/puct_rb$rb.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/puct_rb$rb.json'))['extra_config4_puct'];print('config4 deal batch $rb: %.3e playout env-steps/s, %.1f TFLOP/s'%(d['value'],d['policy_tflops']))"
done
echo done
