#!/bin/bash
# whole-round twist bring-up: env GPU tests (parity, round boundaries,
# exports, overruns, quad equality, debug library), the new PUCT / drop-in
# pins, then an interleaved headline A/B over (twist_round, play_quad).
#   gpurun -- bash tools/round_check.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-round}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_env.log 2>&1
rc=$?; tail -3 $OUT/pytest_env.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_puct.py -k "fp32_reference_net or in_law or reference_training_loss" tests/test_gpu_dropin.py -k "trace or fp32_reference_net or in_law or reference_training_loss" > $OUT/pytest_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|F14|Error" $OUT/pytest_new.log | tail -12; [ $rc -ge 124 ] && exit $rc
for rep in 1 2; do
  for tr in 1 0; do
    for qd in 0 1; do
      timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --twist-round $tr --play-quad $qd > $OUT/b_t${tr}_q${qd}_$rep.json 2> $OUT/b_t${tr}_q${qd}_$rep.err || { tail $OUT/b_t${tr}_q${qd}_$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/b_t${tr}_q${qd}_$rep.json'));r=d['roofline'];print('twist_round $tr quad $qd: %.3e env-steps/s, ms/step %.4f, play %.4f, ahead %.4f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
    done
  done
done
echo done
