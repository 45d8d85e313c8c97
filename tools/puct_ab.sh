#!/bin/bash
# config-4 leg A/B: hipBLASLt heuristics vs the committed TunableOp selections, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-puct_ab}
mkdir -p $OUT
for rep in 1 2; do
  for mode in none tuned; do
    if [ $mode = none ]; then export SECHS_PUCT_TUNED=/nonexistent; else unset SECHS_PUCT_TUNED; fi
    timeout -k 10 300 python bench.py --only puct > $OUT/$mode.$rep.json 2> $OUT/$mode.$rep.err || { echo "fail $mode $rep"; exit 1; }
    python -c "import json,sys; r=json.load(open(sys.argv[1]))['extra_config4_puct']; print(sys.argv[2], round(r['value']/1e6,1), 'M', r['gemm_selection'])" $OUT/$mode.$rep.json $mode
  done
done
