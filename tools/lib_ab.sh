#!/bin/bash
# A/B of two library builds on the config-2 legs (numpy + philox):
#   gpurun -- bash tools/lib_ab.sh <tag> libA.so libB.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-lib_ab}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for L in $2 $3; do
    SECHS_LIB=$R/rl-6-nimmt_amd/$L timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu --no-mcs --no-puct --no-scalar --no-league > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));p=d['extra_config2_philox'];print('$L numpy %.3e ms %.4f k %.4f | philox %.3e ms %.4f k %.4f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],p['value'],p['ms_per_step'],p['roofline']['kernel_ms']))"
  done
done
