#!/bin/bash
# headline A/B over pipeline options, concurrent (as benched) and serial
# (SECHS_PIPE_SERIAL=1: solo kernel times), two interleaved repetitions.
#   gpurun -- bash tools/r05_ab.sh <tag> "<round every quad>" ...
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ab}
shift
CFGS=("$@")
mkdir -p $OUT
for rep in 1 2; do
  for ser in 0 1; do
    for cfg in "${CFGS[@]}"; do
      set -- $cfg
      nm=b_r$1_k$2_q$3_s${ser}_$rep
      SECHS_PIPE_SERIAL=$ser timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --twist-round $1 --twist-every $2 --play-quad $3 > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/$nm.json'));r=d['roofline'];print('serial $ser round $1 every $2 quad $3: %.3e env-steps/s, ms/step %.4f, play %.4f, ahead %.4f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
    done
  done
done
echo done
