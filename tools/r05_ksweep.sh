#!/bin/bash
# headline + DrunkHamster tournament leg per twist cadence K (SECHS_TWIST_EVERY), interleaved
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ksweep}
mkdir -p $OUT
for rep in 1 2; do
  for k in 1 2 3 4; do
    nm=k${k}_$rep
    SECHS_TWIST_EVERY=$k timeout -k 10 300 python bench.py --only headline,league --steps 200 --warmup 10 > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$nm.json'));r=d['roofline'];l=d.get('extra_config5_tournament',{});print('K $k: %.3e env-steps/s, ms/step %.4f, play %.4f, ahead %s; league %.3e'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms'],l.get('value',0)))"
  done
done
echo done
