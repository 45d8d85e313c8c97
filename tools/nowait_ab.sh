#!/bin/bash
# Measurement only: the numpy step with and without the cross-stream wait on
# the twist-ahead event (SECHS_NOWAIT, a -DSECHS_DEBUG_NOWAIT build; racy).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/nowait
mkdir -p $OUT
export SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_devx.so
for nw in "" 1 "" 1; do
  SECHS_NOWAIT=$nw timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-philox > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('nowait=${nw:-0} ms/step %.4f k_play %.4f ahead %.4f'%(d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
done
