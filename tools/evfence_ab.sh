#!/bin/bash
# A/B: pipeline events with the default system-scope release vs device scope
# (hipEventDisableSystemFence), headline leg on the dev library.
#   gpurun -- bash tools/evfence_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-evf}
mkdir -p $OUT
export SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_dev.so
for sf in 0 1 0 1; do
  SECHS_EV_SYSFENCE=$sf timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-philox > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('sysfence=$sf value %.3e ms/step %.4f k_play %.4f ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
done
