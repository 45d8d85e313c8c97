#!/bin/bash
# A/B of SN_OPT_PLAY_SPLIT on the headline leg (dev library): 0 = one wave
# per game does everything, 2 = role-split over the pipelined ring, 3 =
# role-split with the MT19937 twist in the producer waves, 4 = role-split over
# the ring with the next launch's twist in the producer waves.
#   gpurun -- bash tools/split_ab.sh <tag> [modes]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/rl-6-nimmt_amd
OUT=$R/gpurun_out/ab_${1:-cur}
mkdir -p $OUT
for m in ${2:-4 3 2 0}; do
  SECHS_LIB=$L/libsechs_dev.so timeout -k 10 200 python bench.py --steps 50 --warmup 3 --no-cpu --no-mcs --no-puct --no-scalar --no-league --play-split $m > $OUT/b$m.json 2> $OUT/b$m.err || { tail -5 $OUT/b$m.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$m.json'));r=d['roofline'];print('split=$m value %.3e ms/step %.4f k_play %.4f ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms'] if r.get('concurrent') else None))"
done
