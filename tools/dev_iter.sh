#!/bin/bash
# Kernel iteration on the GPU box with the N=4 development libraries:
# parity vs the oracle, k_play phase split, headline bench leg.
#   gpurun -- bash tools/dev_iter.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dev}
mkdir -p $OUT
L=$R/rl-6-nimmt_amd
SECHS_LIB=$L/libsechs_dev.so timeout -k 10 240 python -u tools/dev_parity.py 65536 30 > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
cat $OUT/parity.log
SECHS_LIB=$L/libsechs_devprof.so timeout -k 10 120 python -u tools/phase_prof.py 65536 20 numpy > $OUT/phase.json 2> $OUT/phase.err || { tail $OUT/phase.err; exit 1; }
cat $OUT/phase.json
SECHS_LIB=$L/libsechs_dev.so timeout -k 10 200 python bench.py --steps 50 --warmup 3 --no-cpu --no-mcs --no-puct --no-scalar --no-league > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('value %.3e ms/step %.4f k_play %.4f ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms'] if r.get('concurrent') else None))"
