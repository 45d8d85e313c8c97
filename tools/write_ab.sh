#!/bin/bash
# Is the role-split kernel bound by its output stores?  Headline leg with and
# without the int8 obs (126 of the ~152 MB written per launch), both RNG
# modes and split settings; plus the host enqueue rate (tools/host_rate.py).
#   gpurun -- bash tools/write_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-write_ab}
mkdir -p $OUT
export SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_dev.so
for rng in philox numpy; do
  for sp in 0 1 3; do
    [ $rng = philox ] && [ $sp = 3 ] && continue
    [ $rng = numpy ] && [ $sp = 1 ] && continue
    for obs in "" "--no-obs"; do
      timeout -k 10 120 python bench.py --steps 50 --warmup 3 --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-philox --rng $rng --play-split $sp $obs > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('$rng split=$sp obs=${obs:-yes} value %.3e ms/step %.4f kernel %.4f'%(d['value'],d['ms_per_step'],r['kernel_ms']))"
    done
  done
done
timeout -k 10 120 python tools/host_rate.py numpy 200 2> $OUT/h.err || { tail $OUT/h.err; exit 1; }
timeout -k 10 120 python tools/host_rate.py philox 200 2> $OUT/h.err || { tail $OUT/h.err; exit 1; }
