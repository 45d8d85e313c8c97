#!/bin/bash
# Bandwidth probes of the headline step (timing only, results not checked):
# product, product without obs output, and a build whose k_mt_ahead skips the
# MT write-back (SECHS_PROBE_NO_MT_STORE).  gpurun -- bash tools/probe_ab.sh <tag> <probe.so> [reps]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-probe}; PROBE=$2; REPS=${3:-3}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
B="--no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --no-philox --steps 300 --warmup 20"
summ() { python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(r['value']/1e9,3), 'G ms', round(r['ms_per_step'],4), 'play', round(r['roofline']['kernel_ms']*1e3,1), 'ahead', round(r['roofline']['concurrent']['kernel_ms']*1e3,1))" $1 $2; }
for rep in $(seq 1 $REPS); do
  for v in prod noobs probe; do
    unset SECHS_LIB; X=""
    [ $v = noobs ] && X="--no-obs"
    [ $v = probe ] && export SECHS_LIB=$R/$PROBE
    timeout -k 10 200 python bench.py $B $X > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -3 $OUT/ab_$v.err; exit 1; }
    summ $OUT/ab_$v.json $v
  done
done
echo done
