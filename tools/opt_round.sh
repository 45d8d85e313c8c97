#!/bin/bash
# One GPU-box pass for a k_play change: the whole GPU suite + smoke on the
# product library, then an interleaved headline A/B against an older build.
#   gpurun -- bash tools/opt_round.sh <tag> <old.so> [reps]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-opt}; OLD=$2; REPS=${3:-3}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
B="--no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --steps 300 --warmup 20"
summ() { python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(r['value']/1e9,3), 'G ms', round(r['ms_per_step'],4), 'play', round(r['roofline']['kernel_ms']*1e3,1), 'ahead', round(r['roofline']['concurrent']['kernel_ms']*1e3,1), 'philox', round(r.get('extra_config2_philox',{}).get('value',0)/1e9,3))" $1 $2; }
for rep in $(seq 1 $REPS); do
  for v in new old; do
    if [ $v = old ]; then export SECHS_LIB=$R/$OLD; else unset SECHS_LIB; fi
    timeout -k 10 200 python bench.py $B > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -3 $OUT/ab_$v.err; exit 1; }
    summ $OUT/ab_$v.json $v
  done
done
echo done
