#!/bin/bash
# Targeted parity (N = 4 tests, smoke) of a dev build, then an interleaved
# 3-way headline A/B: dev build, product library, an older build.
#   gpurun -- bash tools/ab3.sh <tag> <dev.so> <old.so> [reps]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; DEV=$2; OLD=$3; REPS=${4:-3}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export SECHS_LIB=$R/$DEV
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ring_options or (play_split and 4) or bench_lanes or full_size_episode or interleave" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
B="--no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --steps 300 --warmup 20"
summ() { python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(r['value']/1e9,3), 'G ms', round(r['ms_per_step'],4), 'play', round(r['roofline']['kernel_ms']*1e3,1), 'ahead', round(r['roofline']['concurrent']['kernel_ms']*1e3,1), 'philox', round(r.get('extra_config2_philox',{}).get('value',0)/1e9,3))" $1 $2; }
for rep in $(seq 1 $REPS); do
  for v in dev prod old; do
    unset SECHS_LIB
    [ $v = dev ] && export SECHS_LIB=$R/$DEV
    [ $v = old ] && export SECHS_LIB=$R/$OLD
    timeout -k 10 200 python bench.py $B > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -3 $OUT/ab_$v.err; exit 1; }
    summ $OUT/ab_$v.json $v
  done
done
echo done
