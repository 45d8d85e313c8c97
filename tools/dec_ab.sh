#!/bin/bash
# Decode-ahead pipeline on one GPU box: its parity tests, then an interleaved
# headline A/B (pipe_dec 0 / 1 on the product library, and optionally 1 on a
# second build), then rocprof kernel stats of pipe_dec 1.
#   gpurun -- bash tools/dec_ab.sh <tag> [other.so] [reps]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dec}; OTHER=${2:-}; REPS=${3:-3}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe_dec.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
B="--no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --no-philox --steps 300 --warmup 20"
summ() { python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(r['value']/1e9,3), 'G ms', round(r['ms_per_step'],4), 'play', round(r['roofline']['kernel_ms']*1e3,1), 'ahead', round(r['roofline']['concurrent']['kernel_ms']*1e3,1))" $1 $2; }
for rep in $(seq 1 $REPS); do
  for v in dec0 dec1 other; do
    [ $v = other ] && [ -z "$OTHER" ] && continue
    if [ $v = other ]; then export SECHS_LIB=$R/$OTHER; D=1; else unset SECHS_LIB; D=${v#dec}; fi
    timeout -k 10 200 python bench.py $B --pipe-dec $D > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -3 $OUT/ab_$v.err; exit 1; }
    summ $OUT/ab_$v.json $v
  done
done
unset SECHS_LIB
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py $B --steps 50 --warmup 10 --pipe-dec 1 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; [ $rc -ne 0 ] && { echo "prof rc=$rc"; tail -3 $OUT/prof_bench.err; exit $rc; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -8 $OUT/kernel_stats.csv | cut -c1-150
echo done
