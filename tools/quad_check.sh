#!/bin/bash
# k_play_quad bring-up on the GPU box: parity vs the oracle (full size and
# ragged), the env GPU tests, an interleaved headline A/B (quad 1 vs 0) and a
# kernel trace of the quad headline.
#   gpurun -- bash tools/quad_check.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-quad}
mkdir -p $OUT
timeout -k 10 240 python -u tools/dev_parity.py 65536 30 > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
timeout -k 10 120 python -u tools/dev_parity.py 1000 23 >> $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
cat $OUT/parity.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_env.log 2>&1
rc=$?; tail -3 $OUT/pytest_env.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for qd in 1 0; do
    timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 10 --play-quad $qd > $OUT/bench_q${qd}_$rep.json 2> $OUT/bench_q${qd}_$rep.err || { tail $OUT/bench_q${qd}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_q${qd}_$rep.json'));r=d['roofline'];print('quad $qd value %.3e ms/step %.4f k_play %.4f ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms']))"
  done
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --only headline --steps 50 --warmup 10 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; [ $rc -ne 0 ] && { echo "prof rc=$rc"; exit $rc; }
find $OUT/prof -name "*kernel_stats.csv" -exec head -6 {} \;
echo done
