#!/bin/bash
# r05: the whole GPU suite, smoke(), a default bench, the headline's rocprof kernel stats and PMC
# traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs), SQ counters of the headline kernels
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_final}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; fatal $rc pytest
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; fatal $rc smoke
fi
timeout -k 10 400 python bench.py > $OUT/bench_1.json 2> $OUT/bench_1.err
rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail $OUT/bench_1.err; exit 1; }
python tools/ab_line.py head $OUT/bench_1.json bench rep=1
cd /tmp
B="python3 $R/bench.py --only headline --steps 20 --warmup 5"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- $B > $OUT/kstats.log 2>&1 || { tail $OUT/kstats.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || { tail $OUT/write.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
cd $R
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv "k_mt_ahead|k_play<4" $OUT/traffic_numpy.json "config2 numpy (r05 defaults: whole-round twists, one per two launches), 65536 games x 10 env-steps per launch" && cat $OUT/traffic_numpy.json
python3 tools/sq_kernels.py $OUT/sq/run_counter_collection.csv > $OUT/sq.json && cat $OUT/sq.json
echo done
