#!/bin/bash
# r06: a default bench, the headline's rocprof kernel stats + per-group-position timeline, PMC FETCH /
# WRITE / SQ passes (twist kinds split, k_decode included), and the config-4 rollout kernel phase split
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_final}
mkdir -p $OUT
cd $R
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 500 python bench.py > $OUT/bench_1.json 2> $OUT/bench_1.err
rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail $OUT/bench_1.err; exit 1; }
python tools/ab_line.py head $OUT/bench_1.json bench rep=1
python tools/ab_line.py puct $OUT/bench_1.json bench
python tools/ab_line.py mixed $OUT/bench_1.json bench
cd /tmp
B="python3 $R/bench.py --only headline --steps 40 --warmup 8"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- $B > $OUT/kstats.log 2>&1 || { tail $OUT/kstats.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_play|k_mt_ahead|k_decode" --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_play|k_mt_ahead|k_decode" --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || { tail $OUT/write.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_play|k_mt_ahead|k_decode" --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
cd $R
head -6 $OUT/kstats/run_kernel_stats.csv
python3 tools/group_trace.py $OUT/kstats/run_kernel_trace.csv 4 > $OUT/groups.json && cat $OUT/groups.json
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv "k_play<4|k_mt_ahead<false|k_decode|k_mt_ahead<true" $OUT/traffic_numpy.json "config2 numpy, decode-ahead (K = 4: one steady twist on one side stream and one k_decode of the next group's episode records on another per four play launches), 65536 games x 10 env-steps per play launch" && cat $OUT/traffic_numpy.json
python3 tools/sq_kernels.py $OUT/sq/run_counter_collection.csv > $OUT/sq.json && cat $OUT/sq.json
SECHS_PIPE_DEC=1 SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_devprof.so timeout -k 10 200 python tools/phase_prof.py 65536 40 numpy > $OUT/phase_headline.json && cat $OUT/phase_headline.json
SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_prof.so timeout -k 10 300 python tools/puct_phase_prof.py 8192 > $OUT/phase_puct.json && cat $OUT/phase_puct.json
echo done
