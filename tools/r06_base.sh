#!/bin/bash
# r06 first GPU call: fresh phase split of the K = 4 default k_play,
# headline kernel trace + per-group-position timeline, PMC FETCH / WRITE / SQ passes
# with the twist dispatch kinds split.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_base}
mkdir -p $OUT
cd $R
SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_devprof.so timeout -k 10 180 python tools/phase_prof.py 65536 40 numpy > $OUT/phase.json 2> $OUT/phase.err || { tail $OUT/phase.err; exit 1; }
cat $OUT/phase.json
timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 20 > $OUT/bench_head.json 2> $OUT/bench_head.err && python tools/ab_line.py head $OUT/bench_head.json base
cd /tmp
B="python3 $R/bench.py --only headline --steps 40 --warmup 8"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- $B > $OUT/kstats.log 2>&1 || { tail $OUT/kstats.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || { tail $OUT/write.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/sq2 -o run -- $B > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
cd $R
python3 tools/group_trace.py $OUT/kstats/run_kernel_trace.csv 4 > $OUT/groups.json && cat $OUT/groups.json
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv "k_play<4|k_mt_ahead<false|k_mt_ahead<true" $OUT/traffic_numpy.json "config2 numpy, K = 4 whole-round twists (one steady twist per four play launches), 65536 games x 10 env-steps per play launch" && cat $OUT/traffic_numpy.json
python3 tools/sq_kernels.py $OUT/sq/run_counter_collection.csv > $OUT/sq.json && python3 tools/sq_kernels.py $OUT/sq2/run_counter_collection.csv > $OUT/sq2.json && cat $OUT/sq.json
echo done
