#!/bin/bash
# decode-ahead diagnostics: solo kernel times (SECHS_PIPE_SERIAL=1) and SQ counters of k_decode / k_play
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_decdiag}
LIB=${2:-$R/rl-6-nimmt_amd/libsechs_dev.so}
mkdir -p $OUT
cd $R
SECHS_LIB=$LIB SECHS_PIPE_SERIAL=1 timeout -k 10 200 python bench.py --only headline --steps 100 --warmup 10 > $OUT/serial.json 2> $OUT/serial.err || { tail $OUT/serial.err; exit 1; }
python tools/ab_line.py head $OUT/serial.json serial
cd /tmp
SECHS_LIB=$LIB timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_play|k_mt_ahead|k_decode" --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --only headline --steps 20 --warmup 5 > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
SECHS_LIB=$LIB timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "k_play|k_mt_ahead|k_decode" --output-format csv -d $OUT/sq2 -o run -- python3 $R/bench.py --only headline --steps 20 --warmup 5 > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
cd $R
python3 tools/sq_kernels.py $OUT/sq/run_counter_collection.csv > $OUT/sq.json && python3 tools/sq_kernels.py $OUT/sq2/run_counter_collection.csv > $OUT/sq2.json && cat $OUT/sq.json $OUT/sq2.json
