#!/bin/bash
# SQ counter pass for the headline kernel (wave cycles split into issue /
# memory-wait / instruction-wait, VALU and LDS instruction counts).
#   gpurun -- bash tools/sq_pass.sh <tag> [numpy|philox]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cur}
MODE=${2:-numpy}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex k_play --output-format csv -d $OUT/sq -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-mcs --no-puct --rng $MODE > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --kernel-include-regex k_play --output-format csv -d $OUT/sq2 -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-mcs --no-puct --rng $MODE > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
python3 tools/sq_summary.py $OUT/sq/run_counter_collection.csv $OUT/sq2/run_counter_collection.csv
