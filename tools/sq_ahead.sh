#!/bin/bash
# SQ counters of the headline step's kernels (k_play, k_mt_ahead), two passes.
#   gpurun -- bash tools/sq_ahead.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cur}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-philox --no-mixed-league --no-dropin"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
python3 tools/sq_kernels.py $OUT/a/run_counter_collection.csv $OUT/b/run_counter_collection.csv > $OUT/sq.json
cat $OUT/sq.json
