#!/bin/bash
# SQ counters of the config-4 (PUCT) kernels, two passes over a reduced
# config-4 game (2048 games; the kernels' shapes per decision as at 8192).
#   gpurun -- bash tools/sq_puct.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-puct}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
B="python3 tools/puct_sq_run.py"
RX="k_puct_step|k_puct_h1|k_puct_seat|k_puct_deal"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "$RX" --output-format csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU --kernel-include-regex "$RX" --output-format csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
python3 tools/sq_kernels.py $OUT/a/run_counter_collection.csv $OUT/b/run_counter_collection.csv > $OUT/sq.json
rm -rf $OUT/a $OUT/b
cat $OUT/sq.json | cut -c1-3000
