#!/bin/bash
# SQ counters (instruction mix, wave-cycle split) and kernel trace of the
# config-3 MCS and config-4 PUCT legs.   gpurun -- bash tools/sq_extras.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sqx_${1:-cur}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/extras_only.py both > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_mcs_rollouts|k_puct_step|k_puct_rows|k_puct_mlp|k_puct_seat" --output-format csv -d $OUT/sq -o run -- python3 tools/extras_only.py both > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --kernel-include-regex "k_mcs_rollouts|k_puct_step|k_puct_rows|k_puct_mlp|k_puct_seat" --output-format csv -d $OUT/sq2 -o run -- python3 tools/extras_only.py both > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
python3 tools/sq_kernels.py $OUT/sq/run_counter_collection.csv $OUT/sq2/run_counter_collection.csv > $OUT/sq_summary.json
cat $OUT/sq_summary.json
