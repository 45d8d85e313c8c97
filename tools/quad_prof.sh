#!/bin/bash
# k_play_quad diagnostics on the GPU box: phase split (devprof library) for
# quad 1 / 0, and SQ counters of the headline step.
#   gpurun -- bash tools/quad_prof.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-qprof}
mkdir -p $OUT
L=$R/rl-6-nimmt_amd
for qd in 1 0; do
  SECHS_PLAY_QUAD=$qd SECHS_LIB=$L/libsechs_devprof.so timeout -k 10 120 python -u tools/phase_prof.py 65536 20 numpy > $OUT/phase_q$qd.json 2> $OUT/phase_q$qd.err || { tail $OUT/phase_q$qd.err; exit 1; }
  cat $OUT/phase_q$qd.json
done
B="python3 $R/bench.py --only headline --steps 5 --warmup 1 --no-cpu"
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/sq1 -o run -- $B > $OUT/sq1.log 2>&1 || { tail $OUT/sq1.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAVES --kernel-include-regex "k_play|k_mt_ahead" --output-format csv -d $OUT/sq2 -o run -- $B > $OUT/sq2.log 2>&1 || { tail $OUT/sq2.log; exit 1; }
python3 $R/tools/sq_kernels.py $OUT/sq1/run_counter_collection.csv > $OUT/sq1.json && python3 $R/tools/sq_kernels.py $OUT/sq2/run_counter_collection.csv > $OUT/sq2.json && cat $OUT/sq1.json $OUT/sq2.json
echo done
