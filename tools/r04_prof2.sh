#!/bin/bash
# r04: headline-only kernel trace, SQ counters of config 3 (MCS) and config 4 (PUCT) in separate runs
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_prof2}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
shrink() { find $R/gpurun_out -name "*.db" -size +1M -delete; find $R/gpurun_out -name "*kernel_trace.csv" -size +1M -delete; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_head -o run -- python3 bench.py --only headline --steps 20 > $OUT/kt_head.log 2>&1
rc=$?; echo "kt_head rc=$rc"; fatal $rc kt_head
[ $rc -ne 0 ] && { tail -5 $OUT/kt_head.log; exit 1; }
python3 tools/db_kstats.py $OUT/kt_head $OUT/kt_head_kernel_stats.csv && python3 tools/trace_gaps.py $OUT/kt_head > $OUT/kt_head_gaps.txt 2>&1; shrink
cat $OUT/kt_head_gaps.txt | head -8
for leg in mcs puct; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_mcs_rollouts|k_puct_step|k_puct_mlp|k_puct_deal" --output-format csv -d $OUT/sq_$leg -o run -- python3 tools/extras_only.py $leg > $OUT/sq_$leg.log 2>&1
  rc=$?; echo "sq $leg rc=$rc"; fatal $rc sq_$leg
  [ $rc -ne 0 ] && { grep -v "^    @" $OUT/sq_$leg.log | tail -4; continue; }
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --kernel-include-regex "k_mcs_rollouts|k_puct_step|k_puct_mlp|k_puct_deal" --output-format csv -d $OUT/sq2_$leg -o run -- python3 tools/extras_only.py $leg > $OUT/sq2_$leg.log 2>&1
  rc=$?; echo "sq2 $leg rc=$rc"; fatal $rc sq2_$leg
  [ $rc -ne 0 ] && { grep -v "^    @" $OUT/sq2_$leg.log | tail -4; continue; }
  python3 tools/sq_kernels.py $OUT/sq_$leg/run_counter_collection.csv $OUT/sq2_$leg/run_counter_collection.csv > $OUT/sq_summary_$leg.json
  shrink
done
du -sh $R/gpurun_out
echo done
