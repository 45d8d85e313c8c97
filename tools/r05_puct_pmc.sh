#!/bin/bash
# r05: kernel stats + SQ counters of the config-4 whole-rollout kernel (eager launches, tools/puct_eager.py)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_puct_pmc}
mkdir -p $OUT
K="k_puct_rollouts|k_puct_deal_batch"
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- python3 tools/puct_eager.py > $OUT/kstats.log 2>&1
rc=$?; echo "kstats rc=$rc"; [ $rc -ne 0 ] && { tail -4 $OUT/kstats.log; exit $rc; }
head -6 $OUT/kstats/run_kernel_stats.csv | cut -c1-150
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$K" --output-format csv -d $OUT/sq -o run -- python3 tools/puct_eager.py > $OUT/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -ne 0 ] && { grep -v "^    @" $OUT/sq.log | tail -4; exit $rc; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH --kernel-include-regex "$K" --output-format csv -d $OUT/sq2 -o run -- python3 tools/puct_eager.py > $OUT/sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; [ $rc -ne 0 ] && { grep -v "^    @" $OUT/sq2.log | tail -4; exit $rc; }
python3 tools/sq_kernels.py $OUT/sq/run_counter_collection.csv $OUT/sq2/run_counter_collection.csv > $OUT/sq_summary.json
cat $OUT/sq_summary.json | head -60
echo done
