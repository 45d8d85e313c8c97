#!/bin/bash
# PMC passes for the headline bench step (k_play + k_mt_ahead in numpy mode,
# k_play alone in philox mode), separate passes per the gfx950 slot limits
# (FETCH_SIZE and WRITE_SIZE cannot share one).  On the GPU box:
#   gpurun -- bash tools/pmc_config2.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cur}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
for mode in numpy philox; do
  B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --no-philox --rng $mode"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_play|k_mt_ahead|k_mt_prep" --output-format csv -d $OUT/fetch_$mode -o run -- $B > $OUT/fetch_$mode.log 2>&1 || { tail $OUT/fetch_$mode.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_play|k_mt_ahead|k_mt_prep" --output-format csv -d $OUT/write_$mode -o run -- $B > $OUT/write_$mode.log 2>&1 || { tail $OUT/write_$mode.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_play|k_mt_ahead|k_mt_prep" --output-format csv -d $OUT/sq_$mode -o run -- $B > $OUT/sq_$mode.log 2>&1 || { tail $OUT/sq_$mode.log; exit 1; }
  K="k_play_split<4|k_play<4"; [ $mode = numpy ] && K="k_mt_ahead|k_mt_prep|k_play<4"
  python3 tools/pmc_traffic.py $OUT/fetch_$mode/run_counter_collection.csv $OUT/write_$mode/run_counter_collection.csv "$K" $OUT/traffic_$mode.json "config2 $mode, 65536 games x 10 env-steps per bench step" || exit 1
done
echo done
