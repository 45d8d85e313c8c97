export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1 || true
for mode in numpy philox; do
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex k_play --output-format csv -d $R/gpurun_out/pmc/sq_$mode -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --rng $mode > $R/gpurun_out/pmc/sq_$mode.log 2>&1 || exit 1
  timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_play --output-format csv -d $R/gpurun_out/pmc/fetch_$mode -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --rng $mode > $R/gpurun_out/pmc/fetch_$mode.log 2>&1 || exit 1
  timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_play --output-format csv -d $R/gpurun_out/pmc/write_$mode -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --rng $mode > $R/gpurun_out/pmc/write_$mode.log 2>&1 || exit 1
  timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT --kernel-include-regex k_play --output-format csv -d $R/gpurun_out/pmc/sq2_$mode -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --rng $mode > $R/gpurun_out/pmc/sq2_$mode.log 2>&1 || echo "sq2 failed $mode"
done
echo done
