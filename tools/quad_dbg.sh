#!/bin/bash
# k_play_quad store-path diagnostics (solo kernel times, SECHS_PIPE_SERIAL=1,
# dev library): SECHS_QUAD_DBG bit 0 plain stores for rewards/actions/done,
# bit 1 skip them, bit 2 skip the state stores (timing only).
#   gpurun -- bash tools/quad_dbg.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-qdbg}
mkdir -p $OUT
cd /tmp
run() {  # name, dbg, bench args
  local nm=$1 dbg=$2; shift 2
  SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_dev.so SECHS_PIPE_SERIAL=1 SECHS_QUAD_DBG=$dbg timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$nm -o run -- python3 $R/bench.py --only headline --steps 40 --warmup 5 --no-cpu --play-quad 1 "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; return 1; }
  echo "$nm: $(grep k_play_quad $OUT/$nm/run_kernel_stats.csv | cut -d, -f4)"
}
run d0 0 && run d1 1 && run d2 2 && run d6 6 && run d6_noobs 6 --no-obs && run d2_noobs 2 --no-obs && run d0_noobs 0 --no-obs && echo done
