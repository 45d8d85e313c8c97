#!/bin/bash
# Solo vs concurrent kernel times of the headline step (diagnostics):
# SECHS_PIPE_SERIAL=1 runs each k_mt_ahead after the play launch before it
# (no overlap), so rocprof's per-kernel averages are solo times.
#   gpurun -- bash tools/quad_variants.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-qvar}
mkdir -p $OUT
cd /tmp
run() {  # name, env, bench args
  local nm=$1; shift
  env "$1" timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$nm -o run -- python3 $R/bench.py --only headline --steps 50 --warmup 5 --no-cpu "${@:2}" > $OUT/$nm.json 2> $OUT/$nm.err || { tail $OUT/$nm.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$nm.json'));print('$nm ms/step %.4f'%d['ms_per_step'])"
  find $OUT/$nm -name "*kernel_stats.csv" -exec sed -n 2,3p {} \;
}
run q1_conc SECHS_PIPE_SERIAL=0 --play-quad 1 && run q0_conc SECHS_PIPE_SERIAL=0 --play-quad 0 && \
run q1_serial SECHS_PIPE_SERIAL=1 --play-quad 1 && run q0_serial SECHS_PIPE_SERIAL=1 --play-quad 0 && \
run q1_noobs SECHS_PIPE_SERIAL=0 --play-quad 1 --no-obs && run q0_noobs SECHS_PIPE_SERIAL=0 --play-quad 0 --no-obs && \
run q1_serial_noobs SECHS_PIPE_SERIAL=1 --play-quad 1 --no-obs && echo done
