#!/bin/bash
# r06 decode-ahead iteration: env parity tests (decode-ahead on by default), then an
# interleaved headline A/B (SN_OPT_PIPE_DEC 1 vs 0) and a kernel trace of the new step
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06_dec}
SEL=${2:-"decode or pipelined or rollout_matches or mt_state or overrun or ring_options or interleave or bench_lanes"}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -v --timeout 240 --timeout-method thread -k "$SEL" > $OUT/pytest_env.log 2>&1
rc=$?; tail -4 $OUT/pytest_env.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for d in 1 0; do
    timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 20 --pipe-dec $d > $OUT/head_d${d}_$rep.json 2> $OUT/head_d${d}_$rep.err || { tail $OUT/head_d${d}_$rep.err; exit 1; }
    python tools/ab_line.py head $OUT/head_d${d}_$rep.json dec=$d rep=$rep
  done
done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- python3 $R/bench.py --only headline --steps 40 --warmup 8 > $OUT/kstats.log 2>&1 || { tail $OUT/kstats.log; exit 1; }
cd $R
head -6 $OUT/kstats/run_kernel_stats.csv
python3 tools/group_trace.py $OUT/kstats/run_kernel_trace.csv 4 > $OUT/groups.json && cat $OUT/groups.json
echo done
