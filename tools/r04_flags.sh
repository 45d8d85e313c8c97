#!/bin/bash
# r04: device-flag pipeline + fused PUCT MLP + seat-parallel PUCT step -- parity tests, then A/Bs
# (historical A/B: the SN_OPT_PIPE_FLAGS modes it selects were measured slower and removed from the
#  library -- DESIGN.md §4; SECHS_PIPE_FLAGS is ignored by the current build)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_flags}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_env.log 2>&1
rc=$?; tail -4 $OUT/tests_env.log; fatal $rc pytest_env
[ $rc -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_puct.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_puct.log 2>&1
rc=$?; tail -4 $OUT/tests_puct.log; fatal $rc pytest_puct
for rep in 1 2; do
  for f in 1 0; do
    SECHS_PIPE_FLAGS=$f timeout -k 10 200 python bench.py --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --no-philox > $OUT/head_f${f}_$rep.json 2> $OUT/head_f${f}_$rep.err
    rc=$?; fatal $rc head
    python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('flags',sys.argv[2],'rep',sys.argv[3],round(r['value']/1e9,3),'G ms',round(r['ms_per_step'],4),'k_play',round(r['roofline']['kernel_ms']*1e3,1),'ahead',round(r['roofline']['concurrent']['kernel_ms']*1e3,1))" $OUT/head_f${f}_$rep.json $f $rep
  done
done
for cfg in "1 1" "1 0" "0 1" "0 0"; do
  set -- $cfg
  SECHS_FUSED_MLP=$1 SECHS_PUCT_STEP_SEATS=$2 timeout -k 10 300 python bench.py --only puct > $OUT/puct_$1$2.json 2> $OUT/puct_$1$2.err
  rc=$?; fatal $rc puct
  python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['extra_config4_puct']; print('fused',sys.argv[2],'seats',sys.argv[3],round(r['value']/1e6,1),'M playout env-steps/s wall',round(r['wall_s'],3))" $OUT/puct_$1$2.json $1 $2
done
SECHS_MLP_LAYER1=seats timeout -k 10 300 python bench.py --only puct > $OUT/puct_seats.json 2> $OUT/puct_seats.err
rc=$?; fatal $rc puct_seats
python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['extra_config4_puct']; print('layer1 in kernel',round(r['value']/1e6,1),'M playout env-steps/s wall',round(r['wall_s'],3))" $OUT/puct_seats.json
cd /tmp && SECHS_MLP_LAYER1=seats timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_puct_seats -o run -- python3 $R/bench.py --only puct > $OUT/prof_puct_seats.log 2>&1
rc=$?; echo "rocprof seats rc=$rc"; fatal $rc rocprof_seats
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_puct -o run -- python3 $R/bench.py --only puct > $OUT/prof_puct.log 2>&1
rc=$?; echo "rocprof rc=$rc"; fatal $rc rocprof
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_env.py --deselect tests/test_gpu_puct.py > $OUT/tests_rest.log 2>&1
rc=$?; tail -4 $OUT/tests_rest.log; fatal $rc pytest_rest
timeout -k 10 400 python bench.py --only mixed > $OUT/mixed.json 2> $OUT/mixed.err
rc=$?; fatal $rc mixed
python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['extra_config5_run_py_league']; print('run.py league s/round',round(r['s_per_round'],3)); print(json.dumps(r['phases']))" $OUT/mixed.json
echo done
