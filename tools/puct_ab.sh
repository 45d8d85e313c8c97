#!/bin/bash
# PUCT-side change on one GPU box: the PUCT / league / ACER GPU tests, then an
# interleaved A/B of the config-4 legs (and the run.py league) against an older build.
#   gpurun -- bash tools/puct_ab.sh <tag> <old.so> [reps] [legs]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; OLD=$2; REPS=${3:-2}; LEGS=${4:-puct}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_puct.py tests/test_gpu_league.py tests/test_gpu_acer.py tests/test_gpu_reinforce.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in $(seq 1 $REPS); do
  for v in new old; do
    unset SECHS_LIB
    [ $v = old ] && export SECHS_LIB=$R/$OLD
    timeout -k 10 400 python bench.py --only $LEGS > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -3 $OUT/ab_$v.err; exit 1; }
    python - $OUT/ab_$v.json $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [sys.argv[2]]
for k, v in r.items():
    if k.startswith("extra") and isinstance(v, dict):
        out.append(f"{k[6:]}={v.get('value', 0):.4g}")
        if "s_per_round" in v: out.append(f"s_per_round={v['s_per_round']:.3f}")
print(" ".join(out))
PY
  done
done
unset SECHS_LIB
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --only puct > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; [ $rc -ne 0 ] && { echo "prof rc=$rc"; tail -3 $OUT/prof_bench.err; exit $rc; }
head -12 $OUT/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
echo done
