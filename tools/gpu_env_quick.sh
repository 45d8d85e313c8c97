#!/bin/bash
# GPU env parity tests (optionally -k) + the headline bench leg only.
#   gpurun -- bash tools/gpu_env_quick.sh <tag> [pytest -k expr] [test file]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-envq}
mkdir -p $OUT
K=${2:-}
F=${3:-tests/test_gpu_env.py}
timeout -k 10 600 python -u -m pytest $F -m gpu -x -v --timeout 240 --timeout-method thread ${K:+-k "$K"} > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
grep -E "passed|failed" $OUT/gpu_tests.log | tail -3
timeout -k 10 200 python bench.py --steps 50 --warmup 3 --no-cpu --no-mcs --no-puct > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('value %.3e ms/step %.4f k_play %.4f ahead %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['concurrent']['kernel_ms'] if r.get('concurrent') else None))"
