#!/bin/bash
# A/B of HIP runtime launch knobs on the headline step (config 2, numpy MT,
# two-stream pipeline): interleaved reps of the headline-only bench per
# variant, one JSON line each into gpurun_out/<tag>/env_ab.jsonl.
#   gpurun -- bash tools/env_ab.sh <tag> [reps]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-env_ab}
REPS=${2:-3}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
: > $OUT/env_ab.jsonl
ARGS="--steps 200 --warmup 5 --no-cpu --no-philox --no-mcs --no-puct --no-league --no-scalar"
for rep in $(seq 1 $REPS); do
  for v in base kernarg1 kernarg0 hwq8 hwq2; do
    case $v in
      base) E="" ;;
      kernarg1) E="HIP_FORCE_DEV_KERNARG=1" ;;
      kernarg0) E="HIP_FORCE_DEV_KERNARG=0" ;;
      hwq8) E="GPU_MAX_HW_QUEUES=8" ;;
      hwq2) E="GPU_MAX_HW_QUEUES=2" ;;
    esac
    line=$(env $E timeout -k 10 120 python bench.py $ARGS 2> $OUT/err_$v.log | tail -1) || { echo "FAIL $v"; tail -5 $OUT/err_$v.log; exit 1; }
    echo "{\"variant\": \"$v\", \"rep\": $rep, \"bench\": $line}" >> $OUT/env_ab.jsonl
    echo "$v rep$rep $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["roofline"]["kernel_ms"],4))')"
  done
done
