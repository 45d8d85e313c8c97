#!/bin/bash
# r04: run.py league leg with the ACER update's decider chunk at 4096 / 16384 / 65536 (A/B)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_acer}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
for c in 16384 4096 65536; do
  SECHS_ACER_DECIDER_CHUNK=$c timeout -k 10 400 python bench.py --only mixed > $OUT/mixed_$c.json 2> $OUT/mixed_$c.err
  rc=$?; fatal $rc mixed
  echo "decider_chunk $c"; python tools/ab_line.py mixed $OUT/mixed_$c.json
done
echo done
