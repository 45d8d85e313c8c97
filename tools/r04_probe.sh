#!/bin/bash
# r04 GPU probe: cross-queue hand-off microbenchmark, new GPU tests, the
# `bench.py --gpus 2` path on the one-GPU box (RCCL, then the gloo rehearsal).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04_probe}
mkdir -p $OUT
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit $1; }; return 0; }
timeout -k 10 120 ./tools/queue_gap 200 62 > $OUT/queue_gap.jsonl 2>&1; rc=$?; cat $OUT/queue_gap.jsonl; fatal $rc queue_gap
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rccl or evolve or every_slot or sharding_invariance or reinforce_agent" > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; fatal $rc pytest
SECHS_BENCH_SHARED_GPU=1 timeout -k 10 120 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-mixed-league > $OUT/gpus2_rccl.json 2> $OUT/gpus2_rccl.err
rc=$?; echo "gpus2 rccl rc=$rc"; grep -v amdgpu.ids $OUT/gpus2_rccl.err | tail -c 1200; fatal $rc gpus2_rccl
SECHS_BENCH_SHARED_GPU=1 SECHS_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --mixed-slots 1024 --mixed-mc-max 20 > $OUT/gpus2_gloo.json 2> $OUT/gpus2_gloo.err
rc=$?; echo "gpus2 gloo rc=$rc"; tail -c 600 $OUT/gpus2_gloo.err; cut -c1-400 $OUT/gpus2_gloo.json; fatal $rc gpus2_gloo
echo done
