#!/bin/bash
# headline A/B of the host's per-call cost: 1 vs 4 launches per sn_rollout call in the timed loop, interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_lpc}
mkdir -p $O
cd $R
for rep in 1 2 3; do for n in 1 4; do
  timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 20 --launches-per-call $n > $O/h_${n}_$rep.json 2> $O/h_${n}_$rep.err || { tail $O/h_${n}_$rep.err; exit 1; }
  python tools/ab_line.py head $O/h_${n}_$rep.json lpc=$n rep=$rep
  python -c "import json; print('  enqueue ms/step', round(json.load(open('$O/h_${n}_$rep.json'))['host_enqueue_ms_per_step'], 4))"
done; done
