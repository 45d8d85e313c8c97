#!/bin/bash
# the driver's headline shape (--steps 20 --warmup 5), 1 vs 4 launches per call, interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_drv}
mkdir -p $O
cd $R
for rep in 1 2 3; do for n in 1 4; do
  timeout -k 10 200 python bench.py --only headline --steps 20 --warmup 5 --launches-per-call $n > $O/h_${n}_$rep.json 2> $O/h_${n}_$rep.err || { tail $O/h_${n}_$rep.err; exit 1; }
  python tools/ab_line.py head $O/h_${n}_$rep.json lpc=$n rep=$rep
done; done
