#!/bin/bash
# headline A/B of the steady twist's grid (SECHS_TWIST_BLOCKS: 0 = a wave per game), interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_twb}
mkdir -p $O
cd $R
for rep in 1 2; do for n in 0 4096 2048 1024 512; do
  SECHS_TWIST_BLOCKS=$n timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 20 > $O/h_${n}_$rep.json 2> $O/h_${n}_$rep.err || { tail $O/h_${n}_$rep.err; exit 1; }
  python tools/ab_line.py head $O/h_${n}_$rep.json blocks=$n rep=$rep
done; done
