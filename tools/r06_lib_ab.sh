#!/bin/bash
# interleaved headline A/B of two library builds: A = $LIB_A, B = $LIB_B (default: libsechs_ab0.so vs libsechs.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_libab}
A=${LIB_A:-$R/rl-6-nimmt_amd/libsechs_ab0.so}
B=${LIB_B:-$R/rl-6-nimmt_amd/libsechs.so}
mkdir -p $O
cd $R
for rep in 1 2 3; do for v in A B; do
  L=$A; [ $v = B ] && L=$B
  SECHS_LIB=$L timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 20 > $O/h_${v}_$rep.json 2> $O/h_${v}_$rep.err || { tail $O/h_${v}_$rep.err; exit 1; }
  python tools/ab_line.py head $O/h_${v}_$rep.json lib=$v rep=$rep
done; done
