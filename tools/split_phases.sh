#!/bin/bash
# Phase split of the role-split k_play (play waves + producer waves) on the
# dev profiling library: philox (default split) and numpy mode 3.
#   gpurun -- bash tools/split_phases.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-phases}
mkdir -p $OUT
export SECHS_LIB=$R/rl-6-nimmt_amd/libsechs_devprof.so
timeout -k 10 120 python3 tools/phase_prof.py 65536 20 philox 1 > $OUT/philox_split.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
timeout -k 10 120 python3 tools/phase_prof.py 65536 20 philox 0 > $OUT/philox_plain.json 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
timeout -k 10 120 python3 tools/phase_prof.py 65536 20 numpy 3 > $OUT/numpy_split3.json 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
cat $OUT/*.json
