#!/bin/bash
# rocprofv3 kernel-trace summary of the headline bench leg only (k_mt_prep + k_play).
#   gpurun -- bash tools/prof_play.sh <tag> [numpy|philox]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_${1:-cur}
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 30 --warmup 2 --no-cpu --no-mcs --no-puct --rng ${2:-numpy} ${3:-} > $OUT/bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 - $OUT/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
PY
cat $OUT/bench.json
