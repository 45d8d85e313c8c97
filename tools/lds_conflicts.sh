#!/bin/bash
# LDS bank-conflict counters of the headline step's k_play (one pass)
#   gpurun -- bash tools/lds_conflicts.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lds_${1:-cur}
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-philox --no-mixed-league --no-dropin"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-include-regex "k_play" --output-format csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 1; }
python3 - $OUT/a/run_counter_collection.csv <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_play<4" in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
w = tot["SQ_WAVES"]
print({k: round(v / w, 1) for k, v in tot.items()}, "per wave")
PY
