#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ timing) for one kernel of the
# headline bench leg.   gpurun -- bash tools/pmc_kernel.sh <tag> <kernel-regex> [numpy|philox]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cur}; KRX=${2:-k_play}; MODE=${3:-numpy}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-mcs --no-puct --rng $MODE"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || { tail $OUT/write.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$KRX" --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || { tail $OUT/sq.log; exit 1; }
python3 - $OUT <<'PY'
import csv, sys, collections
out = sys.argv[1]
for sub in ("fetch", "write", "sq"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{out}/{sub}/run_counter_collection.csv")):
        agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    # counter values are per-dimension rows: sum per dispatch is what we want; report mean over rows*count
    for (k, c), v in sorted(agg.items()):
        print(f"{sub:5s} {k:40s} {c:22s} rows={len(v):4d} sum/dispatch~{sum(v)/max(1,len(set(range(len(v))))):.1f}")
PY
