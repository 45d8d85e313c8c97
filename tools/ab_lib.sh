#!/bin/bash
# interleaved headline A/B: the product library vs another build (SECHS_LIB)
#   gpurun -- bash tools/ab_lib.sh <other.so> [reps]
set -o pipefail
OTHER=$1; REPS=${2:-3}
for rep in $(seq 1 $REPS); do
  for lib in product other; do
    if [ $lib = other ]; then export SECHS_LIB=$(pwd)/$OTHER; else unset SECHS_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu --no-mcs --no-puct --no-scalar --no-league --no-mixed-league --no-dropin --no-philox --steps 300 --warmup 20 > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.err || { tail -3 gpurun_out/ab_$lib.err; exit 1; }
    python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(r['value']/1e9,3), 'G ms', round(r['ms_per_step'],4), 'play', round(r['roofline']['kernel_ms']*1e3,1), 'ahead', round(r['roofline']['concurrent']['kernel_ms']*1e3,1))" gpurun_out/ab_$lib.json $lib
  done
done
