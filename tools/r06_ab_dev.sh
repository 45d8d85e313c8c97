#!/bin/bash
# dev-library A/B of the decode-ahead headline (N = 4 build): parity probe, phase split, interleaved bench
export SECHS_LIB=$PWD/rl-6-nimmt_amd/libsechs_dev.so
O=gpurun_out/${1:-r06_devab}
mkdir -p $O
SECHS_PIPE_DEC=1 timeout -k 10 100 python tools/dec_debug.py 4096 || exit 1
SECHS_PIPE_DEC=1 SECHS_LIB=$PWD/rl-6-nimmt_amd/libsechs_devprof.so timeout -k 10 200 python tools/phase_prof.py 65536 40 numpy > $O/phase_dec.json || exit 1
for rep in 1 2; do for d in 1 0; do
timeout -k 10 200 python bench.py --only headline --steps 200 --warmup 20 --pipe-dec $d > $O/h_${d}_$rep.json 2> $O/h_${d}_$rep.err || { tail $O/h_${d}_$rep.err; exit 1; }
python tools/ab_line.py head $O/h_${d}_$rep.json dec=$d rep=$rep
done; done
python3 -c "
import json; d=json.load(open('$O/phase_dec.json')); p=d['producer']
print('play', d['cycles_per_wave_launch'], 'decoder', p['cycles_per_wave_launch'], {k: v['cycles_per_wave'] for k, v in p.items() if isinstance(v, dict) and v['cycles_per_wave']})"
