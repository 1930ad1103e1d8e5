#!/bin/bash
# phase profile of the state-bounded lane kernel (exo, cfg#3 size, |qdot| <= 1.5)
set -o pipefail
OUT=gpurun_out/phase_xb; mkdir -p $OUT
export MMPC_LIB_PATH=$PWD/mahi-mpc_amd/lib/libmmpc_timing.so
timeout -k 10 300 python tools/phase_profile.py --config cfg3 --x-bound 1.5 > $OUT/phase_cfg3_xb15.json 2> $OUT/xb.err || { tail -5 $OUT/xb.err; exit 1; }

python3 -c "
import json
for n in ('cfg3_xb15',):
    d=json.load(open('$OUT/phase_'+n+'.json')); print(n, d['mean_iters'], d['max_iters'], round(d['cycles_per_wave']), {k: round(v) for k,v in d['per_phase_cycles_per_wave_iteration'].items()})
"
