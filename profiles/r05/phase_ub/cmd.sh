#!/bin/bash
# phase profiles of the control-bounded 16-lane kernel (cfg#2 shape, |u| <= 2, Gauss-Newton) against the unbounded
# Gauss-Newton kernel
set -o pipefail
OUT=gpurun_out/phase_ub; mkdir -p $OUT
export MMPC_LIB_PATH=$PWD/mahi-mpc_amd/lib/libmmpc_timing.so
timeout -k 10 200 python tools/phase_profile.py --config cfg2 --u-bound 2 > $OUT/phase_cfg2_ub2.json 2> $OUT/ub2.err || { tail -5 $OUT/ub2.err; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --config cfg2 --hessian 1 > $OUT/phase_cfg2_gn.json 2> $OUT/gn.err || { tail -5 $OUT/gn.err; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --config cfg2 --u-bound 2 --hessian 2 > $OUT/phase_cfg2_ub2ex.json 2> $OUT/ub2ex.err || { tail -5 $OUT/ub2ex.err; exit 1; }
python3 -c "
import json
for n in ('ub2','gn','ub2ex'):
    d=json.load(open('$OUT/phase_cfg2_'+n+'.json')); print(n, d['mean_iters'], d['max_iters'], round(d['cycles_per_wave']), {k: round(v) for k,v in d['per_phase_cycles_per_wave_iteration'].items()})
"
