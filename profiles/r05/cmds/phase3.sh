#!/bin/bash
# phase profile of the lane kernel (cfg#3) on the tail hand-over build
set -o pipefail
OUT=gpurun_out/phase3; mkdir -p $OUT
export MMPC_LIB_PATH=$PWD/mahi-mpc_amd/lib/libmmpc_timing.so
timeout -k 10 200 python tools/phase_profile.py --config cfg3 > $OUT/phase_cfg3.json 2> $OUT/cfg3.err || { tail -5 $OUT/cfg3.err; exit 1; }
python3 -c "
import json
d=json.load(open('$OUT/phase_cfg3.json')); print(d['mean_iters'], d['max_iters'], round(d['cycles_per_wave']), {k: round(v,3) for k,v in d['share'].items()})
"
