#!/bin/bash
# phase profiles of the state-bounded 16-lane kernel and the cfg#3 lane kernel (timing build), then the A/B of the
# column-wise K store (cur) against the build before it (lib_var/r5s2) on cfg#3 / cfg#5
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5s3; mkdir -p $OUT
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --x-bound 1.5 > $OUT/phase_cfg2_xb15.json || exit 1
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 > $OUT/phase_cfg2.json || exit 1
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 200 python tools/phase_profile.py --config cfg3 > $OUT/phase_cfg3.json || exit 1
python3 -c "
import json
for f in ['phase_cfg2_xb15','phase_cfg2','phase_cfg3']:
    d=json.load(open('$OUT/'+f+'.json')); print(f, d['mean_iters'], d['max_iters'], {k: round(v,3) for k,v in d['share'].items()})"
OUT=gpurun_out/r5s3/ab VARIANTS="r5s2 cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
