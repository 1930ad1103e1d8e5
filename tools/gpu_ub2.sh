#!/bin/bash
# FP64 MFMA vs VALU for the lane kernel's stage products (tools/ubench/mfma_f64_stage.hip, built in the container),
# and the cfg#3 lane kernel's phase shares (diagnostic timing build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_ub2
mkdir -p $OUT
timeout -k 10 120 tools/ubench/mfma_f64_stage > $OUT/mfma_f64_stage.txt 2>&1; rc=$?
cat $OUT/mfma_f64_stage.txt
[ $rc -eq 0 ] || exit $rc
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 300 python tools/phase_profile.py --config cfg3 > $OUT/phase_cfg3.json 2> $OUT/phase_cfg3.err || { tail -5 $OUT/phase_cfg3.err; exit 1; }
python3 -c "
import json,sys
t=open('$OUT/phase_cfg3.json').read(); d=json.loads(t[t.index('{'):])
print(json.dumps(d.get('share'), indent=0)); print(d.get('mean_iters'), d.get('max_iters'))"
