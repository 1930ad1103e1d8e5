#!/bin/bash
# per-phase cycle shares of the exact-Hessian group kernel (cfg#2) and the current lane kernel (cfg#3)
set -o pipefail
OUT=${OUT:-gpurun_out/r02i}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 180 python tools/phase_profile.py --kkt 3 > "$OUT/phase_cfg2_group_exact.json" || exit 1
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 180 python tools/phase_profile.py --config cfg3 --kkt 2 > "$OUT/phase_cfg3_lane.json" || exit 1
cat "$OUT"/phase_*.json
