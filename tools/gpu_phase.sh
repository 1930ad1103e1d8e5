#!/bin/bash
# per-phase cycle shares of the cfg#2 group kernel (diagnostic timing build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/phase2
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 > gpurun_out/phase2/cfg2_group.json || exit 1
cat gpurun_out/phase2/cfg2_group.json
