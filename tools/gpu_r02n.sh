#!/bin/bash
# phase profiles of the current group (cfg#2) and lane (cfg#3) kernels, PMC passes of the cfg#2 kernel
set -o pipefail
OUT=${OUT:-gpurun_out/r02n}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 > "$OUT/phase_cfg2_group.json" || exit 1
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 180 python tools/phase_profile.py --config cfg3 > "$OUT/phase_cfg3_lane.json" || exit 1
OUT=$OUT/pmc_cfg2 KERNEL=sqp_group_kernel BENCH_ARGS="--config cfg2" SUMMARY_ARGS="--traffic-json profiles/traffic_latest.json --key cfg2:sqp_group_kernel<TwoLinkArm> --batch 4096 --horizon 30 --source profiles/r02/pmc_cfg2_group_exact_v2.json" bash tools/pmc.sh > "$OUT/pmc_cfg2.json" || exit 1
cat "$OUT/phase_cfg2_group.json" "$OUT/phase_cfg3_lane.json"
