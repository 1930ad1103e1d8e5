#!/bin/bash
# Round-2 (session 3) baseline: per-phase cycle shares of the cfg#2 group kernel and the cfg#3 lane kernel
# (diagnostic build), plus a rocprof kernel trace of the current cfg#3 lane kernel.
set -o pipefail
OUT=${OUT:-gpurun_out/r02c}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 180 python tools/phase_profile.py --kkt 3 > "$OUT/phase_cfg2_group.json" || exit 1
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 180 python tools/phase_profile.py --config cfg3 --kkt 2 > "$OUT/phase_cfg3_lane.json" || exit 1
cat "$OUT"/phase_*.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg3" -o run -- python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_cfg3.json" || exit 1
cat "$OUT/bench_cfg3.json"
find "$OUT/prof_cfg3" -name "*kernel_stats.csv" -exec cat {} \;
