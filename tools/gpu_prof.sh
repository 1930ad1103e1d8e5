#!/bin/bash
# phase breakdown (diagnostic build) + rocprofv3 kernel-trace summary of the shipped build
set -o pipefail
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 300 python tools/phase_profile.py > "$OUT/phase.json" 2> "$OUT/phase.err" || { tail "$OUT/phase.err"; exit 1; }
cat "$OUT/phase.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/rp.log" 2>&1 || { tail -20 "$OUT/rp.log"; exit 1; }
tail -1 "$OUT/rp.log"
for f in $(find "$OUT/rp" -name "*kernel_stats.csv"); do cat "$f"; done
