#!/bin/bash
# Iteration loop on the GPU: full GPU test suite, bench line, per-phase cycle profile of the group kernel.
# usage: tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; grep -E "FAIL|Error|assert" "$OUT/pytest_gpu.log" | head -30; tail -60 "$OUT/pytest_gpu.log" | head -80; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 > "$OUT/phase.txt" 2>&1 || { tail -20 "$OUT/phase.txt"; exit 1; }
cat "$OUT/phase.txt"
