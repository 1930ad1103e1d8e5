#!/bin/bash
# GPU session: all GPU tests (incl. the SX-generated model libraries), then a short bench.
set -o pipefail
OUT=${OUT:-gpurun_out/sx}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -30 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
