#!/bin/bash
# Round-2 first GPU session: microbenchmarks, GPU tests on the current tree, bench (new timed region), rocprof.
set -o pipefail
OUT=gpurun_out/r02a
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench/f64_latency > "$OUT/ubench.txt" 2>&1 || { cat "$OUT/ubench.txt"; exit 1; }
cat "$OUT/ubench.txt"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
