#!/bin/bash
# Riccati-path GPU session: its parity tests, then the full GPU suite, then a cfg#3 timing.
set -o pipefail
OUT=${OUT:-gpurun_out/ric}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_riccati.py -q -x > "$OUT/pytest_riccati.log" 2>&1; rc=$?
tail -15 "$OUT/pytest_riccati.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest_riccati.log" | head -30; exit $rc; }
timeout -k 10 600 python -m pytest tests -q -m gpu > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
if [ -f bench.py ] && grep -q -- "--config" bench.py; then
  timeout -k 10 300 python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err" || { tail -20 "$OUT/bench_cfg3.err"; exit 1; }
  cat "$OUT/bench_cfg3.json"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof3" -o run -- python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof3.log" 2>&1 || { tail -20 "$OUT/prof3.log"; exit 1; }
for f in $(find "$OUT/prof3" -name "*kernel_stats.csv"); do cat "$f"; done
