#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== rocminfo gfx" && (rocminfo 2>/dev/null | grep -m1 -o "gfx9[0-9a-z]*" || true)
timeout -k 10 900 python -m pytest tests -q -m gpu > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -30 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*stats*" | head
for f in $(find "$OUT/prof" -name "*kernel_stats.csv"); do cat "$f"; done
