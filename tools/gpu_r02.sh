#!/bin/bash
# Round-2 GPU check: parity tests, smoke, cfg#2 / cfg#3 bench lines, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; tail -40 "$OUT/pytest_gpu.log"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -z "$SKIP_CFG3" ]; then
  timeout -k 10 300 python bench.py --config cfg3 --steps 5 --warmup 1 > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err" || { tail -20 "$OUT/bench_cfg3.err"; exit 1; }
  cat "$OUT/bench_cfg3.json"
fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$OUT/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
for f in $(find "$OUT/prof" -name "*kernel_stats.csv"); do cat "$f"; done
