#!/bin/bash
# End-of-session GPU evidence for the current library build: GPU tests, smoke, the driver's default bench command,
# its rocprofv3 kernel-trace summary, and before them the PMC passes of cfg#2 / cfg#3 / cfg#5 (tools/gpu_pmc_all.sh)
# keyed to the library's sha256.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/final}
mkdir -p "$OUT"
export TMPDIR=/tmp
sha256sum mahi-mpc_amd/lib/libmmpc.so > "$OUT/lib_sha256.txt"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  tail -3 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || { grep -E 'FAILED|Error' "$OUT/pytest_gpu.log" | head; echo "pytest gpu rc=$rc: stopping"; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -4 "$OUT/smoke.log"
fi
# PMC first, its summary copied into this tree's profiles/, so the default bench line below attaches the counters of
# this same build (copy $OUT/pmc/traffic_latest.json back into profiles/ after the call)
if [ -z "$SKIP_PMC" ]; then
  OUT="$OUT/pmc" bash tools/gpu_pmc_all.sh || exit 1
  cp "$OUT/pmc/traffic_latest.json" profiles/traffic_latest.json
fi
[ -n "$SKIP_BENCH" ] && { echo "pmc done (SKIP_BENCH)"; exit 0; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/prof_default.json" 2> "$OUT/prof_default.err" || { tail -20 "$OUT/prof_default.err"; exit 1; }
for f in $(find "$OUT/prof_default" -name "*kernel_stats.csv"); do cp "$f" "$OUT/rocprof_kernel_stats_default.csv"; head -5 "$f"; done
echo done
