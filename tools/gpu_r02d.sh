#!/bin/bash
# Exact-Hessian SQP: all GPU tests (agreement logged), then cfg#2 bench (AUTO = exact) under a rocprof kernel trace,
# and the Gauss-Newton cfg#2 line for comparison.
set -o pipefail
OUT=${OUT:-gpurun_out/r02d}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_TEST_LOG="$PWD/$OUT/agreement.log" timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -25 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- python bench.py --no-cpu-baseline > "$OUT/bench_cfg2_exact.json" || exit 1
cat "$OUT/bench_cfg2_exact.json"
find "$OUT/prof_cfg2" -name "*kernel_stats.csv" -exec head -4 {} \;
timeout -k 10 300 python bench.py --hessian gauss_newton --no-cpu-baseline > "$OUT/bench_cfg2_gn.json" || exit 1
cat "$OUT/bench_cfg2_gn.json"
echo rc_pytest=$rc
