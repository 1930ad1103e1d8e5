#!/bin/bash
# rerun of the GPU tests after rebuilding the generated-model libraries; cfg#2 bench with the exact-Hessian CPU baseline
set -o pipefail
OUT=${OUT:-gpurun_out/r02h}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_TEST_LOG="$PWD/$OUT/agreement.log" timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$OUT/pytest_gpu.log"
grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py > "$OUT/bench_cfg2.json" || exit 1
cat "$OUT/bench_cfg2.json"
echo rc_pytest=$rc
