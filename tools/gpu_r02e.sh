#!/bin/bash
# GPU tests from test_gpu_xbounds onwards (the rest passed in r02d), agreement logged
set -o pipefail
OUT=${OUT:-gpurun_out/r02e}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_TEST_LOG="$PWD/$OUT/agreement.log" timeout -k 10 900 python -u -m pytest tests/test_gpu_xbounds.py tests/test_gpu_sx_models.py tests/test_gpu_riccati.py -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -25 "$OUT/pytest_gpu.log"
echo rc_pytest=$rc
