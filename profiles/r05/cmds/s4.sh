#!/bin/bash
# state-bounded 16-lane kernel with the fused alpha_max trial: parity tests, then A/B against lib_var/r5s2
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5s4; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_xbounds.py tests/test_gpu_bounds.py tests/test_gpu_riccati.py -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r5s4/ab VARIANTS="r5s2 cur" CONFIGS="cfg2" REPS=3 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
