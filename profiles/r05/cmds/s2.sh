#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5s2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_xbounds.py tests/test_gpu_bounds.py tests/test_gpu_parity.py tests/test_gpu_init.py -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r5s2/ab VARIANTS="r5s1 cur" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r5s2/ab_ub VARIANTS="r5s1 cur" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--u-bound 2" bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r5s2/ab_def VARIANTS="r5s1 cur" CONFIGS="cfg2" REPS=2 bash tools/gpu_ab.sh || exit 1
