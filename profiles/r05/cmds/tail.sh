#!/bin/bash
# iteration-tail hand-over: its GPU tests and the lane-kernel suites, then A/B against the build before it
# (lib_var/r5s2) on cfg#3 (Gauss-Newton and exact Hessian) and cfg#5
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5tail; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_riccati.py tests/test_gpu_exact_lane.py tests/test_gpu_cfg4.py tests/test_gpu_sx_models.py tests/test_gpu_parity.py -v -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
OUT=gpurun_out/r5tail/ab VARIANTS="r5s2 cur" CONFIGS="cfg3" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r5tail/ab_ex VARIANTS="r5s2 cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--hessian exact" bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r5tail/ab5 VARIANTS="r5s2 cur" CONFIGS="cfg5" REPS=1 bash tools/gpu_ab.sh || exit 1
