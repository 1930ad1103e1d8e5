#!/bin/bash
# tail hand-over, second pass: fp32-factor solves hand over to the fp64 16-lane resume launch, and four rounds of
# resume slots; tests, cfg#5 A/B against the pre-hand-over build, exact-Hessian cap 4 vs 5 on the current build
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5tail2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_riccati.py tests/test_gpu_exact_lane.py -v -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
OUT=gpurun_out/r5tail2/ab5 VARIANTS="r5s2 cur" CONFIGS="cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r5tail2/ex5 VARIANTS="cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--hessian exact" bash tools/gpu_ab.sh || exit 1
MMPC_TAIL_CAP=4 OUT=gpurun_out/r5tail2/ex4 VARIANTS="cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--hessian exact" bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r5tail2/gn VARIANTS="cur" CONFIGS="cfg3" REPS=1 bash tools/gpu_ab.sh || exit 1
MMPC_TAIL_CAP=3 MMPC_TAIL_ROUNDS=40 OUT=gpurun_out/r5tail2/gn3 VARIANTS="cur" CONFIGS="cfg3" REPS=1 bash tools/gpu_ab.sh || exit 1
MMPC_TAIL_CAP=4 MMPC_TAIL_ROUNDS=8 OUT=gpurun_out/r5tail2/ex4r8 VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--hessian exact" bash tools/gpu_ab.sh || exit 1
MMPC_TAIL_CAP=3 MMPC_TAIL_ROUNDS=40 OUT=gpurun_out/r5tail2/gn3f VARIANTS="cur" CONFIGS="cfg5" REPS=1 bash tools/gpu_ab.sh || exit 1
