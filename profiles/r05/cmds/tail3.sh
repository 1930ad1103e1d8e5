#!/bin/bash
# tail hand-over, wave rule (MMPC_TAIL_WAVE, default 8): tests, then cfg#3 / cfg#5 / exact with the rule off (0) and
# on (8), at the default tolerance and at 1e-5
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5tail3; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_riccati.py -v -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
for w in 0 8; do
  MMPC_TAIL_WAVE=$w OUT=$OUT/w$w VARIANTS="cur" CONFIGS="cfg3 cfg5" REPS=1 bash tools/gpu_ab.sh || exit 1
  MMPC_TAIL_WAVE=$w OUT=$OUT/w${w}_tol5 VARIANTS="cur" CONFIGS="cfg3 cfg5" REPS=1 BENCH_ARGS="--tol 1e-5" bash tools/gpu_ab.sh || exit 1
  MMPC_TAIL_WAVE=$w OUT=$OUT/w${w}_tol6 VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--tol 1e-6" bash tools/gpu_ab.sh || exit 1
  MMPC_TAIL_WAVE=$w OUT=$OUT/w${w}_ex VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--hessian exact" bash tools/gpu_ab.sh || exit 1
done
