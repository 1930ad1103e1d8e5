#!/bin/bash
# tail hand-over of control-bounded lane solves: tests, then exo |u| <= 2 / 0.5 at cfg#3 size against the build
# before it (lib_var/prevub), caps 3 / 5 beside the default 4
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ubtail; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_bounds.py tests/test_gpu_exact_lane.py -v -m gpu -x --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
for b in 2 0.5; do
  OUT=$OUT/ab$b VARIANTS="prevub cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--u-bound $b" bash tools/gpu_ab.sh || exit 1
  for c in 3 5; do
    MMPC_TAIL_CAP=$c OUT=$OUT/c${c}_$b VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--u-bound $b" bash tools/gpu_ab.sh || exit 1
  done
done
OUT=$OUT/cfg3 VARIANTS="prevub cur" CONFIGS="cfg3" REPS=1 bash tools/gpu_ab.sh || exit 1
