#!/bin/bash
# primal-dual release rule in the lane kernel's projected SQP: bounded / tail / lane suites, then exo |u| <= 2 / 0.5
# at cfg#3 size against the hold-only build (lib_var/prevrel)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rel; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_tail.py tests/test_gpu_exact_lane.py tests/test_gpu_riccati.py tests/test_gpu_parity.py -q -m gpu -x --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
for b in 2 0.5; do
  OUT=$OUT/ab$b VARIANTS="prevrel cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--u-bound $b" bash tools/gpu_ab.sh || exit 1
done
