#!/bin/bash
# control-bounded hand-over with the shipped policy (wave rule 4, no cap): tests, exo |u| <= 2 / 0.5 against the
# build without it (lib_var/prevub), cfg#2 +-2 Nm (16-lane kernel, unaffected)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ubfinal; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_bounds.py tests/test_gpu_xbounds.py -q -m gpu -x --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
for b in 2 0.5; do
  OUT=$OUT/ab$b VARIANTS="prevub cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--u-bound $b" bash tools/gpu_ab.sh || exit 1
done
