#!/bin/bash
# state-bounded 16-lane kernel: the Riccati sweep's barrier pieces loaded with the stage operands (cur) vs at their
# uses (lib_var/gxb_prev)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/gxb; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_xbounds.py -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="gxb_prev cur" CONFIGS="cfg2" REPS=3 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
