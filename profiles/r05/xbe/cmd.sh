#!/bin/bash
# state-bounded lane kernel: barrier pieces loaded at the top of the backward stage (cur) vs at their uses (xbe0), step sweep at its uses (xbs0)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/xbe; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_xbounds.py -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="xbe0 xbs0 cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
