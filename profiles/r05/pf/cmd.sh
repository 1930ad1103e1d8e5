#!/bin/bash
# lane step sweep: target/defect of the next stage prefetched and pinned (cur) vs loaded at use (lib_var/pf0)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pf; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_riccati.py tests/test_gpu_tail.py -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ab VARIANTS="pf0 cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
