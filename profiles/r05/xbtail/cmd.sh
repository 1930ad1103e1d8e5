#!/bin/bash
# tail hand-over of state-bounded lane solves (wave rule): tests, then the exo |qdot| <= 1.5 cfg#3-size line and
# cfg#3 against the build before it (lib_var/prevxb)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/xbtail; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_xbounds.py tests/test_gpu_graph.py -v -m gpu -x --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
OUT=$OUT/ab VARIANTS="prevxb cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
OUT=$OUT/ab2 VARIANTS="prevxb cur" CONFIGS="cfg3" REPS=1 bash tools/gpu_ab.sh || exit 1
MMPC_TAIL_WAVE=16 OUT=$OUT/w16 VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
MMPC_TAIL_WAVE=4 OUT=$OUT/w4 VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
