#!/bin/bash
# control-bounded 16-lane kernel: Riccati sweep one stage per trip (fewer spills) vs stage pairs (lib_var/bpairs);
# state-bounded kernel one stage per trip (lib_var/xb1) vs pairs (cur); bounds suites on cur and xb1 first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bpass; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_xbounds.py tests/test_gpu_exact_lane.py -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
MMPC_LIB_PATH=$PWD/lib_var/xb1/libmmpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_xbounds.py -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest_xb1.log 2>&1; rc=$?; tail -n 2 $OUT/pytest_xb1.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/ub2 VARIANTS="bpairs cur" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--u-bound 2" bash tools/gpu_ab.sh || exit 1
OUT=$OUT/ub2ex VARIANTS="bpairs cur" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--u-bound 2 --hessian exact" bash tools/gpu_ab.sh || exit 1
OUT=$OUT/xb15 VARIANTS="cur xb1" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
