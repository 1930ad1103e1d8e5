#!/bin/bash
# lane kernel: the targets load and the V write-back through LDS (coalesced rows) -- lane suites on the new build,
# then A/B against the same source with MMPC_LANE_LDS_ROWS=0 (lib_var/rows0)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rows; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_riccati.py tests/test_gpu_tail.py tests/test_gpu_exact_lane.py tests/test_gpu_cfg4.py tests/test_gpu_sx_models.py tests/test_gpu_parity.py tests/test_gpu_xbounds.py -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
OUT=$OUT/ab VARIANTS="rows0 cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
