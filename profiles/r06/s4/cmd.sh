# exact Hessian under state bounds (new kernels) + the state-bound / exact / tail suites; then the icache PMC passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s4; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_xbounds.py tests/test_gpu_exact_lane.py tests/test_gpu_tail.py -v -s -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "exact iterations" $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
bash profiles/r06/icache/cmd.sh || exit 1

timeout -k 10 120 tools/ubench/tail_rounds > $O/tail_rounds.txt 2>&1; cat $O/tail_rounds.txt
