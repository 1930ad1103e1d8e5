set -o pipefail
mkdir -p gpurun_out/lazy3
timeout -k 10 300 python -u -m pytest tests/test_gpu_lazy_steps.py -v -s -m gpu --timeout 200 --timeout-method thread > gpurun_out/lazy3/pytest.log 2>&1; rc=$?
grep -E "regenerated|passed|failed|Error|assert" gpurun_out/lazy3/pytest.log | head; exit $rc
