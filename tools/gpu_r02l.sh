#!/bin/bash
# group-kernel peeling: parity / riccati / init GPU tests, cfg#2 bench
set -o pipefail
OUT=${OUT:-gpurun_out/r02l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_riccati.py tests/test_gpu_init.py tests/test_gpu_bounds.py -q -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_cfg2.json" || exit 1
python3 -c "import json; d=json.load(open('$OUT/bench_cfg2.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['max_sqp_iters'], d['converged'])"
echo rc_pytest=$rc
