#!/bin/bash
# lane kernel: workspace through global (not flat) pointers, exo coefficients through scalar loads
set -o pipefail
OUT=${OUT:-gpurun_out/r02p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_riccati.py tests/test_gpu_parity.py tests/test_gpu_bounds.py tests/test_gpu_xbounds.py tests/test_gpu_init.py -q -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py --config cfg3 --steps 5 --warmup 1 > "$OUT/bench_cfg3.json" || exit 1
python3 -c "import json,sys; d=json.load(open('$OUT/bench_cfg3.json')); print('cfg3', d['value'], d['ms_per_step'], d['kernel_ms'], d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'], d.get('cpu_baseline',{}).get('vs_gpu'))"
timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_cfg5.json" || exit 1
python3 -c "import json,sys; d=json.load(open('$OUT/bench_cfg5.json')); print('cfg5', d['value'], d['kernel_ms'], d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'])"
echo rc_pytest=$rc
