#!/bin/bash
# lane-distributed interior-point (XB) and bounded group kernels: parity tests and bench lines
set -o pipefail
OUT=${OUT:-gpurun_out/r03_check4}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_xbounds.py tests/test_gpu_bounds.py tests/test_gpu_parity.py tests/test_gpu_riccati.py tests/test_gpu_init.py tests/test_gpu_host.py -v -m gpu -x --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20; tail -2 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for args in "--no-secondary" "--no-secondary --u-bound 2" "--no-secondary --x-bound 1.5" "--no-secondary --x-bound 1.5 --u-bound 4"; do
  tag=$(echo "$args" | tr -d ' -.')
  timeout -k 10 300 python bench.py $args --cpu-seconds 3 > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', round(d['value']), round(d['kernel_ms'],4), d['converged'], d['mean_sqp_iters'], d['max_sqp_iters'], d['config']['hessian'], (d.get('cpu_baseline') or {}).get('vs_gpu'))"
done
