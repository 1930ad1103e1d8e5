#!/bin/bash
# bounded (lane-distributed) group kernel: parity tests, smoke, bounded and unbounded cfg#2 bench lines; XB variant diag
set -o pipefail
OUT=${OUT:-gpurun_out/r03_check2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_parity.py tests/test_gpu_riccati.py tests/test_gpu_u0.py tests/test_gpu_multi.py tests/test_gpu_init.py -v -m gpu -x --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20; tail -2 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log" | grep smoke
for args in "--no-secondary" "--no-secondary --u-bound 2" "--no-secondary --u-bound 2 --kkt condensed"; do
  tag=$(echo "$args" | tr -d ' -')
  timeout -k 10 300 python bench.py $args --cpu-seconds 4 > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', round(d['value']), d['kernel_ms'], d['converged'], d['mean_sqp_iters'], d['max_sqp_iters'], d['config']['kkt_solver'], d['config']['hessian'], d.get('cpu_baseline',{}).get('vs_gpu'))"
done
MMPC_LIB_PATH=$PWD/lib_var/xbb_nosb/libmmpc.so timeout -k 10 200 python tools/xb_diag.py "$OUT/xb_nosb.npz" > "$OUT/xb_nosb.txt" 2>&1; head -9 "$OUT/xb_nosb.txt"
