#!/bin/bash
# full GPU tests; bench lines: cfg#2 exact (default), Gauss-Newton, bounded +-2 Nm; phase profiles of the three
set -o pipefail
OUT=${OUT:-gpurun_out/r03_check3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20; tail -2 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for args in "--no-secondary" "--no-secondary --hessian gauss_newton" "--no-secondary --u-bound 2"; do
  tag=$(echo "$args" | tr -d ' -')
  timeout -k 10 300 python bench.py $args --cpu-seconds 3 > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', round(d['value']), round(d['kernel_ms'],4), d['converged'], d['mean_sqp_iters'], d['max_sqp_iters'], d['config']['hessian'], (d.get('cpu_baseline') or {}).get('vs_gpu'))"
done
for args in "" "--hessian 1" "--u-bound 2"; do
  tag=$(echo "phase$args" | tr -d ' -')
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 $args > "$OUT/$tag.json" 2>&1 || { tail -20 "$OUT/$tag.json"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['hessian'], d['mean_iters'], d['max_iters'], round(d['cycles_per_wave']), {k: round(v) for k, v in d['per_phase_cycles_per_wave_iteration'].items()})"
done
