#!/bin/bash
# INIT_ZERO + single-buffer results: GPU init/parity tests, cfg#2 bench (default) and with --init as_given, rocprof
set -o pipefail
OUT=${OUT:-gpurun_out/r02k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_init.py tests/test_gpu_parity.py tests/test_gpu_multi.py -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py > "$OUT/bench_cfg2.json" || exit 1
timeout -k 10 300 python bench.py --init as_given --no-cpu-baseline > "$OUT/bench_cfg2_as_given.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- python bench.py --no-cpu-baseline > "$OUT/prof_cfg2.json" || exit 1
for f in bench_cfg2 bench_cfg2_as_given; do python3 -c "import json,sys; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'], d['max_sqp_iters'], d['gathered_results_match'], d['converged'], d.get('cpu_baseline',{}).get('vs_gpu'))"; done
cat "$OUT/prof_cfg2/run_kernel_stats.csv" | cut -c1-160
echo rc_pytest=$rc
