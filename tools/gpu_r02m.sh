#!/bin/bash
# closed-form 2-link derivatives (two_link_fast.h): full GPU suite, cfg#2 bench, rocprof kernel stats
set -o pipefail
OUT=${OUT:-gpurun_out/r02m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py > "$OUT/bench_cfg2.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- python bench.py --no-cpu-baseline > "$OUT/prof_cfg2.json" || exit 1
python3 -c "import json,sys; d=json.load(open('$OUT/bench_cfg2.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['max_sqp_iters'], d['gathered_results_match'], d['converged'], d.get('cpu_baseline',{}).get('vs_gpu'))"
cut -c1-160 "$OUT/prof_cfg2/run_kernel_stats.csv"
echo rc_pytest=$rc
