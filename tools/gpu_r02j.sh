#!/bin/bash
# first-iteration filter acceptance: all GPU tests, cfg#2 / cfg#3 bench lines, cfg#2 rocprof kernel stats
set -o pipefail
OUT=${OUT:-gpurun_out/r02j}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_TEST_LOG="$PWD/$OUT/agreement.log" timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$OUT/pytest_gpu.log"
grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py > "$OUT/bench_cfg2.json" || exit 1
timeout -k 10 300 python bench.py --config cfg3 --steps 5 --warmup 1 > "$OUT/bench_cfg3.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- python bench.py --no-cpu-baseline > "$OUT/prof_cfg2.json" || exit 1
for f in bench_cfg2 bench_cfg3; do python3 -c "import json,sys; d=json.load(open('$OUT/$f.json')); c=d.get('cpu_baseline',{}); print('$f', d['value'], d['kernel_ms'], d['mean_sqp_iters'], d['max_sqp_iters'], c.get('value'), c.get('vs_gpu'))"; done
head -2 "$OUT/prof_cfg2/run_kernel_stats.csv"
echo rc_pytest=$rc
