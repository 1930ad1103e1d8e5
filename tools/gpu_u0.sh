#!/bin/bash
# u_0* output / host-mapped results: the new GPU tests, then the cfg#2 bench line and its rocprof kernel trace
set -o pipefail
OUT=${OUT:-gpurun_out/u0}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_u0.py tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" || { tail -20 "$OUT/bench_cfg2.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_cfg2.json')); print('cfg2', d['value'], d['ms_per_step'], d['kernel_ms'], d['converged'], d['gathered_results_match'], d['roofline']['frac'], d['roofline']['traffic'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_cfg2.log" 2>&1 || { tail -20 "$OUT/prof_cfg2.log"; exit 1; }
for f in $(find "$OUT/prof_cfg2" -name "*kernel_stats.csv"); do cp "$f" "$OUT/rocprof_kernel_stats_cfg2.csv"; cut -c1-200 "$f"; done
