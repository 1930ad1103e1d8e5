#!/bin/bash
# quick cfg#3 / cfg#5 kernel-time check (lane kernel iterations)
set -o pipefail
OUT=${OUT:-gpurun_out/cfg3q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_riccati.py -q -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -2 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
for c in cfg3 cfg5; do
timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_$c.json" || exit 1
python3 -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['kernel_ms'], d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'])"
done
