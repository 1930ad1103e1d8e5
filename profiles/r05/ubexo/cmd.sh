#!/bin/bash
set -o pipefail
OUT=gpurun_out/ubexo; mkdir -p $OUT
for b in 2 0.5 0.2; do
timeout -k 10 200 python bench.py --config cfg3 --u-bound $b --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --no-sweep > $OUT/ub$b.json 2> $OUT/ub$b.err || { tail -5 $OUT/ub$b.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/ub$b.json')); print('$b', round(d['kernel_ms'],3), d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'])"
done
