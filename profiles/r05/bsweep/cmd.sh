#!/bin/bash
set -o pipefail
OUT=gpurun_out/bsweep; mkdir -p $OUT
for b in 512 1024 1536 2048 2560 3072 3584 4096; do
  timeout -k 10 120 python bench.py --batch $b --steps 30 --warmup 3 --no-cpu-baseline --no-secondary --no-sweep > $OUT/b$b.json 2> $OUT/b$b.err || { tail -5 $OUT/b$b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$b.json')); print($b, round(d['kernel_ms'],4), d['mean_sqp_iters'], d['max_sqp_iters'])"
done
