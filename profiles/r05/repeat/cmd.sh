#!/bin/bash
# run-to-run spread of the driver's default bench line on one box (three back-to-back runs, CPU baseline skipped)
set -o pipefail
OUT=gpurun_out/repeat; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -5 $OUT/bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json')); s=d['secondary']
print($i, round(d['value']), round(d['kernel_ms'],4), round(s['cfg3']['value']), round(s['cfg3']['kernel_ms'],3), round(s['cfg5']['value']), round(s['cfg5']['kernel_ms'],3), d['roofline']['pmc_status'][:20])"
done
