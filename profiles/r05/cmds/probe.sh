#!/bin/bash
# per-iteration latency of the exo on the 16-lane kernel (N = 24, small batches) vs the lane kernel
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5probe; mkdir -p $OUT
run() { n=$1; shift; timeout -k 10 200 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --no-sweep > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }; python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['kernel_ms'],4), d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'], d['config']['kkt_solver'])"; }
run g24_256 --config cfg3 --horizon 24 --batch 256 --kkt group && run l24_256 --config cfg3 --horizon 24 --batch 256 --kkt riccati && \
run g24_1024 --config cfg3 --horizon 24 --batch 1024 --kkt group && run l50_256 --config cfg3 --horizon 50 --batch 256 --kkt riccati && \
run l50_64 --config cfg3 --horizon 50 --batch 64 --kkt riccati && run g12_256 --config cfg3 --horizon 12 --batch 256 --kkt group
