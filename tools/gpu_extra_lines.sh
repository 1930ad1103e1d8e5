#!/bin/bash
# Secondary bench lines of the current build: --strong at B = 4096, small batches, control / state bounds
set -o pipefail
OUT=gpurun_out/extra; mkdir -p $OUT
run() { n=$1; shift; timeout -k 10 200 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-sweep > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }; python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']), round(d['kernel_ms'],4), d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'], d['config'].get('hessian'))"; }
run strong4096 --strong --batch 4096 && run b512 --batch 512 && run b1024 --batch 1024 && run ub2 --u-bound 2 && run ub2gn --u-bound 2 --hessian gauss_newton && run ub2ex --u-bound 2 --hessian exact && run xb15 --x-bound 1.5 && run xb15exo --config cfg3 --x-bound 1.5 && run ubexo05 --config cfg3 --u-bound 0.5 && run cfg3tol5 --config cfg3 --tol 1e-5
