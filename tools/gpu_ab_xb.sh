#!/bin/bash
# A/B of the exo state-bounded lane kernel at cfg#3 size (|qdot| <= 1.5): lib_var/base vs lib_var/xbb, after the
# x-bounds and Riccati parity tests on the in-tree build
set -o pipefail
OUT=gpurun_out/ab_xbb; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_xbounds.py tests/test_gpu_riccati.py -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_xb.log 2>&1 || { tail -5 $OUT/pytest_xb.log; exit 1; }
tail -1 $OUT/pytest_xb.log
for rep in 1 2; do for v in base xbb; do
  MMPC_LIB_PATH=$PWD/lib_var/$v/libmmpc.so timeout -k 10 300 python bench.py --config cfg3 --x-bound 1.5 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-sweep > $OUT/b_${v}_$rep.json 2> $OUT/b_$v.err || { tail -5 $OUT/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${v}_$rep.json')); print('$v', round(d['kernel_ms'],3), d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'])"
done; done
