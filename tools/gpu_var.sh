#!/bin/bash
# cfg#3 kernel time of compile-time variants of the lane kernel (mahi-mpc_amd/lib/var_*.so)
set -o pipefail
OUT=${OUT:-gpurun_out/var}
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in mahi-mpc_amd/lib/var_*.so; do
  n=$(basename $lib .so)
  MMPC_LIB_PATH=$lib timeout -k 10 120 python bench.py --config ${CFG:-cfg3} --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$n.json" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['kernel_ms'], d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'])"
done
