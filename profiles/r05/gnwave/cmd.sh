#!/bin/bash
# wave-rule threshold for unbounded lane solves at loose tolerances (cfg#3, tol 1e-5 / 1e-6): 4 / 8 (default) / 16
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/gnwave; mkdir -p $OUT
for t in 1e-5 1e-6; do
  for w in 4 8 16; do
    MMPC_TAIL_WAVE=$w OUT=$OUT/w${w}_$t VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--tol $t" bash tools/gpu_ab.sh | sed "s/^/w$w tol$t /" || exit 1
  done
done
