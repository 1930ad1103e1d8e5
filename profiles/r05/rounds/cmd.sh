#!/bin/bash
# resume slots (rounds of resume workgroups) for the bounded exo solves at cfg#3 size: 4 (default) vs 8 / 16
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/rounds; mkdir -p $OUT
for a in "--x-bound 1.5" "--u-bound 0.5"; do
  for r in 4 8 16; do
    MMPC_TAIL_ROUNDS=$r OUT=$OUT/r$r VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="$a" bash tools/gpu_ab.sh | sed "s/^/r$r $a /" || exit 1
  done
done
