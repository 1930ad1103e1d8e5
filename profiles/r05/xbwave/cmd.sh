#!/bin/bash
# wave-rule threshold sweep for the state-bounded lane solve (exo |qdot| <= 1.5, cfg#3 size)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/xbwave; mkdir -p $OUT
for w in 0 1 2 3 4 6; do
  MMPC_TAIL_WAVE=$w OUT=$OUT/w$w VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
done
for w in 2 4; do
  MMPC_TAIL_WAVE=$w OUT=$OUT/r$w VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
done
