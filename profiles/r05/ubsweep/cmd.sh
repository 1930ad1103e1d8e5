#!/bin/bash
# cap / wave-rule sweep for control-bounded lane solves (exo |u| <= 2 and 0.5, cfg#3 size)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ubsweep; mkdir -p $OUT
for b in 2 0.5; do
  for cw in ${CWS:-0_0 4_8 5_4 6_4 5_2 4_2 6_2}; do
    c=${cw%_*}; w=${cw#*_}
    MMPC_TAIL_CAP=$c MMPC_TAIL_WAVE=$w OUT=$OUT/c${c}w${w}_$b VARIANTS="cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--u-bound $b" bash tools/gpu_ab.sh | sed "s/^/c$c w$w u$b /" || exit 1
  done
done
