#!/bin/bash
# A/B: bounded and state-bounded cfg#2 on the one-lane sweeps (library at the start of round 3) vs the lane-distributed
# sweeps; and the cfg#2 batch sweep (per-GPU B for strong scaling: 512 .. 16384) on the current library
set -o pipefail
OUT=${OUT:-gpurun_out/r03_ab1}
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in prev_r2 current; do
  [ "$lib" = current ] && L=mahi-mpc_amd/lib/libmmpc.so || L=lib_var/$lib/libmmpc.so
  for args in "--u-bound 2" "--x-bound 1.5"; do
    tag=$lib$(echo "$args" | tr -d ' -.')
    MMPC_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline $args > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', round(d['value']), round(d['kernel_ms'],4), d['converged'], d['mean_sqp_iters'], d['max_sqp_iters'])"
  done
done
for B in 512 1024 2048 4096 8192 16384; do
  timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --batch $B > "$OUT/bench_B$B.json" 2> "$OUT/bench_B$B.err" || { tail -20 "$OUT/bench_B$B.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_B$B.json')); print('B=$B', round(d['value']), round(d['kernel_ms'],4), round(d['ms_per_step'],4), d['config']['kkt_solver'], d['mean_sqp_iters'], d['max_sqp_iters'])"
done
