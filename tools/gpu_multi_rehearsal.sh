#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: two gloo ranks sharing device 0 (test hooks), then the N = 1 line
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/multi}
mkdir -p "$OUT"
MMPC_BENCH_SAME_DEVICE=1 MMPC_BENCH_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || { tail -30 "$OUT/bench_n2.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_n2.json')); print('n2', d['n_gpus'], d['config']['global_batch'], d['value'], d['ms_per_step'], d['converged'], d['gathered_results_match'])"
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err" || { tail -30 "$OUT/bench_n1.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_n1.json')); print('n1', d['n_gpus'], d['value'], d['ms_per_step'], d['kernel_ms'], d['converged'], d['gathered_results_match'], d['roofline']['traffic'])"
