#!/bin/bash
set -o pipefail
OUT=${OUT:-gpurun_out/cfg5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_riccati.py -q -x > "$OUT/pytest_riccati.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_riccati.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest_riccati.log" | head -30; exit $rc; }
timeout -k 10 600 python tools/cfg5_sweep.py > "$OUT/cfg5_sweep.json" 2> "$OUT/cfg5.err" || { tail -20 "$OUT/cfg5.err"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/cfg5_sweep.json')); print('ref', d['reference'])
for r in d['sweep']: print(r['factor'], r['tol_grad'], 'conv %.2f%%' % r['converged_pct'], 'iters %.2f/%d' % (r['mean_iters'], r['max_iters']), 'ms %.2f' % r['kernel_ms'], 'relV %.2e' % r['max_rel_V_vs_fp64'])"
timeout -k 10 300 python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err" || { tail -20 "$OUT/bench_cfg3.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_cfg3.json')); print('cfg3 solves/s %.4g kernel_ms %.3f frac %.4f iters %.3f' % (d['value'], d['kernel_ms'], d['roofline']['frac'], d['mean_sqp_iters']))"
