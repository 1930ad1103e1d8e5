#!/bin/bash
# Full GPU check of the tree: all GPU tests, smoke, the three bench lines (cfg#2 headline, cfg#3, cfg#5) and the
# rocprofv3 kernel-trace summaries of cfg#2 and cfg#3.  Every GPU step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/full}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -3 "$OUT/smoke.log"
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['kernel_ms'], d['converged'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
done
for c in cfg2 cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_$c.log" 2>&1 || { tail -20 "$OUT/prof_$c.log"; exit 1; }
  for f in $(find "$OUT/prof_$c" -name "*kernel_stats.csv"); do cp "$f" "$OUT/rocprof_kernel_stats_$c.csv"; head -4 "$f"; done
done
echo done
