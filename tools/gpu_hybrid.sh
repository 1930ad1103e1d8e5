#!/bin/bash
# Co-scheduled solver: parity tests, bench of every cfg#2 solver, rocprof kernel trace of the hybrid solve.
set -o pipefail
OUT=${OUT:-gpurun_out/hybrid}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_riccati.py tests/test_gpu_parity.py tests/test_gpu_bounds.py -q -x > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -30; exit $rc; }
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; return 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag solves/s %.4g kernel_ms %.4f iters %.3f conv %d' % (d['value'], d['kernel_ms'], d['mean_sqp_iters'], d['converged']))"
}
run auto && run condensed --kkt condensed && run group --kkt group && run hybrid --kkt hybrid || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
for f in $(find "$OUT/prof" -name "*kernel_stats.csv"); do cat "$f"; done
