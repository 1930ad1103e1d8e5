#!/bin/bash
# GPU check of the bounded (projected GN-SQP) kernels and the unchanged unbounded paths.
set -o pipefail
OUT=${OUT:-gpurun_out/bounds}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_bounds.py tests/test_gpu_parity.py tests/test_gpu_riccati.py tests/test_gpu_host.py -q -x > "$OUT/pytest.log" 2>&1; rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" "$OUT/pytest.log" | head -40; exit $rc; }
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; return 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag solves/s %.4g kernel_ms %.4f iters %.3f conv %d' % (d['value'], d['kernel_ms'], d['mean_sqp_iters'], d['converged']))"
}
run cfg2 && run cfg3 --config cfg3
