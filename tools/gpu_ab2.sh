#!/bin/bash
# lane kernel A/B: library at the start of the change (lib_var/r03a) vs current, cfg#3 and cfg#5 bench lines, after
# the lane-kernel parity tests and the smoke on the current library
set -o pipefail
OUT=${OUT:-gpurun_out/r03_ab2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_riccati.py tests/test_gpu_cfg4.py} -v -m gpu -x --timeout 300 --timeout-method thread -rA > "$OUT/pytest.log" 2>&1; rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest.log" | head -20; tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
for lib in ${LIBS:-r03a current}; do
  [ "$lib" = current ] && L=mahi-mpc_amd/lib/libmmpc.so || L=lib_var/$lib/libmmpc.so
  for c in cfg3 cfg5; do
    tag=${lib}_$c
    MMPC_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --config $c --no-secondary --no-cpu-baseline --no-sweep > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', round(d['value']), round(d['kernel_ms'],4), d['converged'], d['mean_sqp_iters'], d['max_sqp_iters'])"
  done
done
