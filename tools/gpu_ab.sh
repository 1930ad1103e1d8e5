#!/bin/bash
# Generic GPU A/B of library builds: the listed GPU tests on the current library (and the smoke), then bench lines
# for every (library, argument set) pair, REPS times each in alternating order (box-to-box spread is ~2 %, so
# builds are only compared within one call).
#   OUT=gpurun_out/x LIBS="base current" ARGSETS="--no-secondary;--u-bound 2 --no-secondary" TESTS="tests/..." tools/gpu_ab.sh
# lib names other than "current" are lib_var/<name>/libmmpc.so (built in the container, travel with the tree).
set -o pipefail
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v -m gpu -x --timeout 300 --timeout-method thread -rA > "$OUT/pytest.log" 2>&1; rc=$?
  grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; tail -2 "$OUT/pytest.log"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${SMOKE:-}" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  cat "$OUT/smoke.log"
fi
IFS=';' read -r -a SETS <<< "${ARGSETS:---no-secondary}"
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-current}; do
    [ "$lib" = current ] && L=mahi-mpc_amd/lib/libmmpc.so || L=lib_var/$lib/libmmpc.so
    for i in "${!SETS[@]}"; do
      args="${SETS[$i]}"
      tag=${lib}_a${i}_r$rep
      MMPC_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --no-cpu-baseline $args > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', '$args', round(d['value']), round(d['kernel_ms'],4), d['converged'], d['mean_sqp_iters'], d['max_sqp_iters'])"
    done
  done
done
