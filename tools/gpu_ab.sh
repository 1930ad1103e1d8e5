#!/bin/bash
# Same-box A/B of library builds: lib_var/<v>/libmmpc.so (or "cur" = mahi-mpc_amd/lib/libmmpc.so) through
# MMPC_LIB_PATH, alternating the builds REPS times per config, each run a bench.py line without CPU baseline,
# secondaries or sweeps.  Optional parity suite first (TESTS, on the current build).
#   OUT=gpurun_out/ab VARIANTS="prev cur" CONFIGS="cfg2 cfg3 cfg5" REPS=2 TESTS="tests/" bash tools/gpu_ab.sh
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -q -m gpu -x --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CONFIGS:-cfg2}; do
  for rep in $(seq 1 ${REPS:-2}); do
    for v in ${VARIANTS:-prev cur}; do
      if [ "$v" = cur ]; then unset MMPC_LIB_PATH; else export MMPC_LIB_PATH=$PWD/lib_var/$v/libmmpc.so; fi
      f="$OUT/b_${v}_${cfg}_${rep}.json"
      timeout -k 10 200 python bench.py --config "$cfg" ${BENCH_ARGS:-} --steps 20 --warmup 3 --no-cpu-baseline \
        --no-secondary --no-sweep > "$f" 2> "$OUT/b_${v}.err" || { tail -5 "$OUT/b_${v}.err"; exit 1; }
      python3 -c "import json; d=json.load(open('$f')); print('$cfg $v', round(d['value']), round(d['kernel_ms'], 5), d['mean_sqp_iters'], d['max_sqp_iters'], d['converged'])"
    done
  done
done
