#!/bin/bash
# A/B kernel variants: lib_var/<v>/libmmpc.so through MMPC_LIB_PATH, cfg#2 bench kernel time (and parity tests on
# the variants named in TEST_VARIANTS)
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/var}
mkdir -p "$OUT"
for v in ${VARIANTS:-a b}; do
  export MMPC_LIB_PATH=$PWD/lib_var/$v/libmmpc.so
  for rep in 1 2; do
    timeout -k 10 200 python bench.py ${BENCH_ARGS:-} --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench_$v.$rep.json" 2> "$OUT/bench_$v.err" || { tail -5 "$OUT/bench_$v.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$v.$rep.json')); print('$v', d['value'], d['ms_per_step'], d['kernel_ms'], d['mean_sqp_iters'], d['converged'])"
  done
done
for v in ${TEST_VARIANTS:-}; do
  export MMPC_LIB_PATH=$PWD/lib_var/$v/libmmpc.so
  timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_riccati.py} -q -m gpu -x --timeout 120 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1; rc=$?
  echo "tests $v rc=$rc"; tail -2 "$OUT/pytest_$v.log"
  [ $rc -le 1 ] || exit $rc
done
