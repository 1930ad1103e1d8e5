#!/bin/bash
# A/B of library variants (tools/gpu_ab.sh) followed by the cfg#2-relevant parity tests on each variant library.
#   OUT=gpurun_out/x LIBS="current v1 v2" ARGSETS="..." REPS=3 PTESTS="tests/..." tools/gpu_ab_parity.sh
set -o pipefail
OUT=${OUT:-gpurun_out/abp}
mkdir -p "$OUT"
bash tools/gpu_ab.sh || exit $?
for lib in ${LIBS:-current}; do
  [ "$lib" = current ] && continue
  MMPC_LIB_PATH=$PWD/lib_var/$lib/libmmpc.so timeout -k 10 400 python -u -m pytest ${PTESTS:-tests/test_gpu_parity.py tests/test_gpu_riccati.py tests/test_gpu_bounds.py} -q -m gpu -x --timeout 120 --timeout-method thread > "$OUT/pytest_$lib.log" 2>&1; rc=$?
  echo "$lib: $(tail -1 $OUT/pytest_$lib.log)"
  [ $rc -eq 0 ] || { grep -E '^(FAILED|ERROR)' "$OUT/pytest_$lib.log" | head; exit $rc; }
done
