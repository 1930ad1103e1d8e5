#!/bin/bash
# GPU half of tools/lane_variants.sh: the exo lane-kernel tests that exposed the round-3 wrong-result builds, run
# on every lib_var/<variant>_<flags>/libmmpc.so through MMPC_LIB_PATH (no -x: a variant may fail by design).
# Stops at the first run that ends in anything but pass/fail (timeout, abort, fault).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/lanevar}
mkdir -p "$OUT"
TESTS=${TESTS:-"tests/test_gpu_xbounds.py::test_exo_state_bounds_lane tests/test_gpu_xbounds.py::test_state_bounds_match_scipy_golden tests/test_gpu_riccati.py::test_exo_batch_vs_oracle tests/test_gpu_riccati.py::test_exo_solve_vs_scipy_golden tests/test_gpu_riccati.py::test_exo_cfg3_full_batch_properties"}
for d in ${VARIANTS:-$(ls -d lib_var/*/ | xargs -n1 basename)}; do
  [ -f "lib_var/$d/libmmpc.so" ] || { echo "$d: no library"; continue; }
  MMPC_LIB_PATH=$PWD/lib_var/$d/libmmpc.so timeout -k 10 300 python -u -m pytest $TESTS -q -m gpu --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$d.log" 2>&1; rc=$?
  echo "$d rc=$rc $(tail -1 "$OUT/pytest_$d.log")"
  grep -E "^FAILED" "$OUT/pytest_$d.log" | cut -c1-160
  [ $rc -le 1 ] || { echo "stopping: rc=$rc"; exit $rc; }
done
