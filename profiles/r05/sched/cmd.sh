#!/bin/bash
# A/B of the AMDGPU scheduling strategy: max-ILP (lib_var/ilp), max-ILP without the high-RP reschedule stage
# (lib_var/nopost) against the shipped build; parity subset on each variant first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sched; mkdir -p $OUT
for v in ilp nopost; do
  MMPC_LIB_PATH=$PWD/lib_var/$v/libmmpc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_riccati.py tests/test_gpu_tail.py -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1; rc=$?; echo "$v tests rc=$rc"; tail -n 2 $OUT/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
OUT=$OUT/ab VARIANTS="cur ilp nopost" CONFIGS="cfg2 cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh
