#!/bin/bash
# Lane Riccati kernel: W in LDS + fused alpha=1 trial.  Riccati/bounds/xbounds GPU tests, cfg#3 bench (+ rocprof
# stats), cfg#3 PMC traffic pass.
set -o pipefail
OUT=${OUT:-gpurun_out/r02f}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_TEST_LOG="$PWD/$OUT/agreement.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_riccati.py tests/test_gpu_bounds.py tests/test_gpu_xbounds.py tests/test_gpu_sx_models.py -q -m gpu -x --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_cfg3.json" || exit 1
cat "$OUT/bench_cfg3.json"
head -3 "$OUT/prof_cfg3/run_kernel_stats.csv"
mkdir -p "$OUT/pmc3"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc3/fetch" -o run -- python3 bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc3/fetch.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc3/write" -o run -- python3 bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc3/write.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/pmc3/sq" -o run -- python3 bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc3/sq.log" 2>&1
echo rc_pytest=$rc
