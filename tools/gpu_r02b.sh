#!/bin/bash
# Round-2 GPU check after the parity tightening: all GPU tests with the achieved agreement logged, then PMC
# passes (traffic, FP64 VALU, MFMA counters) for the cfg#2 and cfg#3 solve kernels.
set -o pipefail
OUT=${OUT:-gpurun_out/r02b}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_TEST_LOG="$PWD/$OUT/agreement.log" timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -15 "$OUT/pytest_gpu.log"
grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
OUT=$OUT/pmc_cfg2 KERNEL=sqp_group_kernel BENCH_ARGS="--config cfg2" \
  SUMMARY_ARGS="--traffic-json profiles/traffic_latest.json --key cfg2:sqp_group_kernel<TwoLinkArm> --batch 4096 --horizon 30 --source profiles/r02/pmc_cfg2_group_v2.json" \
  ./tools/pmc.sh > "$OUT/pmc_cfg2.log" 2>&1 || { tail -20 "$OUT/pmc_cfg2.log"; exit 1; }
OUT=$OUT/pmc_cfg3 KERNEL=sqp_lane_kernel BENCH_ARGS="--config cfg3" \
  SUMMARY_ARGS="--traffic-json profiles/traffic_latest.json --key cfg3:sqp_lane_kernel<ExoArm> --batch 65536 --horizon 50 --source profiles/r02/pmc_cfg3_lane_v1.json" \
  ./tools/pmc.sh > "$OUT/pmc_cfg3.log" 2>&1 || { tail -20 "$OUT/pmc_cfg3.log"; exit 1; }
cp profiles/traffic_latest.json "$OUT/traffic_latest.json"
tail -30 "$OUT/pmc_cfg2.log"
echo rc_pytest=$rc
