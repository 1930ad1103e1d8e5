#!/bin/bash
# Round-2 checkpoint: all GPU tests, the three bench lines (cfg#2 headline, cfg#3, cfg#5 with its tolerance sweep),
# rocprof kernel stats of cfg#2 / cfg#3, and PMC passes for both solve kernels (refreshes profiles/traffic_latest.json).
set -o pipefail
OUT=${OUT:-gpurun_out/r02g}
mkdir -p "$OUT"
export TMPDIR=/tmp
MMPC_TEST_LOG="$PWD/$OUT/agreement.log" timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$OUT/pytest_gpu.log"
grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20
[ $rc -le 1 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py > "$OUT/bench_cfg2.json" || exit 1
timeout -k 10 300 python bench.py --config cfg3 --steps 5 --warmup 1 > "$OUT/bench_cfg3.json" || exit 1
timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 > "$OUT/bench_cfg5.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg2" -o run -- python bench.py --no-cpu-baseline > "$OUT/prof_cfg2.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg3" -o run -- python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_cfg3.json" || exit 1
OUT=$OUT/pmc_cfg2 KERNEL=sqp_group_kernel BENCH_ARGS="--config cfg2" \
  SUMMARY_ARGS="--traffic-json profiles/traffic_latest.json --key cfg2:sqp_group_kernel<TwoLinkArm> --batch 4096 --horizon 30 --source profiles/r02/pmc_cfg2_group_exact_v1.json" \
  ./tools/pmc.sh > "$OUT/pmc_cfg2.log" 2>&1 || { tail -20 "$OUT/pmc_cfg2.log"; exit 1; }
OUT=$OUT/pmc_cfg3 KERNEL=sqp_lane_kernel BENCH_ARGS="--config cfg3" \
  SUMMARY_ARGS="--traffic-json profiles/traffic_latest.json --key cfg3:sqp_lane_kernel<ExoArm> --batch 65536 --horizon 50 --source profiles/r02/pmc_cfg3_lane_v3.json" \
  ./tools/pmc.sh > "$OUT/pmc_cfg3.log" 2>&1 || { tail -20 "$OUT/pmc_cfg3.log"; exit 1; }
cp profiles/traffic_latest.json "$OUT/traffic_latest.json"
for f in bench_cfg2 bench_cfg3 bench_cfg5; do python3 -c "import json,sys; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['kernel_ms'], d['mean_sqp_iters'], d['max_sqp_iters'], d.get('cpu_baseline',{}).get('value'))"; done
echo rc_pytest=$rc
