#!/bin/bash
# Group Riccati kernel: parity tests, solver comparison benches, phase profile (diagnostic build).
set -o pipefail
OUT=${OUT:-gpurun_out/group}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_riccati.py tests/test_gpu_bounds.py -q -x -k "group or exo" > "$OUT/pytest_group.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_group.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest_group.log" | head -30; exit $rc; }
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -20 "$OUT/bench_$tag.err"; return 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag solves/s %.4g kernel_ms %.4f iters %.3f conv %d' % (d['value'], d['kernel_ms'], d['mean_sqp_iters'], d['converged']))"
}
run cfg2_condensed --kkt condensed && run cfg2_group --kkt group && \
run n100_group --kkt group --horizon 100 && run n100_lane --kkt riccati --horizon 100 && \
run exo_n20_group --config cfg3 --batch 4096 --horizon 20 --kkt group && run exo_n20_lane --config cfg3 --batch 4096 --horizon 20 --kkt riccati || exit 1
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 > "$OUT/phase_cfg2_group.json" || exit 1
python -c "import json; d=json.load(open('$OUT/phase_cfg2_group.json')); print({k: round(v) for k, v in d['per_phase_cycles_per_wave_iteration'].items()})"
