#!/bin/bash
# Riccati-path iteration: its parity tests, a cfg#3 bench line, the cfg#3 phase profile
set -o pipefail
OUT=${OUT:-gpurun_out/lane}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_riccati.py -q -x > "$OUT/pytest_riccati.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_riccati.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest_riccati.log" | head -30; exit $rc; }
timeout -k 10 300 python bench.py --config cfg3 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err" || { tail -20 "$OUT/bench_cfg3.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_cfg3.json')); print('cfg3 solves/s %.4g kernel_ms %.3f frac %.4f iters %.3f' % (d['value'], d['kernel_ms'], d['roofline']['frac'], d['mean_sqp_iters']))"
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 300 python tools/phase_profile.py --config cfg3 > "$OUT/phase3.json" 2> "$OUT/phase3.err" || { tail "$OUT/phase3.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/phase3.json')); print({k: int(v) for k, v in d['per_phase_cycles_per_wave_iteration'].items()})"
