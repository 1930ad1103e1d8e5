#!/bin/bash
# fast iteration loop: GPU parity tests, phase profile (diagnostic build), bench line
set -o pipefail
OUT=${OUT:-gpurun_out/iter}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest_gpu.log" | head -20; exit $rc; }
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 300 python tools/phase_profile.py > "$OUT/phase.json" 2> "$OUT/phase.err" || { tail "$OUT/phase.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/phase.json')); print('cycles/wave', int(d['cycles_per_wave'])); print({k: int(v) for k, v in d['per_phase_cycles_per_wave_iteration'].items()})"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('solves/s %.4g  kernel_ms %.4f  frac %.4f  iters %.3f' % (d['value'], d['kernel_ms'], d['roofline']['frac'], d['mean_sqp_iters']))"
