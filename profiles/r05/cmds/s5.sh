#!/bin/bash
# instance generators (draws once per instance in LDS): bit-identity with the oracle, then their kernel times
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5s5; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg4.py -q -m gpu -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sweep > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
grep -i "synth\|Name" $(find $OUT/prof -name "*kernel_stats.csv") | cut -c1-200
python3 -c "
import json; b=json.load(open('$OUT/bench.json')); print(b['value'], b['value_solve_only'], b['kernel_ms'], b['step_gpu_ms'])
for c,v in b['secondary'].items(): print(c, v['value'], v['value_solve_only'], v['kernel_ms'], v['step_gpu_ms'])"
