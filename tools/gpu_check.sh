#!/bin/bash
# One GPU check of the tree: GPU tests (names of failures kept in the log), smoke, the default bench line (cfg#2
# headline with the cfg#3 / cfg#5 secondary lines) and a rocprofv3 kernel-trace summary of it.
#   OUT=gpurun_out/r03_check1 tools/gpu_check.sh [pytest selection...]
set -o pipefail
OUT=${OUT:-gpurun_out/check}
mkdir -p "$OUT"
export TMPDIR=/tmp
SEL=${*:-tests}
timeout -k 10 900 python -u -m pytest $SEL -v -m gpu -x --timeout 300 --timeout-method thread -rA > "$OUT/pytest_gpu.log" 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" "$OUT/pytest_gpu.log" | grep -E "FAILED|ERROR" | head -20
tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest gpu rc=$rc: stopping"; exit $rc; }
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
def show(tag, x):
    cb = x.get("cpu_baseline") or {}
    print(tag, "value", round(x["value"]), "ms/step", round(x["ms_per_step"], 4), "kernel", round(x["kernel_ms"], 4),
          "conv", x["converged"], "iters", round(x["mean_sqp_iters"], 3), x["max_sqp_iters"], "frac",
          round(x["roofline"]["frac"], 4), "cpu", cb.get("value"), (cb.get("vs_gpu") or {}).get("max_rel_diff_V_same_iters"))
show("cfg2", d)
for k, v in (d.get("secondary") or {}).items():
    show(k, v)
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sweep > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
for f in $(find "$OUT/prof" -name "*kernel_stats.csv"); do cp "$f" "$OUT/rocprof_kernel_stats.csv"; head -6 "$f" | cut -c1-200; done
echo done
