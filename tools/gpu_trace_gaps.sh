#!/bin/bash
# rocprofv3 kernel trace of the default cfg#2 bench (no secondary lines): per-launch durations and the gaps between
# consecutive solve kernels (negative = the next kernel started before the previous one ended).
set -o pipefail
OUT=${OUT:-gpurun_out/gaps}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --no-sweep > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted((r for r in csv.DictReader(open(sys.argv[1])) if 'sqp_group' in r['Kernel_Name']),
              key=lambda r: int(r['Start_Timestamp']))
prev = None
for r in rows:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(e - s, (s - prev) if prev is not None else None)
    prev = e
PY
cat "$OUT/bench.json"
