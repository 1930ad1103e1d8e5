#!/bin/bash
# rocprofv3 kernel-trace summaries of the bounded exo solves at cfg#3 size (lane kernel + 16-lane resume launch)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_bounded; mkdir -p $OUT
for c in "xb15:--x-bound 1.5" "ub05:--u-bound 0.5"; do
  n=${c%%:*}; a=${c#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 bench.py --config cfg3 $a --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-sweep > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  f=$(find $OUT/$n -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/${n}_kernel_stats.csv; grep -E "sqp_" "$f" | cut -c1-160
done
