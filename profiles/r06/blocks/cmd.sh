# cfg#3 per instance block (the blocks bench.py's timed steps solve): kernel time, iterations, line-search halvings
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/blocks
timeout -k 10 300 python tools/block_stats.py --config cfg3 --blocks 24 > gpurun_out/blocks/cfg3.jsonl 2> gpurun_out/blocks/err.txt || { tail -5 gpurun_out/blocks/err.txt; exit 1; }
cut -c1-220 gpurun_out/blocks/cfg3.jsonl
