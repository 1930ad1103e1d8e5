# cfg#2 at tol 1e-5 vs 1e-8: instruction-cache counters of the solve kernel (one rocprofv3 pass each), and the
# tail-latency microbenchmark (memory-busy waves leaving: does a lone wave's memory latency change?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/icache; mkdir -p $O
timeout -k 10 200 tools/ubench/tail_latency > $O/tail_latency.txt 2>&1 || exit 1
for t in 1e-5 1e-8; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$t -o run -- python3 bench.py --tol $t --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_$t.log 2>&1 || { tail -5 $O/pmc_$t.log; exit 1; }
done
echo ok
