# (bench.py patch of this A/B not kept: see DESIGN.md 5)
# bench.py: step k+1's input generation on a second stream overlapping step k's solve (double-buffered inputs;
# default) against generation and solve in sequence (--no-overlap), alternating, cfg#2 / cfg#3 / cfg#5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/overlap; mkdir -p $O
for rep in 1 2 3; do
  for c in cfg2 cfg3 cfg5; do
    for v in seq ovl; do
      a=""; [ $v = seq ] && a="--no-overlap"
      timeout -k 10 200 python bench.py --config $c $a --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-sweep > $O/${c}_${v}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${c}_${v}_$rep.json')); print('$c $v', round(d['value']), round(d['ms_per_step'], 4), round(d['kernel_ms'], 4), round(d['step_gpu_ms'], 4), d['converged'], d['gathered_results_match'], d['zero_copy_results_checked'])"
    done
  done
done
echo ok
