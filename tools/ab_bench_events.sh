set -o pipefail
mkdir -p gpurun_out/ab_ev
for r in 1 2; do
  for v in old new; do
    f=bench.py; [ $v = old ] && f=bench_old_ab.py
    timeout -k 10 120 python $f --no-cpu-baseline --no-secondary --no-sweep --steps 50 --warmup 5 > gpurun_out/ab_ev/$v$r.json 2> gpurun_out/ab_ev/$v$r.err || { tail gpurun_out/ab_ev/$v$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_ev/$v$r.json')); print('$v', d['value'], d['ms_per_step'], d['kernel_ms'])"
  done
done
