# two more runs of the driver's default command on the final build (run-to-run spread)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final8r; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so > $O/sha.txt
for r in 1 2; do
  timeout -k 10 400 python bench.py > $O/bench_$r.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$r.json')); s=d['secondary']; print($r, round(d['value']), round(d['kernel_ms'],4), round(s['cfg3']['value']), round(s['cfg3']['kernel_ms'],3), round(s['cfg5']['value']), round(s['cfg5']['kernel_ms'],3), d['roofline']['pmc_status'][:30])"
done
