# Round-6 final build, part 3: phase profiles of the timing build (spread end-of-wave atomics) for cfg#2 and cfg#3,
# and two more runs of the driver's default command on the same box (run-to-run spread)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final7c; mkdir -p $O/phase $O/repeat
sha256sum mahi-mpc_amd/lib/libmmpc.so mahi-mpc_amd/lib/libmmpc_timing.so > $O/sha.txt
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 > $O/phase/phase_cfg2.json || exit 1
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 200 python tools/phase_profile.py --config cfg3 > $O/phase/phase_cfg3.json || exit 1
for r in 1 2; do
  timeout -k 10 400 python bench.py > $O/repeat/bench_$r.json 2> $O/repeat/err.txt || { tail -5 $O/repeat/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/repeat/bench_$r.json')); s=d['secondary']; print($r, round(d['value']), round(d['kernel_ms'],4), round(s['cfg3']['value']), round(s['cfg3']['kernel_ms'],3), round(s['cfg5']['value']), round(s['cfg5']['kernel_ms'],3))"
done
echo ok
