# Lane kernel line-search hand-over (cur) against lsh0, and -- if cur's cfg#3 line is faster -- the final evidence of
# cur in the same call (PMC of cfg#2/#3/#5 keyed to its sha, the default bench line, its rocprof summary)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lsh; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python tools/block_stats.py --config cfg3 --blocks 24 > $O/blocks_cur.jsonl || exit 1
python3 -c "
import json
print(';'.join(str((d['block'], d['kernel_ms'])) for d in map(json.loads, open('$O/blocks_cur.jsonl'))))"
for c in cfg3 cfg5; do
  timeout -k 10 120 python tools/v_dump.py --config $c --out /tmp/v_cur_$c.npz > /dev/null || exit 1
  MMPC_LIB_PATH=$PWD/lib_var/lsh0/libmmpc.so timeout -k 10 120 python tools/v_dump.py --config $c --out /tmp/v_lsh0_$c.npz > /dev/null || exit 1
  python tools/v_dump.py --compare /tmp/v_cur_$c.npz /tmp/v_lsh0_$c.npz | tee -a $O/compare.txt
  rm -f /tmp/v_*_$c.npz
done
OUT=$O/ab VARIANTS="lsh0 cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
python3 - $O/ab > $O/decision.txt <<'PY'
import json, glob, sys, statistics as st
d = sys.argv[1]
m = {v: st.mean(json.load(open(f))["ms_per_step"] for f in glob.glob(f"{d}/b_{v}_cfg3_*.json")) for v in ("lsh0", "cur")}
print("adopt" if m["cur"] < m["lsh0"] else "reject", m)
PY
cat $O/decision.txt
grep -q adopt $O/decision.txt || { echo "not adopted: no final evidence for this build"; exit 0; }
OUT=gpurun_out/final8 SKIP_BENCH=1 PMC_LABEL_DIR=profiles/r06/final/pmc bash tools/gpu_final.sh || exit 1
cp gpurun_out/final8/pmc/traffic_latest.json profiles/traffic_latest.json
F=gpurun_out/final8
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $F/bench_default.json 2> $F/bench_default.err || { tail -20 $F/bench_default.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $F/prof_default -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $F/prof_default.json 2> $F/prof_default.err || { tail -20 $F/prof_default.err; exit 1; }
for f in $(find $F/prof_default -name "*kernel_stats.csv"); do cp "$f" $F/rocprof_kernel_stats_default.csv; done
rm -f $F/prof_default/run_kernel_trace.csv
echo ok
