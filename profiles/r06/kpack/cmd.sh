# Lane kernel gain record with H_ww^-1 (10 values) instead of K_u (16) for unbounded and state-bounded solves (cur)
# against the previous layout (kp0): full GPU suite on cur; V* cur vs kp0 (roundoff: same iteration counts?);
# same-box A/B cfg#3 / cfg#5 and the exact-Hessian cfg#3 line (also against lz0: lazy step records off); PMC of cur
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/kpack; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for w in "cfg3" "cfg5" "cfg3 --hessian exact" "cfg3 --x-bound 1.5"; do
  set -- $w; tag=$(echo "$w" | tr ' ' '_' | tr -d '-')
  timeout -k 10 120 python tools/v_dump.py --config $w --out /tmp/v_cur_$tag.npz > /dev/null || exit 1
  MMPC_LIB_PATH=$PWD/lib_var/kp0/libmmpc.so timeout -k 10 120 python tools/v_dump.py --config $w --out /tmp/v_kp0_$tag.npz > /dev/null || exit 1
  python tools/v_dump.py --compare /tmp/v_cur_$tag.npz /tmp/v_kp0_$tag.npz >> $O/compare.txt
  python - /tmp/v_cur_$tag.npz /tmp/v_kp0_$tag.npz >> $O/compare.txt <<'PY'
import sys, numpy as np
a, b = (np.load(f) for f in sys.argv[1:])
same = a["iters"] == b["iters"]
rel = np.abs(a["V"] - b["V"]).max(1) / np.abs(b["V"]).max(1)
print(f"  same iteration count {same.sum()} / {same.size}, max rel V (same counts) {rel[same].max():.2e}, all {rel.max():.2e}, converged {(a['status'] == 0).sum()}")
PY
  rm -f /tmp/v_*_$tag.npz
done
cat $O/compare.txt
OUT=$O/ab VARIANTS="kp0 cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=$O/abx VARIANTS="kp0 lz0 cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--hessian exact" bash tools/gpu_ab.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_cur_$c -o run -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_cur_$c.log 2>&1 || { tail -5 $O/pmc_cur_$c.log; exit 1; }
done
echo ok
