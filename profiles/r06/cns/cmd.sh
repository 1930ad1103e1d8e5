# Lane kernel without the C record (lib_var/cns: the backward sweep recomputes c_k from its Jacobian evaluation, the
# forward pass and the fused trial store no C): the lane-kernel GPU tests on that build, V* against the shipped build
# (roundoff expected, same iteration counts?), same-box A/B cfg#3 / cfg#5, FETCH / WRITE PMC on cfg#3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cns; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
MMPC_LIB_PATH=$PWD/lib_var/cns/libmmpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_riccati.py tests/test_gpu_tail.py tests/test_gpu_exact_lane.py tests/test_gpu_xbounds.py tests/test_gpu_bounds.py tests/test_gpu_parity.py tests/test_gpu_cfg4.py -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for w in "cfg3" "cfg5" "cfg3 --hessian exact" "cfg3 --u-bound 0.5"; do
  set -- $w; tag=$(echo "$w" | tr ' ' '_' | tr -d '-')
  timeout -k 10 120 python tools/v_dump.py --config $w --out /tmp/v_cur_$tag.npz > /dev/null || exit 1
  MMPC_LIB_PATH=$PWD/lib_var/cns/libmmpc.so timeout -k 10 120 python tools/v_dump.py --config $w --out /tmp/v_cns_$tag.npz > /dev/null || exit 1
  python tools/v_dump.py --compare /tmp/v_cur_$tag.npz /tmp/v_cns_$tag.npz | tee -a $O/compare.txt
  python - /tmp/v_cur_$tag.npz /tmp/v_cns_$tag.npz >> $O/compare.txt <<'PY'
import sys, numpy as np
a, b = (np.load(f) for f in sys.argv[1:])
same = a["iters"] == b["iters"]
rel = np.abs(a["V"] - b["V"]).max(1) / np.abs(a["V"]).max(1)
print(f"  same iteration count {same.sum()} / {same.size}, max rel V (same counts) {rel[same].max():.2e}, all {rel.max():.2e}")
PY
  rm -f /tmp/v_*_$tag.npz
done
cat $O/compare.txt
OUT=$O/ab VARIANTS="cur cns" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
export MMPC_LIB_PATH=$PWD/lib_var/cns/libmmpc.so
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_cns_$c -o run -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_cns_$c.log 2>&1 || { tail -5 $O/pmc_cns_$c.log; exit 1; }
done
echo ok
