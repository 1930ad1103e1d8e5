# State-bounded lane kernel: Sigma, b, z_u - z_l formed at their uses from the duals (cur) instead of SG / BB / ZG
# records written by the forward pass (xr0): state-bound GPU tests on cur, V* bit for bit on two state-bounded
# workloads, same-box A/B of the exo |qdot| <= 1.5 line at cfg#3 size (Gauss-Newton and exact) and cfg#3 / cfg#5
# (unchanged kernels: control)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/xrc; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_xbounds.py tests/test_gpu_tail.py tests/test_gpu_riccati.py tests/test_gpu_exact_lane.py -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for w in "cfg3 --x-bound 1.5" "cfg3 --x-bound 1.5 --hessian exact" "cfg2 --x-bound 1.5 --kkt riccati"; do
  set -- $w; tag=$(echo "$w" | tr ' ' '_' | tr -d '-')
  timeout -k 10 200 python tools/v_dump.py --config $w --out /tmp/v_cur_$tag.npz > /dev/null || exit 1
  MMPC_LIB_PATH=$PWD/lib_var/xr0/libmmpc.so timeout -k 10 200 python tools/v_dump.py --config $w --out /tmp/v_xr0_$tag.npz > /dev/null || exit 1
  python tools/v_dump.py --compare /tmp/v_cur_$tag.npz /tmp/v_xr0_$tag.npz | tee -a $O/compare.txt
  rm -f /tmp/v_*_$tag.npz
done
OUT=$O/xb VARIANTS="xr0 cur" CONFIGS="cfg3" REPS=2 BENCH_ARGS="--x-bound 1.5" bash tools/gpu_ab.sh || exit 1
OUT=$O/xbex VARIANTS="xr0 cur" CONFIGS="cfg3" REPS=1 BENCH_ARGS="--x-bound 1.5 --hessian exact" bash tools/gpu_ab.sh || exit 1
OUT=$O/ctl VARIANTS="xr0 cur" CONFIGS="cfg3 cfg5" REPS=1 bash tools/gpu_ab.sh || exit 1
echo ok
