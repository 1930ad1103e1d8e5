# cfg#2: the 2-link arm's structural zeros of W_k stored only in a launch's first W pass (cur) against every pass
# (wz0): group-kernel GPU tests on cur, V* bit for bit on cfg#2 (exact, unbounded / |u| <= 2 / |qdot| <= 1.5 exact),
# same-box A/B, WRITE / FETCH PMC of both on cfg#2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wzero; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_xbounds.py tests/test_gpu_bounds.py tests/test_gpu_exact_lane.py tests/test_gpu_tail.py tests/test_gpu_init.py -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for w in "cfg2" "cfg2 --hessian exact --u-bound 2" "cfg2 --hessian exact --x-bound 1.5"; do
  set -- $w; tag=$(echo "$w" | tr ' ' '_' | tr -d '-')
  timeout -k 10 120 python tools/v_dump.py --config $w --out /tmp/v_cur_$tag.npz > /dev/null || exit 1
  MMPC_LIB_PATH=$PWD/lib_var/wz0/libmmpc.so timeout -k 10 120 python tools/v_dump.py --config $w --out /tmp/v_wz0_$tag.npz > /dev/null || exit 1
  python tools/v_dump.py --compare /tmp/v_cur_$tag.npz /tmp/v_wz0_$tag.npz | tee -a $O/compare.txt
  rm -f /tmp/v_*_$tag.npz
done
OUT=$O/ab VARIANTS="wz0 cur" CONFIGS="cfg2" REPS=3 bash tools/gpu_ab.sh || exit 1
for v in wz0 cur; do
  L=$PWD/lib_var/$v/libmmpc.so; [ $v = cur ] && L=$PWD/mahi-mpc_amd/lib/libmmpc.so
  export MMPC_LIB_PATH=$L
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- python3 bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_${v}_$c.log 2>&1 || { tail -5 $O/pmc_${v}_$c.log; exit 1; }
  done
  unset MMPC_LIB_PATH
done
echo ok
