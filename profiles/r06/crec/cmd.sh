# Lane kernel stage-record traffic: the step sweep recomputes c_k from its own model evaluation instead of loading C
# (cur) against loading it (noc), and a probe that stores the gains K back (xk: + the K record's write traffic).
# Full GPU suite on cur; V* bit for bit cur vs noc on five lane workloads; same-box A/B on cfg#3 / cfg#5; FETCH/WRITE
# PMC passes of each build on cfg#3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/crec; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for w in "cfg3" "cfg5" "cfg3 --hessian exact" "cfg3 --u-bound 0.5" "cfg3 --x-bound 1.5"; do
  set -- $w; tag=$(echo "$w" | tr ' ' '_' | tr -d '-')
  timeout -k 10 120 python tools/v_dump.py --config $w --out $O/v_cur_$tag.npz || exit 1
  MMPC_LIB_PATH=$PWD/lib_var/noc/libmmpc.so timeout -k 10 120 python tools/v_dump.py --config $w --out $O/v_noc_$tag.npz || exit 1
  python tools/v_dump.py --compare $O/v_cur_$tag.npz $O/v_noc_$tag.npz | tee -a $O/bitwise.txt
done
OUT=$O/ab VARIANTS="noc cur xk" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
for v in noc cur xk; do
  L=$PWD/lib_var/$v/libmmpc.so; [ $v = cur ] && L=$PWD/mahi-mpc_amd/lib/libmmpc.so
  export MMPC_LIB_PATH=$L
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_${v}_$c.log 2>&1 || { tail -5 $O/pmc_${v}_$c.log; exit 1; }
  done
  unset MMPC_LIB_PATH
done
echo ok
