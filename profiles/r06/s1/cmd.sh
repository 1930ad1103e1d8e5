set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s1; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/prev/libmmpc.so > $O/sha.txt
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$O/ab VARIANTS="prev cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=$O/ab_tol5 BENCH_ARGS="--tol 1e-5" VARIANTS="prev cur" CONFIGS="cfg3 cfg2" REPS=1 bash tools/gpu_ab.sh || exit 1
for t in "1e-5 1e-7" "1e-6 1e-8" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg2_$1.json || exit 1
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --config cfg3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg3_$1.json || exit 1
done
echo ok
