# resident finish of the 16-lane kernel (finished waves stay resident, sleeping, until <= 1/32 of the launch's waves
# still run): full GPU suite on the new build, then A/B against the same source with it compiled out (lib_var/nohold)
# at cfg#2 tol 1e-8 / 1e-6 / 1e-5 and at B = 512 / 8192 (the latter: grid beyond one resident round, hold off)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/resfin; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/nohold/libmmpc.so > $O/sha.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
OUT=$O/t8 VARIANTS="nohold cur" CONFIGS="cfg2" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=$O/t6 VARIANTS="nohold cur" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--tol 1e-6" bash tools/gpu_ab.sh || exit 1
OUT=$O/t5 VARIANTS="nohold cur" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--tol 1e-5" bash tools/gpu_ab.sh || exit 1
OUT=$O/b512 VARIANTS="nohold cur" CONFIGS="cfg2" REPS=1 BENCH_ARGS="--batch 512" bash tools/gpu_ab.sh || exit 1
OUT=$O/b8k VARIANTS="nohold cur" CONFIGS="cfg2" REPS=1 BENCH_ARGS="--batch 8192" bash tools/gpu_ab.sh || exit 1
for t in "1e-5 1e-7" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg2_$1.json || exit 1
done
echo ok
