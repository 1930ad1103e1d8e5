# GPU suite on the current build (new: trig domain, batch composition, multi-device lane solver); A/B of the driver
# lines against round 5's final library (synth staging + lean sweep); cfg#2 tolerance anomaly: phase profiles with the
# wall-clock extents (span, longest wave, clock) at three tolerances, twice each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s2; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/prev/libmmpc.so > $O/sha.txt
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
OUT=$O/ab VARIANTS="prev cur" CONFIGS="cfg3 cfg5 cfg2" REPS=2 bash tools/gpu_ab.sh || exit 1
for rep in 1 2; do
for t in "1e-5 1e-7" "1e-6 1e-8" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg2_$1_$rep.json || exit 1
done
done
echo ok
