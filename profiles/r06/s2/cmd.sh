# cfg#2 tolerance anomaly: phase profiles with the wall-clock extents (span, longest wave, clock) at three tolerances,
# twice each, plus the lane kernel's at 1e-5 / 1e-8
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s2; mkdir -p $O
for rep in 1 2; do
for t in "1e-5 1e-7" "1e-6 1e-8" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg2_$1_$rep.json || exit 1
done
done
for t in "1e-5 1e-7" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --config cfg3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg3_$1.json || exit 1
done
echo ok
