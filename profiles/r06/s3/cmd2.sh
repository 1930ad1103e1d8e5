# cfg#2 tol 1e-5: the W pass's stores vs its fence (timing build with -DMMPC_PHASE_FENCE_IN_LOAD: the fence's wait
# accumulates into the "load" phase)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s3b; mkdir -p $O
for t in "1e-5 1e-7" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg2_$1.json || exit 1
done
echo ok
