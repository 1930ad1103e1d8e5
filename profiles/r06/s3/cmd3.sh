# cfg#2 tol 1e-5: per-wave time by the wave's slowest instance at B = 512 / 1024 / 2048 / 4096 (waves per CU 0.5-4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s3c; mkdir -p $O
for b in 512 1024 2048 4096; do
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --batch $b --tol-grad 1e-5 --tol-defect 1e-7 > $O/phase_cfg2_b$b.json || exit 1
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --batch $b > $O/phase_cfg2_b${b}_tol8.json || exit 1
done
echo ok
