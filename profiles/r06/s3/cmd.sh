# cfg#2 at tol 1e-5 vs 1e-6 vs 1e-8: per-wave durations and clocks (the slowest waves and their instances' counts)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s3; mkdir -p $O
for t in "1e-5 1e-7" "1e-6 1e-8" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg2_$1.json || exit 1
done
echo ok
timeout -k 10 120 tools/ubench/tail_latency > $O/tail_latency.txt 2>&1 || exit 1
