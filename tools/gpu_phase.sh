set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/phase1
for k in 1 3; do
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt $k > gpurun_out/phase1/cfg2_kkt$k.json || exit 1
done
MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --horizon 100 > gpurun_out/phase1/n100_kkt3.json
cat gpurun_out/phase1/*.json
