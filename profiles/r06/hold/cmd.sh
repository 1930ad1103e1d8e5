# cfg#2 tolerance anomaly: finished waves held resident until the whole launch has finished (lib_var/hold,
# -DMMPC_GROUP_HOLD_EXIT) against the shipped exit, at tol 1e-8 / 1e-6 / 1e-5, alternating builds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hold; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/hold/libmmpc.so > $O/sha.txt
OUT=$O/t8 VARIANTS="cur hold" CONFIGS="cfg2" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=$O/t6 VARIANTS="cur hold" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--tol 1e-6" bash tools/gpu_ab.sh || exit 1
OUT=$O/t5 VARIANTS="cur hold" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--tol 1e-5" bash tools/gpu_ab.sh || exit 1
echo ok
