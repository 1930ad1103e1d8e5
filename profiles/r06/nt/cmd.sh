# cfg#2 A/B: non-temporal W / K workspace stores (lib_var/nt) vs plain (cur), at tol 1e-8 and 1e-5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/nt; mkdir -p $O
OUT=$O/t8 VARIANTS="cur nt" CONFIGS="cfg2" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=$O/t5 VARIANTS="cur nt" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--tol 1e-5" bash tools/gpu_ab.sh || exit 1
echo ok
