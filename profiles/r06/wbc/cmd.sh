# cfg#2 tolerance anomaly, second probe: (1) V written back 16 consecutive doubles per store (lib_var/wbc) against the
# shipped row-wise write-back, tol 1e-8 / 1e-5, alternating builds; (2) phase profiles of the timing build whose
# end-of-wave atomics are now spread over 64 lines (per-wave durations without the one-line atomic hot spot);
# (3) state bounds with the exact Hessian against Gauss-Newton at full size (cfg#2 |qdot| <= 1.5, exo cfg#3 size)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wbc; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/wbc/libmmpc.so mahi-mpc_amd/lib/libmmpc_timing.so > $O/sha.txt
OUT=$O/t8 VARIANTS="cur wbc" CONFIGS="cfg2" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=$O/t5 VARIANTS="cur wbc" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--tol 1e-5" bash tools/gpu_ab.sh || exit 1
for t in "1e-5 1e-7" "1e-6 1e-8" "1e-8 1e-10"; do set -- $t
  MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad $1 --tol-defect $2 > $O/phase_cfg2_$1.json || exit 1
done
for hs in gauss_newton exact; do
  timeout -k 10 200 python bench.py --x-bound 1.5 --hessian $hs --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --no-sweep > $O/xb_cfg2_$hs.json || exit 1
  timeout -k 10 300 python bench.py --config cfg3 --x-bound 1.5 --hessian $hs --steps 5 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/xb_cfg3_$hs.json || exit 1
done
echo ok
