# cfg#2 at tol 1e-5: is the last iteration of the straggler waves slow because the chip is idle around them?
# Timing builds whose finished waves stay resident 40 % of their own duration longer, sleeping (tsleep) or issuing
# FP64 FMAs (tspin), against the timing build whose waves exit; then the product build with a 30 % sleep (sleep)
# against the shipped one at tol 1e-5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sleep; mkdir -p $O
sha256sum lib_var/*/libmmpc.so mahi-mpc_amd/lib/libmmpc*.so > $O/sha.txt
for rep in 1 2; do
for v in timing tsleep tspin; do
  L=$PWD/lib_var/$v/libmmpc.so; [ $v = timing ] && L=$PWD/mahi-mpc_amd/lib/libmmpc_timing.so
  MMPC_LIB_PATH=$L timeout -k 10 120 python tools/phase_profile.py --kkt 3 --tol-grad 1e-5 --tol-defect 1e-7 > $O/phase_${v}_1e-5_$rep.json || exit 1
  python3 -c "import json; d=json.load(open('$O/phase_${v}_1e-5_$rep.json')); print('$v', d['span_us'], d['wave_us_percentiles'], d['mean_us_by_wave_max_iters'])"
done
done
OUT=$O/t5 VARIANTS="cur sleep" CONFIGS="cfg2" REPS=2 BENCH_ARGS="--tol 1e-5" bash tools/gpu_ab.sh || exit 1
echo ok
