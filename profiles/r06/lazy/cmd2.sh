# second half of cmd.sh (its lazy-step test failed on a wrong expectation for one case): the lazy-step test, same-box
# A/B base / cns / cur on cfg#3 / cfg#5, FETCH / WRITE PMC of cur on cfg#3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lazy2; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_lazy_steps.py -v -s -m gpu --timeout 200 --timeout-method thread > $O/pytest_lazy.log 2>&1 || { grep -E "FAILED|Error|assert" $O/pytest_lazy.log | head; exit 1; }
grep -E "regenerated|passed" $O/pytest_lazy.log
OUT=$O/ab VARIANTS="base cns cur" CONFIGS="cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_cur_$c -o run -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_cur_$c.log 2>&1 || { tail -5 $O/pmc_cur_$c.log; exit 1; }
done
echo ok
