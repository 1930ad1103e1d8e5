# cfg#2 with the K / W workspace stores non-temporal (lib_var/nt, -DMMPC_GROUP_NT_STORES=1; rejected: profiles/r06/nt/t8)
# against the shipped build: kernel time and the FETCH / WRITE / SQ wait counters of both, to show why
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ntpmc; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
OUT=$O/ab VARIANTS="nt cur" CONFIGS="cfg2" REPS=2 bash tools/gpu_ab.sh || exit 1
for v in nt cur; do
  L=$PWD/lib_var/$v/libmmpc.so; [ $v = cur ] && L=$PWD/mahi-mpc_amd/lib/libmmpc.so
  export MMPC_LIB_PATH=$L
  for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
    tag=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${v}_$tag -o run -- python3 bench.py --config cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_${v}_$tag.log 2>&1 || { tail -5 $O/pmc_${v}_$tag.log; exit 1; }
  done
  unset MMPC_LIB_PATH
done
echo ok
