# FETCH / WRITE PMC passes of the three builds of profiles/r06/crec/cmd.sh on cfg#3 (that call's npz dumps overflowed
# the copy-back, so its PMC output was lost)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/crecpmc; mkdir -p $O
sha256sum mahi-mpc_amd/lib/libmmpc.so lib_var/*/libmmpc.so > $O/sha.txt
for v in noc cur xk; do
  L=$PWD/lib_var/$v/libmmpc.so; [ $v = cur ] && L=$PWD/mahi-mpc_amd/lib/libmmpc.so
  export MMPC_LIB_PATH=$L
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > $O/pmc_${v}_$c.log 2>&1 || { tail -5 $O/pmc_${v}_$c.log; exit 1; }
  done
  unset MMPC_LIB_PATH
done
echo ok
