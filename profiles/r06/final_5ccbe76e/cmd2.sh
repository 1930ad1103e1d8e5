# Round-6 final build, part 2 (profiles/traffic_latest.json now holds part 1's PMC of this build): the driver's default
# bench line, its rocprofv3 kernel-trace summary, the secondary lines and three tolerance lines
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final7b; mkdir -p $OUT
sha256sum mahi-mpc_amd/lib/libmmpc.so > $OUT/lib_sha256.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_default -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_default.json 2> $OUT/prof_default.err || { tail -20 $OUT/prof_default.err; exit 1; }
for f in $(find $OUT/prof_default -name "*kernel_stats.csv"); do cp "$f" $OUT/rocprof_kernel_stats_default.csv; head -6 "$f" | cut -c1-200; done
OUT2=$OUT/extra
sed "s#OUT=gpurun_out/extra#OUT=$OUT2#" tools/gpu_extra_lines.sh > /tmp/extra.sh
bash /tmp/extra.sh || exit 1
for t in 1e-5 1e-6; do
  timeout -k 10 200 python bench.py --tol $t --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-sweep > $OUT2/cfg2tol$t.json || exit 1
  timeout -k 10 200 python bench.py --config cfg3 --tol $t --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-sweep > $OUT2/cfg3tol$t.json || exit 1
done
echo done
