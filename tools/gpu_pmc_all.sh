#!/bin/bash
# PMC passes (tools/pmc.sh) for the three bench configurations on the current library build: cfg#2 (16-lane group
# kernel, exact Hessian), cfg#3 (lane kernel, fp64), cfg#5 (lane kernel, fp32 factor, single tolerance).  Each
# summary is keyed to the library's sha256 in a copy of profiles/traffic_latest.json under $OUT (copy it back into
# profiles/ after the call); bench.py attaches the PMC fields only to a run of that same build.
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_all}
mkdir -p "$OUT"
export TMPDIR=/tmp
cp profiles/traffic_latest.json "$OUT/traffic_latest.json"
run() {  # tag kernel-substring key batch horizon bench-args
  local tag=$1 kern=$2 key=$3 batch=$4 hor=$5 bargs=$6
  local tj="$OUT/traffic_latest.json"
  OUT="$OUT/$tag" KERNEL="$kern" BENCH_ARGS="$bargs" \
    SUMMARY_ARGS="--traffic-json $tj --key $key --batch $batch --horizon $hor --source ${PMC_LABEL_DIR:-profiles/r05/final2/pmc}/${tag}_pmc_summary.json" \
    bash tools/pmc.sh > "$OUT/$tag.log" 2>&1 || { echo "pmc $tag failed"; tail -20 "$OUT/$tag.log"; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$tag/pmc_summary.json')); print('$tag', d.get('kernel_ms_trace_pass'), d.get('hbm_bytes_per_launch'), d.get('fp64_valu_frac_of_peak'), d.get('lib_sha256')[:12])"
}
run cfg2 "sqp_group_kernel<mmpc::TwoLinkArm" "cfg2:sqp_group_kernel<TwoLinkArm>" 4096 30 "--config cfg2" && \
run cfg3 "sqp_lane_kernel<mmpc::ExoArm, double" "cfg3:sqp_lane_kernel<ExoArm>" 65536 50 "--config cfg3" && \
run cfg5 "sqp_lane_kernel<mmpc::ExoArm, float" "cfg5:sqp_lane_kernel<ExoArm,fp32>" 65536 50 "--config cfg5"
