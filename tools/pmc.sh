#!/bin/bash
# PMC passes over a short bench run: one counter group per rocprofv3 invocation (kernel-trace only, no
# sys/runtime tracing), plus a kernel-trace-only pass for the undisturbed kernel duration.
#   OUT=gpurun_out/pmc_cfg2 KERNEL=sqp_group_kernel BENCH_ARGS="--config cfg2" tools/pmc.sh
# The summary records the sha256 of the library the passes loaded; bench.py attaches PMC fields only to a run of
# that same build.  Every pass is a single-configuration, single-tolerance bench run (no secondary lines, no
# cfg#5 tolerance sweep, no CPU baseline).
set -o pipefail
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, rocprofv3 options...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace "$@" --output-format csv -d "$OUT/$name" -o run -- python3 bench.py ${BENCH_ARGS:-} --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-sweep > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$OUT/$name.log"; return 1; }
}
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
have() { grep -qw "$1" "$OUT/counters.txt"; }
MF=""
for c in SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64; do have $c && MF="$MF $c"; done
run trace --stats && \
run fetch --pmc FETCH_SIZE && run write --pmc WRITE_SIZE && \
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run sq2 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SALU && \
run sq3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM && \
{ [ -z "$MF" ] || run mfma --pmc $MF; } && \
LIBSHA=$(sha256sum "${MMPC_LIB_PATH:-mahi-mpc_amd/lib/libmmpc.so}" | cut -d' ' -f1)
python3 tools/pmc_summary.py "$OUT" "${KERNEL:-sqp_group_kernel}" --lib-sha256 "$LIBSHA" ${SUMMARY_ARGS:-}
