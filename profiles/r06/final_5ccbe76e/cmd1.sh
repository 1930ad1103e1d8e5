# Round-6 final build, part 1: the whole GPU suite, smoke, and the PMC passes of cfg#2 / cfg#3 / cfg#5 keyed to the
# library's sha256 (tools/gpu_final.sh without the bench; its traffic_latest.json goes into profiles/ afterwards)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final7 SKIP_BENCH=1 PMC_LABEL_DIR=profiles/r06/final/pmc bash tools/gpu_final.sh
