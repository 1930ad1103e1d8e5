#!/bin/bash
# Round-5 session GPU evidence: the suite + smoke + default bench + rocprof of the current build (tools/gpu_final.sh,
# no PMC), then same-box A/B lines: the round-4 build (lib_var/r4, sha a8e1740d) against this one on cfg#2/#3/#5,
# the fp32-factor lane kernel at 2 waves per SIMD (lib_var/wpe2) on cfg#5, then the secondary lines.
set -o pipefail
SKIP_PMC=1 OUT=gpurun_out/r5a bash tools/gpu_final.sh || exit 1
OUT=gpurun_out/r5ab VARIANTS="r4 cur" CONFIGS="cfg2 cfg3 cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r5ab VARIANTS="wpe2 cur" CONFIGS="cfg5" REPS=2 bash tools/gpu_ab.sh || exit 1
bash tools/gpu_extra_lines.sh
