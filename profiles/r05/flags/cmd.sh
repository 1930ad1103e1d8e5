#!/bin/bash
# compiler-flag A/B of the whole library (cfg#2 headline, cfg#3): scheduler metric bias 0, AMDGPU register-pressure
# trackers, no high-RP reschedule stage, -O2
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/flags; mkdir -p $OUT
OUT=$OUT/cfg2 VARIANTS="cur bias0 trk nohrp o2" CONFIGS="cfg2" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$OUT/cfg3 VARIANTS="cur bias0 trk nohrp o2" CONFIGS="cfg3" REPS=1 bash tools/gpu_ab.sh || exit 1
