#!/bin/bash
# Runs the ThreadSanitizer builds of tools/tsan_build.sh on the GPU box: ModelControl's threaded loop
# (model_control_example ... thread: worker thread + 1 kHz plant thread) and BatchModelControl's async loop.
# Reports go to gpurun_out/tsan/tsan.<pid>; the script prints the number of reports (after tools/tsan.supp, which
# drops reports inside the uninstrumented HIP/ROCr runtimes).
set -o pipefail
REPO=$PWD
BIN=$REPO/mahi-mpc_amd/host/bin/tsan
MODEL=$PWD/mahi-mpc_amd/lib/user/nonlinear_double_pendulum
OUT=${OUT:-gpurun_out/tsan}
mkdir -p "$OUT" && cd "$OUT" || exit 1
export TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 log_path=$PWD/tsan suppressions=$REPO/tools/tsan.supp"
# gcc 11's TSan expects the executable in its fixed application range; the box's ASLR places PIE binaries
# elsewhere ("unexpected memory mapping"), so the runs start with address randomisation off (setarch -R execs the
# program before anything touches the GPU)
R="setarch $(uname -m) -R"
timeout -k 10 240 $R "$BIN/model_control_example" 20 0.5 n - thread > mc_thread.out 2> mc_thread.err
echo "model_control thread rc=$?"; tail -2 mc_thread.out
timeout -k 10 240 $R "$BIN/batch_control_example" "$MODEL" 64 0.3 async > bc_async.out 2> bc_async.err
echo "batch_control async rc=$?"; tail -2 bc_async.out
echo "race reports: $(cat tsan.* 2>/dev/null | grep -c 'WARNING: ThreadSanitizer')"
ls
