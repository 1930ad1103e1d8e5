#!/bin/bash
# ThreadSanitizer build of the multi-threaded host mirror (ModelControl's worker thread, BatchModelControl's
# streams/events and host-side publication) with its two threaded drivers, for a run on the GPU box
# (tools/tsan_run.sh).  Host code only: g++ -fsanitize=thread over mahi-mpc_amd/host/src; libmmpc.so and the HIP
# runtime stay uninstrumented (no GPU sanitizer).  Output: mahi-mpc_amd/host/bin/tsan/ (not in git).
set -e
cd "$(dirname "$0")/../mahi-mpc_amd/host"
OUT=bin/tsan
mkdir -p $OUT
FL="-O1 -g -std=c++17 -fPIC -fsanitize=thread -include $PWD/../../tools/tsan_compat.h -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__"
LIBS="-L../lib -lmmpc -Wl,-rpath,$PWD/../lib -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lpthread -ldl"
SRCS="src/ModelParameters.cpp src/ModelControl.cpp src/ModelGenerator.cpp src/External.cpp src/SX.cpp src/BatchModelControl.cpp"
g++ $FL -o $OUT/model_control_example examples/model_control_example.cpp $SRCS $LIBS &
g++ $FL -o $OUT/batch_control_example examples/batch_control_example.cpp $SRCS $LIBS &
wait
ls -la $OUT
