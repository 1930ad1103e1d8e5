#!/bin/bash
# A/B library build: lib_var/<name>/libmmpc.so from a copy of mahi-mpc_amd/ (csrc + Makefile) of SRC (default: this
# tree; e.g. a `git worktree` of an older commit) with extra compiler flags (e.g. -DMMPC_LANE_WPE32=2), for
# tools/gpu_ab.sh.  Usage: tools/build_variant.sh <name> "<extra hipcc flags>" [SRC]
set -eo pipefail
cd "$(dirname "$0")/.."
name=$1; extra=${2:-}; SRC=${3:-$PWD}
d=lib_var/$name
rm -rf "$d" && mkdir -p "$d/mahi-mpc_amd" "$d/include"
cp -r "$SRC/mahi-mpc_amd/csrc" "$SRC/mahi-mpc_amd/Makefile" "$d/mahi-mpc_amd/"
cp "$SRC/include/mmpc.h" "$d/include/"
base="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm -pragma-unroll-threshold=1000000"
make -s -j4 -C "$d/mahi-mpc_amd" HIPFLAGS="$base $extra" lib/libmmpc.so 2>&1 | grep -v "argument unused" || true
cp "$d/mahi-mpc_amd/lib/libmmpc.so" "$d/libmmpc.so"
rm -rf "$d/mahi-mpc_amd/build"
sha256sum "$d/libmmpc.so"
