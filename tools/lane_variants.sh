#!/bin/bash
# Rebuilds the three exo lane-kernel variants that computed wrong results in round 3 under several
# code-generation settings, for the miscompile diagnosis of round 4.  Each build is a patched copy of csrc/ in
# lib_var/<variant>_<flags>/ (git-ignored):
#   shipped   the tree as is
#   xbload    interior-point (XB) instantiation with the gains loaded in one batch before use (round 2/3 fault)
#   unifw     shared weights read through a lane-uniform pointer (Q, R, Rm in SGPRs; commit d1aa924)
#   lup       u_prev read at its uses instead of four registers (commit 630b29e)
# flag sets:
#   f0        the library's HIPFLAGS
#   nolr      + -mllvm -amdgpu-opt-vgpr-liverange=0   (SIOptimizeVGPRLiveRange off: VGPR live ranges across
#             divergent if/else and loop exits are not shortened)
#   prealloc  + -mllvm -amdgpu-prealloc-sgpr-spill-vgprs (the VGPRs that hold spilled SGPR lanes reserved up front)
#   sgprbasic / wwmbasic / vgprbasic
#             + -mllvm -{sgpr,wwm,vgpr}-regalloc=basic (the basic instead of the greedy allocator for that register
#             class: SGPRs, the whole-wave VGPRs that hold spilled SGPR lanes, ordinary VGPRs)
# SRC: the tree whose csrc/ is patched (default: this one; e.g. a git worktree of the round-3 commit e022ea8)
# Usage: tools/lane_variants.sh "shipped xbload unifw lup" "f0 nolr prealloc"   (builds in parallel, 4 at a time)
set -o pipefail
cd "$(dirname "$0")/.."
SRC=${SRC:-$PWD}
VARS=${1:-"shipped xbload unifw lup"}
FLAGS=${2:-"f0 nolr prealloc"}
BASE="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm -pragma-unroll-threshold=1000000"
build() {
  local v=$1 f=$2 d=lib_var/${1}_${2}
  rm -rf "$d" && mkdir -p "$d/csrc" "$d/include" && cp "$SRC"/mahi-mpc_amd/csrc/* "$d/csrc/" && cp "$SRC"/include/mmpc.h "$d/include/"
  local L=$d/csrc/sqp_lane.h
  case $v in
    xbload) python3 - "$L" <<'EOF'
import sys; p = sys.argv[1]; s = open(p).read()
old = "if constexpr (!XB) {\n                        // all loads of [K_k | kff_k]"
assert s.count(old) == 1; open(p, "w").write(s.replace(old, "if constexpr (true) {\n                        // all loads of [K_k | kff_k]"))
EOF
    ;;
    unifw) python3 - "$L" <<'EOF'
import sys; p = sys.argv[1]; s = open(p).read()
old = "const double* w = p.weights + inst * p.w_stride;"
assert s.count(old) == 1; open(p, "w").write(s.replace(old, "const double* w = p.weights;  // VARIANT unifw: shared weights only"))
EOF
    ;;
    lup) python3 - "$L" <<'EOF'
import sys; p = sys.argv[1]; s = open(p).read()
n = s.count("= up[c]") + s.count("= up[t]")
assert n >= 5, n
s = s.replace("= up[c]", "= p.u_prev[inst * NU + c]").replace("= up[t]", "= p.u_prev[inst * NU + t]")
open(p, "w").write(s)
EOF
    ;;
    shipped) ;;
    *) echo "unknown variant $v"; return 1;;
  esac
  local extra=""
  case $f in
    f0) ;;
    nolr) extra="-mllvm -amdgpu-opt-vgpr-liverange=0";;
    prealloc) extra="-mllvm -amdgpu-prealloc-sgpr-spill-vgprs";;
    sgprbasic) extra="-mllvm -sgpr-regalloc=basic";;
    wwmbasic) extra="-mllvm -wwm-regalloc=basic";;
    vgprbasic) extra="-mllvm -vgpr-regalloc=basic";;
    *) echo "unknown flags $f"; return 1;;
  esac
  # the copied mmpc.hip includes ../../include/mmpc.h relative to csrc: point it at the copy
  sed -i 's#"\.\./\.\./include/mmpc.h"#"../include/mmpc.h"#' "$d/csrc/mmpc.hip"
  /opt/rocm/bin/hipcc $BASE $extra -shared -Wl,-Bsymbolic -o "$d/libmmpc.so" "$d/csrc/mmpc.hip" > "$d/build.log" 2>&1 &&
  /opt/rocm/bin/hipcc $BASE $extra --cuda-device-only -S -o "$d/mmpc.s" "$d/csrc/mmpc.hip" >> "$d/build.log" 2>&1 &&
  echo "built $d" || { echo "FAILED $d"; tail -5 "$d/build.log"; }
}
jobs=0
for v in $VARS; do for f in $FLAGS; do
  build "$v" "$f" &
  jobs=$((jobs + 1))
  if [ $jobs -ge ${PAR:-4} ]; then wait -n; jobs=$((jobs - 1)); fi
done; done
wait
