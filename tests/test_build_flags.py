"""CPU: the register-allocator policy of the build.  ROCm 7.2's greedy SGPR allocator miscompiled six
kernels at the 512-register limit (five exo lane-kernel builds, the exo group kernel with the exact Hessian); every
kernel unit is therefore compiled with -mllvm -sgpr-regalloc=basic except csrc/group_two_link.hip (the built-in 2-link
group kernels of cfg#2, which do not spill VGPRs).  These checks keep a later edit of the Makefile or of
ModelGenerator::compile_model from dropping the flag silently."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AMD = os.path.join(ROOT, "mahi-mpc_amd")


def _rules(makefile):
    """target -> recipe lines of a simple Makefile"""
    rules, cur = {}, None
    for line in open(makefile).read().splitlines():
        m = re.match(r"^([^\s:=#][^:=]*):(?!=)", line)
        if m:
            cur = m.group(1).strip()
            rules[cur] = []
        elif line.startswith("\t") and cur:
            rules[cur].append(line.strip())
    return rules


def test_makefile_units_and_allocator():
    mk = os.path.join(AMD, "Makefile")
    text = open(mk).read()
    assert re.search(r"^LANEFLAGS \?= -mllvm -sgpr-regalloc=basic$", text, re.M)
    r = _rules(mk)
    for obj in ("build/mmpc.o", "build/lane_kernels.o", "build/mmpc_timing.o", "build/lane_kernels_timing.o"):
        assert any("$(LANEFLAGS)" in l for l in r[obj]), obj
    for obj in ("build/group_two_link.o", "build/group_two_link_timing.o"):
        assert r[obj] and not any("LANEFLAGS" in l for l in r[obj]), obj
    link = " ".join(r["lib/libmmpc.so"])
    for obj in ("build/mmpc.o", "build/lane_kernels.o", "build/group_two_link.o"):
        assert obj in link


def test_two_link_group_kernels_only_in_their_unit():
    """mmpc.hip launches the built-in 2-link group kernels through group_launch.h and never instantiates them"""
    src = open(os.path.join(AMD, "csrc", "mmpc.hip")).read()
    assert "launch_group_two_link(" in src
    assert "sqp_group_kernel<TwoLinkArm" not in src
    grp = open(os.path.join(AMD, "csrc", "group_two_link.hip")).read()
    assert "sqp_group_kernel<TwoLinkArm" in grp


def test_generated_model_libraries_use_the_basic_allocator():
    """ModelGenerator::compile_model builds both kernel units of a user model with the basic SGPR allocator"""
    src = open(os.path.join(AMD, "host", "src", "ModelGenerator.cpp")).read()
    i = src.index("const std::string cmds[3]")
    block = src[i:src.index("};", i)]
    compiles = [l for l in block.splitlines() if "-c '" in l]
    assert len(compiles) == 2 and all("-sgpr-regalloc=basic" in l for l in compiles), compiles
