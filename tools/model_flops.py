#!/usr/bin/env python3
"""FP64 flops of one evaluation of each built-in model function, counted in the compiled gfx950 code.

    python tools/model_flops.py            # compiles tools/model_flops.hip, writes mahi-mpc_amd/mmpc/model_flops.json

Counts the FP64 VALU operations of each one-thread kernel of tools/model_flops.hip: v_fma/v_fmac_f64 = 2 flops,
every other v_*_f64 arithmetic op (add, mul, rcp, sqrt, rsq, ldexp, fract, trig_preop, div_scale/fmas/fixup,
min/max) = 1.  This is the model's DAG as the compiler emitted it, so sin/cos, division and square root count with
their expansions, except sin and cos: one op each as SURVEY.md 8(d) counts them (model_flops.hip replaces sincos by an
opaque stub; its asm markers are counted, 2 flops per sincos).  Loads,
stores, moves, selects and compares are not counted.  The JSON is read by bench.py's roofline to report the model
evaluation flops beside the kernel's own KKT-algebra count (mmpc.riccati_flops_per_iteration)."""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "model_flops.hip")
OUT = os.path.join(REPO, "mahi-mpc_amd", "mmpc", "model_flops.json")
ASM = "/tmp/model_flops.s"

NOT_FLOPS = ("v_mov", "v_cndmask", "v_cmp", "v_readlane", "v_writelane", "v_accvgpr", "v_class", "v_frexp_exp")


def count(body):
    fl, ops = 0, {}
    nsc = sum(1 for line in body if "sincos_stub" in line) // 2
    if nsc:
        ops["sin_cos_calls"] = nsc
        fl += 2 * nsc
    for line in body:
        m = re.match(r"\s+(v_\w+)", line)
        if not m or "f64" not in m.group(1) or m.group(1).startswith(NOT_FLOPS):
            continue
        op = m.group(1).replace("_e32", "").replace("_e64", "")
        ops[op] = ops.get(op, 0) + 1
        fl += 2 if op.startswith(("v_fma_f64", "v_fmac_f64")) else 1
    return fl, ops


def main():
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-mllvm", "-pragma-unroll-threshold=1000000", "-o", ASM, SRC], check=True)
    s = open(ASM).read()
    res = {}
    for m in re.finditer(r"^(flops_(\w+?)_(TwoLinkArm|ExoArm)):", s, re.M):
        name, fn, model = m.group(1), m.group(2), m.group(3)
        end = s.index(".Lfunc_end", m.end())
        fl, ops = count(s[m.end():end].split("\n"))
        res.setdefault(model, {})[fn] = {"flops": fl, "fp64_ops": ops}
    doc = {"_comment": "FP64 flops of one evaluation of each built-in model function in the compiled gfx950 code "
                       "(tools/model_flops.py over tools/model_flops.hip; FMA = 2, other FP64 VALU arithmetic = 1, "
                       "division/sqrt with their expansions, sin and cos 1 op each)", "models": res}
    json.dump(doc, open(OUT, "w"), indent=1)
    for model, fns in res.items():
        print(model, {k: v["flops"] for k, v in fns.items()})
    return 0


if __name__ == "__main__":
    sys.exit(main())
