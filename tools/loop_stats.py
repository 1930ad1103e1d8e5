#!/usr/bin/env python3
"""Instruction mix per loop (innermost-header attribution) of a kernel in mahi-mpc_amd/build/mmpc.s
(make -C mahi-mpc_amd asm).  Diagnostic only.

    python tools/loop_stats.py [kernel-substring]   (default: the unbounded cfg#2 group kernel)"""
import collections
import re
import sys

ASM = sys.argv[2] if len(sys.argv) > 2 else "mahi-mpc_amd/build/mmpc.s"
key = sys.argv[1] if len(sys.argv) > 1 else "sqp_group_kernelINS_10TwoLinkArmELb0ELb0"
s = open(ASM).read()
name = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, re.M) if key in m.group(1)][0]
i = s.index(name + ":")
lines = s[i:s.index(".Lfunc_end", i)].split("\n")
loops = collections.OrderedDict()
cur = None
for l in lines:
    m = re.search(r"(?:Header=BB(\S+) Depth=(\d))|(?:This (?:Inner )?Loop Header: Depth=(\d))", l)
    lab = re.match(r"^(\.LBB(\S+)):", l) or re.match(r"^; %bb", l)
    if lab or (l.startswith(";") and "Loop Header" in l):
        if m and m.group(1):
            cur = ("BB" + m.group(1), m.group(2))
        elif m and m.group(3):
            lm = re.match(r"^\.LBB(\S+):", l)
            cur = ("BB" + lm.group(1), m.group(3)) if lm else cur
        elif lab:
            cur = None
        continue
    if cur and l.startswith("\t") and not l.strip().startswith(";") and not l.strip().startswith("."):
        loops.setdefault(cur, []).append(l.strip())
for (h, d), seg in loops.items():
    c = collections.Counter(x.split()[0] for x in seg)
    f64 = sum(v for k, v in c.items() if "f64" in k)
    salu = sum(v for k, v in c.items() if k.startswith("s_"))
    ds = sum(v for k, v in c.items() if k.startswith("ds_"))
    gl = sum(v for k, v in c.items() if k.startswith("global_"))
    dpp = sum(v for k, v in c.items() if "dpp" in k)
    cnd = sum(v for k, v in c.items() if "cndmask" in k)
    scr = sum(v for k, v in c.items() if k.startswith("scratch_"))
    acc = sum(v for k, v in c.items() if k.startswith("v_accvgpr"))
    lane = sum(v for k, v in c.items() if k.startswith(("v_readlane", "v_writelane")))
    vmw = sum(1 for x in seg if x.startswith("s_waitcnt") and "vmcnt" in x)
    print(f"{h:8s} depth {d} instr {len(seg):4d}  f64 {f64:3d}  dpp {dpp:3d}  cndmask {cnd:3d}  ds {ds:3d}  "
          f"global {gl:3d}  scratch {scr:3d}  accvgpr {acc:3d}  r/wlane {lane:3d}  vmcnt-waits {vmw:3d}  salu {salu:3d}  "
          f"other {len(seg) - f64 - dpp - cnd - ds - gl - salu - scr - acc - lane:3d}")
