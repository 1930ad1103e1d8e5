#!/usr/bin/env python3
"""Per-kernel ISA statistics from a device assembly file (hipcc --cuda-device-only -S): register and spill
metadata (.vgpr_count, .agpr_count, .vgpr_spill_count, .sgpr_spill_count, private segment / scratch bytes),
instruction counts (scratch loads/stores, global loads/stores, vmcnt waits) -- used to compare builds of one kernel
without a GPU.

    python3 tools/isa_kernel_stats.py <file.s> <mangled-name-substring> [more .s files ...]
"""
import re
import sys


def kernel_body(text, name):
    m = re.search(r"^(%s[^\s:]*):" % re.escape(name), text, re.M)
    if not m:
        raise SystemExit(f"{name}: not found")
    sym = m.group(1)
    start = m.end()
    end = text.index(".Lfunc_end", start)
    return sym, text[start:end]


def metadata(text, sym):
    i = text.index(f".name:           {sym}")
    blk = text[text.rfind("- .agpr_count", 0, i):i + 4000]
    out = {}
    for k in ("agpr_count", "vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
              "private_segment_fixed_size", "group_segment_fixed_size"):
        mm = re.search(r"\.%s:\s+(\d+)" % k, blk)
        out[k] = int(mm.group(1)) if mm else None
    return out


def stats(body):
    lines = [ln.strip() for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", ".", "//"))]
    ins = [ln for ln in lines if not ln.endswith(":")]
    c = lambda p: sum(1 for ln in ins if re.match(p, ln))  # noqa: E731
    return {"instructions": len(ins), "scratch_load": c(r"scratch_load"), "scratch_store": c(r"scratch_store"),
            "buffer_spill": c(r"buffer_(load|store).*off.*offset"), "global_load": c(r"global_load"),
            "global_store": c(r"global_store"), "flat": c(r"flat_"), "vmcnt0": c(r"s_waitcnt vmcnt\(0\)"),
            "waitcnt": c(r"s_waitcnt"), "accvgpr_moves": c(r"v_accvgpr_(read|write)"),
            "exec_writes": c(r"s_(and|or|xor|mov|andn2|orn2)_(saveexec_)?b64 exec")}


if __name__ == "__main__":
    name = sys.argv[2]
    files = [sys.argv[1]] + sys.argv[3:]
    for f in files:
        text = open(f).read()
        sym, body = kernel_body(text, name)
        md = metadata(text, sym)
        print(f, sym)
        print("  metadata", md)
        print("  isa     ", stats(body))
