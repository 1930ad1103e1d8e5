#!/usr/bin/env python3
"""Summarise a tools/pmc.sh run for one kernel: per-dispatch means of every counter, the undisturbed mean
kernel duration (the kernel-trace-only pass), HBM traffic per launch with the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE counts 1/2 of the bytes of wide coalesced reads -> x2; WRITE_SIZE exact for
16-B stores; both in KB), and the issued FP64 VALU rate against the FP64 vector peak.

    python3 tools/pmc_summary.py <pmc out dir> <kernel name substring> [--traffic-json profiles/traffic_latest.json
                                 --key cfg2:sqp_group_kernel<TwoLinkArm> --batch 4096 --horizon 30 --source ...]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

FP64_PEAK_TFLOPS = 78.6

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("kernel")
ap.add_argument("--traffic-json")
ap.add_argument("--key")
ap.add_argument("--batch", type=int)
ap.add_argument("--horizon", type=int)
ap.add_argument("--source")
ap.add_argument("--lib-sha256", help="sha256 of the library the PMC passes loaded (bench.py merges by it)")
a = ap.parse_args()

vals = defaultdict(list)
for f in glob.glob(os.path.join(a.out, "*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if a.kernel not in row.get("Kernel_Name", ""):
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
# rocprofv3 csv: one row per (dispatch, counter), already summed over the device
summary = {k: sum(v) / len(v) for k, v in vals.items()}
res = {"kernel": a.kernel, "per_dispatch_mean": summary, "lib_sha256": a.lib_sha256}
durs = []
for f in glob.glob(os.path.join(a.out, "trace", "**", "*kernel_trace.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if a.kernel in row.get("Kernel_Name", ""):
            durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
if durs:
    res["kernel_ms_trace_pass"] = sum(durs) / len(durs) / 1e6
    res["dispatches_trace_pass"] = len(durs)
if "FETCH_SIZE" in summary and "WRITE_SIZE" in summary:
    fetch_b = summary["FETCH_SIZE"] * 1024 * 2.0
    write_b = summary["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = fetch_b + write_b
    res["fetch_bytes_corrected"] = fetch_b
    res["write_bytes"] = write_b
    if durs:
        res["hbm_gbs"] = res["hbm_bytes_per_launch"] / (res["kernel_ms_trace_pass"] * 1e-3) / 1e9
if "SQ_INSTS_VALU_FMA_F64" in summary:
    # wave-level instruction counts x 64 lanes (issued lane slots; an FMA = 2 flops)
    fl = 64 * (2 * summary["SQ_INSTS_VALU_FMA_F64"] + summary.get("SQ_INSTS_VALU_MUL_F64", 0)
               + summary.get("SQ_INSTS_VALU_ADD_F64", 0))
    res["fp64_valu_flops_issued_per_launch"] = fl
    if durs:
        tf = fl / (res["kernel_ms_trace_pass"] * 1e-3) / 1e12
        res["fp64_valu_tflops_issued"] = tf
        res["fp64_valu_frac_of_peak"] = tf / FP64_PEAK_TFLOPS
mf = {k: v for k, v in summary.items() if "MFMA" in k}
res["mfma_counters"] = mf if mf else "no MFMA counter available in this rocprofv3 build"
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(a.out, "pmc_summary.json"), "w"), indent=1)

if a.traffic_json and a.key and "hbm_bytes_per_launch" in res:
    tj = json.load(open(a.traffic_json)) if os.path.exists(a.traffic_json) else {}
    tj[a.key] = {"batch": a.batch, "horizon": a.horizon, "kernel": a.key.split(":", 1)[1],
                 "hbm_bytes_per_launch": res["hbm_bytes_per_launch"],
                 "kernel_ms_at_measurement": res.get("kernel_ms_trace_pass"),
                 "fp64_valu_flops_issued_per_launch": res.get("fp64_valu_flops_issued_per_launch"),
                 "mfma_counters": res["mfma_counters"],
                 "lds_bank_conflict_cycles": summary.get("SQ_LDS_BANK_CONFLICT"),
                 "valu_active_frac": (summary["SQ_ACTIVE_INST_VALU"] / summary["SQ_WAVE_CYCLES"]
                                      if summary.get("SQ_WAVE_CYCLES") and "SQ_ACTIVE_INST_VALU" in summary else None),
                 "source": a.source,
                 "lib_sha256": a.lib_sha256}
    json.dump(tj, open(a.traffic_json, "w"), indent=1)
