#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for the SQP kernel: per-dispatch averages of every counter, and the
HBM traffic per launch with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reads 1/2 of the
bytes of wide coalesced reads -> x2; WRITE_SIZE exact for 16-B stores; both in KB)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "sqp_wave_kernel"
vals = defaultdict(list)
for f in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if kname not in row.get("Kernel_Name", ""):
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
# counters are reported per dispatch (summed over dimensions by rocprofv3 v3 csv: one row per dispatch+counter)
summary = {k: sum(v) / len(v) for k, v in vals.items()}
res = {"kernel": kname, "per_dispatch_mean": summary}
if "FETCH_SIZE" in summary and "WRITE_SIZE" in summary:
    fetch_b = summary["FETCH_SIZE"] * 1024 * 2.0
    write_b = summary["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = fetch_b + write_b
    res["fetch_bytes_corrected"] = fetch_b
    res["write_bytes"] = write_b
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, "pmc_summary.json"), "w"), indent=1)
