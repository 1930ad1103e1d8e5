#!/usr/bin/env python3
"""SURVEY.md 8d cfg#5: cfg#3 (exo, B = 65536, N = 50, one MI355X) with the fp32 Riccati factor/solve and fp64
residuals, swept over the outer tolerance {1e-5, 1e-6, 1e-8} (tol_grad = tol, tol_defect = tol / 100, the
ratio of the defaults).  Reports % converged, mean/max SQP iterations, kernel time and
max_i ||V_i - V_i,fp64|| / ||V_i,fp64|| against the fp64-factor solve at the default tolerances.

    python tools/cfg5_sweep.py [--batch 65536] > profiles/r01/cfg5_sweep.json
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import mmpc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
B, N, nx, nu = a.batch, 50, 8, 4
path = mmpc.write_model_json(os.path.join(tempfile.mkdtemp(), "exo.json"), "exo", nx, nu, 2000, N, model="exo_arm")
f = dict(dtype=torch.float64, device="cuda")
x0 = torch.empty((B, nx), **f); up = torch.empty((B, nu), **f); tr = torch.empty((B, N, nx), **f)
w = torch.tensor([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4, **f)


def run(tol_grad, tol_defect, fp32):
    s = mmpc.Solver(path, tol_grad=tol_grad, tol_defect=tol_defect, factor_fp32=int(fp32), max_iter=50)
    s.reserve_workspace(B)
    s.synth(20250213, 0, B, x0, up, tr)
    V = torch.zeros((B, s.NV), **f)
    st = torch.zeros(B, dtype=torch.int32, device="cuda")
    it = torch.zeros(B, dtype=torch.int32, device="cuda")
    kkt = torch.zeros(B, **f)
    times = []
    for _ in range(a.reps):
        V.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s.solve_batch(B, x0, up, tr, w, V, st, it, kkt)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    s.close()
    return V.clone(), st.cpu().numpy(), it.cpu().numpy(), kkt.cpu().numpy(), float(np.median(times))


Vref, st_ref, it_ref, _, t_ref = run(1e-8, 1e-10, False)
out = {"workload": "cfg#5 = cfg#3 (exo, B=%d, N=50) with fp32 Riccati factor/solve, fp64 residuals" % B,
       "reference": {"factor": "fp64", "tol_grad": 1e-8, "tol_defect": 1e-10, "kernel_ms": t_ref,
                     "converged_pct": float((st_ref == 0).mean() * 100), "mean_iters": float(it_ref.mean())},
       "sweep": []}
nref = torch.linalg.vector_norm(Vref, dim=1)
for fp32 in (True, False):
    for tol in (1e-5, 1e-6, 1e-8):
        V, st, it, kkt, t = run(tol, tol / 100, fp32)
        rel = (torch.linalg.vector_norm(V - Vref, dim=1) / nref).cpu().numpy()
        out["sweep"].append({"factor": "fp32" if fp32 else "fp64", "tol_grad": tol, "tol_defect": tol / 100,
                             "converged_pct": float((st == 0).mean() * 100),
                             "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                             "mean_iters": float(it.mean()), "max_iters": int(it.max()), "kernel_ms": t,
                             "solves_per_s": B / (t * 1e-3), "max_rel_V_vs_fp64": float(rel.max()),
                             "median_rel_V_vs_fp64": float(np.median(rel))})
print(json.dumps(out, indent=1))
