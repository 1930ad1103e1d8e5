#!/usr/bin/env python3
"""Diagnostic (not a test): how often the accepted step is the full step (alpha = 1) in the bench workloads, per
instance-iteration and per WAVE-iteration (a lane-per-instance wave skips a pass only when none of its active lanes
needs it).  Uses mmpc_debug_solve_trace (the same kernels, with the per-iteration trace) on the bench's synthetic
inputs.

    python tools/alpha_stats.py [--config cfg3|cfg2] [--batch B]"""
import argparse
import ctypes as C
import json
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import mmpc  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3")
ap.add_argument("--batch", type=int, default=None)
a = ap.parse_args()
cfg = bench.CONFIGS[a.config]
nx, nu, N, B = cfg["nx"], cfg["nu"], cfg["N"], a.batch or cfg["B"]
d = tempfile.mkdtemp()
s = mmpc.Solver(mmpc.write_model_json(os.path.join(d, "m.json"), cfg["model"], nx, nu, 2000, N, model=cfg["model"]),
                max_iter=60)
f64 = dict(dtype=torch.float64, device="cuda")
x0 = torch.empty((B, nx), **f64)
up = torch.empty((B, nu), **f64)
tr = torch.empty((B, N, nx), **f64)
s.synth(bench.SEED, 0, B, x0, up, tr)
w = torch.tensor(cfg["weights"], **f64)
V = torch.zeros((B, s.NV), **f64)
st = torch.zeros(B, dtype=torch.int32, device="cuda")
it = torch.zeros(B, dtype=torch.int32, device="cuda")
kk = torch.zeros(B, **f64)
trace = torch.zeros((B, 61, 8), **f64)
L = s._L
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
rc = L.mmpc_debug_solve_trace(s._h, B, x0.data_ptr(), up.data_ptr(), tr.data_ptr(), w.data_ptr(), 0, V.data_ptr(),
                              st.data_ptr(), it.data_ptr(), kk.data_ptr(), trace.data_ptr(), None)
assert rc == 0, L.mmpc_last_error()
torch.cuda.synchronize()
iters = it.cpu().numpy()
alpha = trace[:, :, 5].cpu().numpy()
K = int(iters.max())
steps = np.arange(61)[None, :] < iters[:, None]          # (instance, iteration) pairs that took a step
full = steps & (alpha == 1.0)
per_wave = {}
lanes = 64 if s.kkt_solver_for(B) == 2 else 4        # instances per wave: lane kernel 64, group kernel 4
W = B // lanes
sw = steps[:W * lanes].reshape(W, lanes, 61)
fw = full[:W * lanes].reshape(W, lanes, 61)
active = sw.any(1)                                        # wave-iterations with any lane stepping
all_full = (sw == fw).all(1) & active                    # ... in which every stepping lane took alpha = 1
res = {
    "config": a.config, "batch": B, "kkt_solver": s.kkt_solver_for(B), "instances_per_wave": lanes,
    "mean_iters": float(iters.mean()), "max_iters": K,
    "instance_iterations": int(steps.sum()), "full_step_fraction": float(full.sum() / steps.sum()),
    "full_step_fraction_by_iteration": [float(full[:, k].sum() / max(1, steps[:, k].sum())) for k in range(K)],
    "wave_iterations": int(active.sum()), "wave_iterations_all_full": int(all_full.sum()),
    "wave_all_full_fraction_by_iteration": [float(all_full[:, k].sum() / max(1, active[:, k].sum())) for k in range(K)],
}
print(json.dumps(res, indent=1))
