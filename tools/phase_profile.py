#!/usr/bin/env python3
"""Per-phase cycle breakdown of the SQP kernel (diagnostic build lib/libmmpc_timing.so).

    MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so python tools/phase_profile.py [--batch 4096]

Stamps serialise the instruction stream, so read the SHARES, not the absolute time."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import mmpc  # noqa: E402

NAMES = ["load", "stage_eval", "d_forward", "adjoint+grad+check", "lyapunov", "hessian", "gauss_jordan",
         "dx_forward", "line_search", "writeback"]
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--horizon", type=int, default=30)
a = ap.parse_args()
B, N = a.batch, a.horizon
L = mmpc.lib()
L.mmpc_debug_phase_cycles.argtypes = [C.c_void_p, C.c_int]
path = mmpc.write_model_json("/tmp/mmpc_phase.json", "nonlinear_double_pendulum", 4, 2, 2000, N)
s = mmpc.Solver(path)
f = dict(dtype=torch.float64, device="cuda")
x0 = torch.empty((B, 4), **f); up = torch.empty((B, 2), **f); tr = torch.empty((B, N, 4), **f)
s.synth(20250213, 0, B, x0, up, tr)
w = torch.tensor([10, 1, 5, 5, 5, 5, .01, .01], **f)
V = torch.zeros((B, s.NV), **f)
it = torch.zeros(B, dtype=torch.int32, device="cuda")
s.solve_batch(B, x0, up, tr, w, V, None, it, None)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 16)()
L.mmpc_debug_phase_cycles(buf, 1)
V.zero_()
s.solve_batch(B, x0, up, tr, w, V, None, it, None)
torch.cuda.synchronize()
L.mmpc_debug_phase_cycles(buf, 1)
cyc = np.array(buf[:10], dtype=np.float64)
waves = buf[15]
iters = it.cpu().numpy()
out = {"waves": int(waves), "mean_iters": float(iters.mean()),
       "cycles_per_wave": float(cyc.sum() / waves),
       "per_phase_cycles_per_wave_iteration": {n: float(c / waves / (iters.mean() + 1)) for n, c in zip(NAMES, cyc)},
       "share": {n: float(c / cyc.sum()) for n, c in zip(NAMES, cyc)}}
print(json.dumps(out, indent=1))
