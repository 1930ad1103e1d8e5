#!/usr/bin/env python3
"""Diagnostic (not a test): per-instance, per-iteration SQP trace of a bench workload (mmpc_debug_solve_trace: the
same kernels with the trace written), saved as an .npz for offline analysis -- iterations, status and the trace
[B][max_iter+1][8] = (||2g||, ||c||, J, |c|_1, dJ, alpha, mu, ||lam||) as the lane / group kernels record it.

    python tools/trace_dump.py --config cfg3 --batch 16384 --out gpurun_out/trace_cfg3.npz"""
import argparse
import ctypes as C
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
ap.add_argument("--max-iter", type=int, default=30)
ap.add_argument("--out", required=True)
a = ap.parse_args()
cfg = bench.CONFIGS[a.config]
nx, nu, N, B = cfg["nx"], cfg["nu"], cfg["N"], a.batch or cfg["B"]
d = tempfile.mkdtemp()
s = mmpc.Solver(mmpc.write_model_json(os.path.join(d, "m.json"), cfg["model"], nx, nu, 2000, N, model=cfg["model"]),
                max_iter=a.max_iter, init_states=mmpc.INIT_ZERO)
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
trace = torch.zeros((B, a.max_iter + 1, 8), **f64)
L = s._L
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
rc = L.mmpc_debug_solve_trace(s._h, B, x0.data_ptr(), up.data_ptr(), tr.data_ptr(), w.data_ptr(), 0, V.data_ptr(),
                              st.data_ptr(), it.data_ptr(), kk.data_ptr(), trace.data_ptr(), None)
assert rc == 0, L.mmpc_last_error()
torch.cuda.synchronize()
np.savez_compressed(a.out, iters=it.cpu().numpy(), status=st.cpu().numpy(), trace=trace.cpu().numpy(),
                    kkt_solver=s.kkt_solver_for(B))
print(a.out, "mean iters", float(it.float().mean()), "max", int(it.max()))
