#!/usr/bin/env python3
"""Diagnostic (not a test): solve one bench workload with the library MMPC_LIB_PATH names and save V*, status and
iterations (.npz), so that two builds can be compared bit for bit (same iterates = a pure code-generation change).

    MMPC_LIB_PATH=lib_var/x/libmmpc.so python tools/v_dump.py --config cfg3 --out a.npz [--hessian exact]
    python tools/v_dump.py --compare a.npz b.npz"""
import argparse
import os
import sys

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3")
ap.add_argument("--batch", type=int, default=None)
ap.add_argument("--hessian", choices=["auto", "gauss_newton", "exact"], default="auto")
ap.add_argument("--u-bound", type=float, default=None)
ap.add_argument("--x-bound", type=float, default=None)
ap.add_argument("--kkt", choices=["auto", "riccati", "group"], default="auto")
ap.add_argument("--out")
ap.add_argument("--compare", nargs=2)
a = ap.parse_args()

if a.compare:
    x, y = (np.load(f) for f in a.compare)
    same = {k: bool(np.array_equal(x[k], y[k])) for k in ("V", "status", "iters")}
    d = np.abs(x["V"] - y["V"]).max()
    print(f"{a.compare[0]} vs {a.compare[1]}: bitwise equal {same}, max |dV| {d:.3e}, "
          f"iterations {x['iters'].mean():.4f} / {y['iters'].mean():.4f}")
    sys.exit(0 if all(same.values()) else 1)

import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import bench  # noqa: E402
import mmpc  # noqa: E402

cfg = bench.CONFIGS[a.config]
nx, nu, N = cfg["nx"], cfg["nu"], cfg["N"]
B = a.batch or cfg["B"]
model = "exo_arm" if nx == 8 else "two_link_arm"
path = mmpc.write_model_json(f"/tmp/v_dump_{a.config}.json", model, nx, nu, 2000, N, model=model)
hess = {"auto": 0, "gauss_newton": mmpc.HESSIAN_GAUSS_NEWTON, "exact": mmpc.HESSIAN_EXACT}[a.hessian]
s = mmpc.Solver(path, hessian=hess, init_states=mmpc.INIT_ZERO, factor_fp32=1 if cfg.get("fp32") else 0,
                kkt_solver={"auto": 0, "riccati": 2, "group": 3}[a.kkt])
if a.x_bound is not None:
    s.set_state_bounds([-np.inf] * (nx // 2) + [-a.x_bound] * (nx // 2), [np.inf] * (nx // 2) + [a.x_bound] * (nx // 2))
f = dict(dtype=torch.float64, device="cuda")
x0 = torch.empty((B, nx), **f)
up = torch.empty((B, nu), **f)
tr = torch.empty((B, N, nx), **f)
s.synth(bench.SEED, 0, B, x0, up, tr)
w = torch.tensor(cfg["weights"], **f)
lb = None if a.u_bound is None else torch.full((nu,), -a.u_bound, **f)
ub = None if a.u_bound is None else torch.full((nu,), a.u_bound, **f)
V = torch.zeros((B, s.NV), **f)
st = torch.zeros(B, dtype=torch.int32, device="cuda")
it = torch.zeros(B, dtype=torch.int32, device="cuda")
s.solve_batch(B, x0, up, tr, w, V, st, it, None, u_lb=lb, u_ub=ub)
torch.cuda.synchronize()
np.savez(a.out, V=V.cpu().numpy(), status=st.cpu().numpy(), iters=it.cpu().numpy())
print(f"{a.out}: {a.config} B={B} converged {(st == 0).sum().item()}, iterations {it.float().mean().item():.4f}")
