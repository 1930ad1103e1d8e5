#!/usr/bin/env python3
"""Diagnostic (not a test): state-bounded exo solves (|qdot| <= 0.3) on the 16-lane and lane kernels with both
Hessians against the oracle's interior point: iteration agreement and max relative V* difference per combination."""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import mmpc  # noqa: E402
import oracle_lib as oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 70
d = tempfile.mkdtemp()
p = mmpc.write_model_json(os.path.join(d, "exo.json"), "exo", 8, 4, 2000, N, model="exo_arm")
xl = np.array([-np.inf] * 4 + [-0.3] * 4)
xu = np.array([np.inf] * 4 + [0.3] * 4)
x0, up, tr = oracle.synth(20250213, 0, B, N, 0.002, model=oracle.EXO)
x0[:, 4:] = np.clip(x0[:, 4:], -0.25, 0.25)
w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
orc = {}
for hess in (1, 2):
    orc[hess] = oracle.solve_batch(N, 0.002, x0, up, tr, w, x_lb=xl, x_ub=xu, max_iter=100, model=oracle.EXO,
                                   hessian=oracle.HESS_EXACT if hess == 2 else oracle.HESS_GAUSS_NEWTON)
for ks in (3, 2):
    for hess in (1, 2):
        s = mmpc.Solver(p, max_iter=100, kkt_solver=ks, hessian=hess)
        s.set_state_bounds(xl, xu)
        g = s.solve_batch_host(x0, up, tr, w)
        o = orc[hess]
        same = g["iters"] == o["iters"]
        rel = np.abs(g["V"] - o["V"]).max(1) / np.abs(o["V"]).max(1)
        print(f"N={N} B={B} kkt={ks} hess={hess}: status {np.bincount(g['status']).tolist()} oracle "
              f"{np.bincount(o['status']).tolist()}, same iters {int(same.sum())}/{B}, max rel V (same) "
              f"{rel[same].max() if same.any() else -1:.2e}, max rel V {rel.max():.2e}; first diffs "
              f"{g['iters'][~same][:6].tolist()} vs {o['iters'][~same][:6].tolist()}")
        s.close()
