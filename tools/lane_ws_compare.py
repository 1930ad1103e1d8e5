#!/usr/bin/env python3
"""Compare two tools/lane_ws_diag.py dumps (exo lane kernel, no bounds, B = 64, one 64-lane block) field by field, and
check in each build the step recursion dx_{k+1} = A_k dx_k + B_k du_k + c_k against the oracle's Jacobians at the
cold-start iterate (the max_iter = 0 dump's x_k, u_k) -- whether a build forms the step from its own du correctly.

    python3 tools/lane_ws_compare.py good.npz bad.npz"""
import sys

import numpy as np

sys.path.insert(0, "tests")
import oracle_lib as o  # noqa: E402

SS, NST, h, N = 116, 52, 0.002, 50
F = {"X": (0, 8), "U": (8, 4), "R": (12, 8), "C": (20, 8), "D": (28, 8), "DX": (36, 8), "DU": (44, 4), "KFF": (48, 4),
     "K": (52, 48), "X1": (104, 8), "U1": (112, 4)}
g, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for it in (0, 1, 2):
    wg = g[f"ws_{it}"][:NST * SS * 64].reshape(NST, SS, 64)
    wb = b[f"ws_{it}"][:NST * SS * 64].reshape(NST, SS, 64)
    print(f"max_iter {it}: fields that differ (stages 0..{N - 1}); V max |diff| "
          f"{np.abs(g[f'V_{it}'] - b[f'V_{it}']).max():.3e}")
    for name, (off, n) in F.items():
        d = np.abs(wg[:N, off:off + n] - wb[:N, off:off + n])
        st = np.where(d.max(axis=(1, 2)) > 0)[0]
        print(f"  {name:4s} max |diff| {d.max():.3e}  stages {st[:6].tolist()}{'...' if len(st) > 6 else ''} ({len(st)})")
W0 = g["ws_0"][:NST * SS * 64].reshape(NST, SS, 64)
for tag, z in (("first build", g), ("second build", b)):
    W = z["ws_1"][:NST * SS * 64].reshape(NST, SS, 64)
    worst = np.zeros(N)
    for lane in range(64):
        for k in range(N - 1):
            A, B, _ = o.exo_jac(W0[k, 0:8, lane], W0[k, 8:12, lane])
            dx, du = W[k, 36:44, lane], W[k, 44:48, lane]
            pred = dx + h * A @ dx + h * B @ du + W0[k, 20:28, lane]
            worst[k] = max(worst[k], np.abs(W[k + 1, 36:44, lane] - pred).max())
    print(f"{tag}: max |dx_(k+1) - (A dx_k + B du_k + c_k)| over lanes, stages 0..5: "
          + " ".join(f"{v:.1e}" for v in worst[:6]) + f"; stages 1..{N - 2} max {worst[1:N - 1].max():.2e}")

# the defect of the fused alpha = 1 trial (step sweep) against the oracle model at each build's own stored full-step
# point (X1, U1), and the d recursion built on it: which stage's trial evaluation is wrong
for tag, z in (("first build", g), ("second build", b)):
    W = z["ws_1"][:NST * SS * 64].reshape(NST, SS, 64)
    wc, wd = np.zeros(N), np.zeros(N)
    for lane in range(64):
        d = np.zeros(8)
        for k in range(N):
            x1, u1, xn = W[k, 104:112, lane], W[k, 112:116, lane], W[k + 1, 104:112, lane]
            A, _, xd = o.exo_jac(x1, u1)
            c = x1 + h * xd - xn
            wc[k] = max(wc[k], np.abs(W[k, 20:28, lane] - c).max())
            d = d + h * A @ d + c
            wd[k] = max(wd[k], np.abs(W[k + 1, 28:36, lane] - d).max())
    print(f"{tag}: max |c_k - (F(x1_k, u1_k) - x1_(k+1))| stages 0..5: " + " ".join(f"{v:.1e}" for v in wc[:6])
          + f"; stages 1..{N - 1} max {wc[1:].max():.2e}; d recursion max {wd.max():.2e}")
