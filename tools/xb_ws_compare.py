#!/usr/bin/env python3
"""Compare two tools/xb_ws_diag.py dumps field by field (exo XB lane-kernel workspace, B = 64, one 64-lane block):
max_iter 0 holds the first backward sweep's gains at the cold-start iterate, max_iter 1 the first step (DX, DU).
For the step it also checks dx_{k+1} = A_k dx_k + B_k du_k + c_k against the oracle's Jacobians at the stored
iterate (x_k, u_k), i.e. whether a build forms the step recursion correctly from its own du.

    python3 tools/xb_ws_compare.py good.npz bad.npz"""
import sys

import numpy as np

sys.path.insert(0, "tests")
import oracle_lib as o  # noqa: E402

SS, NST, h = 160, 52, 0.002
F = {"X": (0, 8), "U": (8, 4), "R": (12, 8), "C": (20, 8), "D": (28, 8), "DX": (36, 8), "DU": (44, 4), "KFF": (48, 4),
     "K": (52, 48), "ZL": (100, 12), "ZU": (112, 12), "SG": (124, 12), "BB": (136, 12), "ZG": (148, 12)}
g, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for it in (0, 1):
    wg, wb = g[f"ws_{it}"].reshape(NST, SS, 64), b[f"ws_{it}"].reshape(NST, SS, 64)
    print(f"max_iter {it}: fields that differ (stages 0..49)")
    for name, (off, n) in F.items():
        d = np.abs(wg[:50, off:off + n] - wb[:50, off:off + n])
        st = np.where(d.max(axis=(1, 2)) > 0)[0]
        print(f"  {name:4s} max |diff| {d.max():.3e}  stages {st[:6].tolist()}{'...' if len(st) > 6 else ''} ({len(st)})")
W0 = g["ws_0"].reshape(NST, SS, 64)
for tag, W in (("first build", g["ws_1"].reshape(NST, SS, 64)), ("second build", b["ws_1"].reshape(NST, SS, 64))):
    worst = np.zeros(50)
    for lane in range(64):
        for k in range(49):
            A, B, _ = o.exo_jac(W0[k, 0:8, lane], W0[k, 8:12, lane])
            dx, du = W[k, 36:44, lane], W[k, 44:48, lane]
            pred = dx + h * A @ dx + h * B @ du + W0[k, 20:28, lane]
            worst[k] = max(worst[k], np.abs(W[k + 1, 36:44, lane] - pred).max())
    print(f"{tag}: max |dx_(k+1) - (A dx_k + B du_k + c_k)| over lanes, stages 0..5: "
          + " ".join(f"{v:.1e}" for v in worst[:6]) + f"; stages 1..48 max {worst[1:49].max():.2e}")
