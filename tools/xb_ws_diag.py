#!/usr/bin/env python3
"""Diagnostic (not a test): the lane kernel's per-stage workspace after an interior-point (XB) exo solve with
max_iter = 0 (the gains [K_k | kff_k] of the first backward sweep, at the cold-start iterate) and max_iter = 1 (the
first step dx, du), for the library named by MMPC_LIB_PATH -- to compare two builds field by field.

    MMPC_LIB_PATH=... python tools/xb_ws_diag.py OUT.npz"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import mmpc  # noqa: E402
import oracle_lib as o  # noqa: E402

N, h, B = 50, 0.002, 64
path = mmpc.write_model_json("/tmp/xb_ws_exo.json", "exo", 8, 4, 2000, N, model="exo_arm",
                             x_min=[-1e31] * 4 + [-0.3] * 4, x_max=[1e31] * 4 + [0.3] * 4)
x0, up, tr = o.synth(20250213, 0, B, N, h, model=o.EXO)
x0[:, 4:] = np.clip(x0[:, 4:], -0.25, 0.25)
w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
dev = dict(dtype=torch.float64, device="cuda")
res = {}
for k in (0, 1):
    s = mmpc.Solver(path, max_iter=k)
    L = s._L
    L.mmpc_debug_workspace.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
    tx0, tup, ttr, tw = (torch.tensor(a, **dev).contiguous() for a in (x0, up, tr, w))
    V = torch.zeros((B, s.NV), **dev)
    s.solve_batch(B, tx0, tup, ttr, tw, V)
    torch.cuda.synchronize()
    ptr, nb = C.c_void_p(), C.c_uint64()
    assert L.mmpc_debug_workspace(s._h, C.byref(ptr), C.byref(nb)) == 0
    host = np.empty(nb.value // 8, dtype=np.float64)
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(host.ctypes.data, ptr, nb.value, 2) == 0   # hipMemcpyDeviceToHost
    res[f"ws_{k}"] = host
    res[f"V_{k}"] = V.cpu().numpy()
    s.close()
np.savez(sys.argv[1], **res)
print("saved", {k: v.shape for k, v in res.items()})
