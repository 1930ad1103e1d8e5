#!/usr/bin/env python3
"""Diagnostic (not a test): the exo lane kernel's per-stage workspace (cfg#3 kernel, no bounds) after max_iter = 0
(the first backward sweep's gains at the cold-start iterate) and max_iter = 1 (the first step dx, du), for the library
named by MMPC_LIB_PATH -- to compare two builds field by field (tools/lane_ws_compare.py), as tools/xb_ws_diag.py
does for the state-bounded instantiation.

    MMPC_LIB_PATH=... python tools/lane_ws_diag.py OUT.npz"""
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
path = mmpc.write_model_json("/tmp/lane_ws_exo.json", "exo", 8, 4, 2000, N, model="exo_arm")
x0, up, tr = o.synth(20250213, 0, B, N, h, model=o.EXO)
w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
dev = dict(dtype=torch.float64, device="cuda")
res = {}
hip = C.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
for k in (0, 1, 2):
    s = mmpc.Solver(path, max_iter=k, kkt_solver=mmpc.KKT_RICCATI, init_states=2)
    L = s._L
    L.mmpc_debug_workspace.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
    tx0, tup, ttr, tw = (torch.tensor(a, **dev).contiguous() for a in (x0, up, tr, w))
    V = torch.zeros((B, s.NV), **dev)
    it = torch.zeros(B, dtype=torch.int32, device="cuda")
    st = torch.zeros(B, dtype=torch.int32, device="cuda")
    s.solve_batch(B, tx0, tup, ttr, tw, V, st, it)
    torch.cuda.synchronize()
    ptr, nb = C.c_void_p(), C.c_uint64()
    assert L.mmpc_debug_workspace(s._h, C.byref(ptr), C.byref(nb)) == 0
    host = np.empty(nb.value // 8, dtype=np.float64)
    assert hip.hipMemcpy(host.ctypes.data, ptr, nb.value, 2) == 0   # hipMemcpyDeviceToHost
    res[f"ws_{k}"] = host
    res[f"V_{k}"] = V.cpu().numpy()
    s.close()
np.savez(sys.argv[1], **res)
print("saved", {k: v.shape for k, v in res.items()})
