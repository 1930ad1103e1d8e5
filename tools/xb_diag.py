#!/usr/bin/env python3
"""Diagnostic (not a test): per-iteration iterates of the lane kernel's interior-point (XB) variant on the exo
state-bounds case of tests/test_gpu_xbounds.py::test_exo_state_bounds_lane, for the library named by
MMPC_LIB_PATH, against the CPU oracle truncated at the same iteration count.

    MMPC_LIB_PATH=lib_var/<v>/libmmpc.so python tools/xb_diag.py OUT.npz

Per max_iter k = 1..K the solve is re-run from the cold start with max_iter = k; the first k at which an instance's
V leaves the oracle's (relative 1e-8) names the iteration whose step went wrong, and the per-iteration debug trace
(mmpc_debug_solve_trace: ||2g||, ||c||, J, |c|_1, alpha_max, alpha, mu, ||lam||) shows which quantity."""
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

N, h, B, K = 50, 0.002, 64, 8
INF = np.inf
out = sys.argv[1]
path = mmpc.write_model_json("/tmp/xb_diag_exo.json", "exo", 8, 4, 2000, N, model="exo_arm",
                             x_min=[-1e31] * 4 + [-0.3] * 4, x_max=[1e31] * 4 + [0.3] * 4)
xl = np.array([-INF] * 4 + [-0.3] * 4)
xu = np.array([INF] * 4 + [0.3] * 4)
x0, up, tr = o.synth(20250213, 0, B, N, h, model=o.EXO)
x0[:, 4:] = np.clip(x0[:, 4:], -0.25, 0.25)
w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
res = {}
first_bad = np.full(B, -1)
for k in range(1, K + 1):
    s = mmpc.Solver(path, max_iter=k)
    g = s.solve_batch_host(x0, up, tr, w)
    r = o.solve_batch(N, h, x0, up, tr, w, x_lb=xl, x_ub=xu, max_iter=k, model=o.EXO)
    rel = np.abs(g["V"] - r["V"]).max(1) / np.abs(r["V"]).max(1)
    newly = (rel > 1e-8) & (first_bad < 0)
    first_bad[newly] = k
    res[f"rel_{k}"] = rel
    res[f"iters_{k}"] = g["iters"]
    print(f"max_iter {k}: instances off the oracle (>1e-8): {int((rel > 1e-8).sum())}, max rel {rel.max():.3e}",
          flush=True)
    s.close()
# full solve with the per-iteration trace
s = mmpc.Solver(path, max_iter=60)
L = s._L
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
dev = dict(dtype=torch.float64, device="cuda")
tx0, tup, ttr, tw = (torch.tensor(a, **dev).contiguous() for a in (x0, up, tr, w))
V = torch.zeros((B, s.NV), **dev)
st = torch.zeros(B, dtype=torch.int32, device="cuda")
it = torch.zeros(B, dtype=torch.int32, device="cuda")
kk = torch.zeros(B, **dev)
trace = torch.zeros((B, 61, 8), **dev)
rc = L.mmpc_debug_solve_trace(s._h, B, tx0.data_ptr(), tup.data_ptr(), ttr.data_ptr(), tw.data_ptr(), 0,
                              V.data_ptr(), st.data_ptr(), it.data_ptr(), kk.data_ptr(), trace.data_ptr(), None)
assert rc == 0, L.mmpc_last_error()
torch.cuda.synchronize()
res.update(first_bad=first_bad, status=st.cpu().numpy(), iters=it.cpu().numpy(), trace=trace.cpu().numpy())
bad = np.where(first_bad > 0)[0]
print("instances leaving the oracle:", bad.tolist(), "at max_iter", first_bad[bad].tolist())
print("final status histogram:", np.bincount(st.cpu().numpy()))
for b in bad[:4]:
    print(f"instance {b} trace (||2g||, ||c||, J, |c|_1, amax, alpha, mu, ||lam||):")
    for i in range(min(int(it[b]) + 1, 12)):
        print("   ", i, " ".join(f"{v:.3e}" for v in trace[b, i].tolist()))
np.savez(out, **res)
