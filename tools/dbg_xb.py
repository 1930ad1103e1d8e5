"""Debug: per-iteration trace of the XB (state-bounded) group kernel vs the oracle's iteration counts."""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import mmpc  # noqa: E402
import oracle_lib as O  # noqa: E402

N, h, B = 30, 0.002, 128
inf = np.inf
xl, xu = np.array([-inf, -inf, -1.5, -1.5]), np.array([inf, inf, 1.5, 1.5])
path = mmpc.write_model_json("/tmp/dbgxb.json", "dbgxb", 4, 2, 2000, N)
s = mmpc.Solver(path, max_iter=100, kkt_solver=mmpc.KKT_RICCATI_GROUP)
s.set_state_bounds(xl, xu)
x0, up, tr = O.synth(20250213, 0, B, N, h)
w = np.array([10.0, 1, 5, 5, 5, 5, 0.01, 0.01])
o = O.solve_batch(N, h, x0, up, tr, w, x_lb=xl, x_ub=xu, max_iter=100)
L = s._L
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
f = dict(dtype=torch.float64, device="cuda")
t = lambda a: torch.tensor(a, **f)  # noqa: E731
X0, UP, TR, W = t(x0), t(up), t(tr), t(w)
V = torch.zeros((B, s.NV), **f)
st = torch.zeros(B, dtype=torch.int32, device="cuda")
it = torch.zeros(B, dtype=torch.int32, device="cuda")
kk = torch.zeros(B, **f)
trace = torch.full((B, 101, 8), float("nan"), **f)
rc = L.mmpc_debug_solve_trace(s._h, B, X0.data_ptr(), UP.data_ptr(), TR.data_ptr(), W.data_ptr(), 0, V.data_ptr(),
                              st.data_ptr(), it.data_ptr(), kk.data_ptr(), trace.data_ptr(), None)
torch.cuda.synchronize()
print("rc", rc, "gpu status", np.bincount(st.cpu().numpy()), "oracle", np.bincount(o["status"]))
st, it, trace = st.cpu().numpy(), it.cpu().numpy(), trace.cpu().numpy()
for b in np.where(st != 0)[0][:4]:
    print("instance", b, "gpu iters", it[b], "oracle iters", o["iters"][b])
    for i in range(it[b] + 1):
        print("  it %2d gmax %.2e cmax %.2e J %.4e cmpl %.2e amax %.3e alpha %.3e mub %.2e lmax %.2e" % (i, *trace[b, i]))
