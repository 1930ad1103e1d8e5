"""Debug: iteration-0 quantities of the Riccati kernel (trace) vs a numpy replay with oracle Jacobians."""
import ctypes as C, json, os, sys, tempfile
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch, mmpc, oracle_lib as o
L = mmpc.lib()
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
g = json.load(open(os.path.join(REPO, "tests/golden/exo_golden.json")))
W = np.array(g["weights"]); h = 0.002
c = [c for c in g["cases"] if c["N"] == 20][0]
def replay(N, x0, up, tr):
    Q, R, Rm = W[:8], W[8:12], W[12:16]
    X = np.zeros((N + 1, 8)); X[0] = x0; U = np.zeros((N, 4))
    A = []; B = []; F = []
    for k in range(N):
        a, b, xd = o.exo_jac(X[k], U[k]); A.append(np.eye(8) + h * a); B.append(h * b); F.append(X[k] + h * xd)
    cc = np.array([F[k] - X[k + 1] for k in range(N)])
    d = np.zeros((N + 1, 8))
    for k in range(N): d[k + 1] = A[k] @ d[k] + cc[k]
    J0 = sum(((F[k] - tr[k]) ** 2 * Q).sum() for k in range(N)) + sum((((U[k] - (up if k == 0 else U[k - 1])) ** 2) * R).sum() for k in range(N))
    lam = Q * (d[N] + X[N] - tr[N - 1]); gmax = 0; lmax = np.abs(lam).max()
    for k in range(N - 1, -1, -1):
        um = up if k == 0 else U[k - 1]
        gk = B[k].T @ lam + R * (U[k] - um) + Rm * U[k]
        if k + 1 < N: gk -= R * (U[k + 1] - U[k])
        gmax = max(gmax, np.abs(2 * gk).max())
        if k >= 1:
            lam = Q * (d[k] + X[k] - tr[k - 1]) + A[k].T @ lam; lmax = max(lmax, np.abs(lam).max())
    return dict(gmax=gmax, cmax=np.abs(cc).max(), J0=J0, c1=np.abs(cc).sum(), lmax=lmax)
td = tempfile.mkdtemp()
for N in (1, 2, 3, 20):
    x0 = np.array(c["x0"]); up = np.array(c["u_prev"]); tr = np.array(c["traj"])[:N]
    p = mmpc.write_model_json(os.path.join(td, f"e{N}.json"), "e", 8, 4, 2000, N)
    s = mmpc.Solver(p, max_iter=0, kkt_solver=mmpc.KKT_RICCATI)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")
    x0d, upd, trd, wd = t(x0[None]), t(up[None]), t(tr[None]), t(W)
    V = torch.zeros((1, s.NV), dtype=torch.float64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda"); it = torch.zeros(1, dtype=torch.int32, device="cuda")
    kk = torch.zeros(1, dtype=torch.float64, device="cuda"); trc = torch.zeros((1, 1, 8), dtype=torch.float64, device="cuda")
    rc = L.mmpc_debug_solve_trace(s._h, 1, x0d.data_ptr(), upd.data_ptr(), trd.data_ptr(), wd.data_ptr(), 0, V.data_ptr(),
                                  st.data_ptr(), it.data_ptr(), kk.data_ptr(), trc.data_ptr(), None)
    torch.cuda.synchronize()
    tv = trc.cpu().numpy()[0, 0]
    ref = replay(N, x0, up, tr)
    print(N, "rc", rc, "gpu gmax %.10e cmax %.10e J0 %.10e c1 %.10e lmax %.10e" % (tv[0], tv[1], tv[2], tv[3], tv[7]))
    print(N, "      ref gmax %.10e cmax %.10e J0 %.10e c1 %.10e lmax %.10e" % (ref["gmax"], ref["cmax"], ref["J0"], ref["c1"], ref["lmax"]))
