import sys, numpy as np, torch
sys.path.insert(0, "mahi-mpc_amd"); sys.path.insert(0, "tests")
import mmpc, oracle_lib as o
W = np.array([10.0]*4 + [1.0]*4 + [1.0]*4 + [0.01]*4)
N = 50
path = mmpc.write_model_json("/tmp/exo_bd.json", "exo", 8, 4, 2000, N, model="exo_arm")
f = dict(dtype=torch.float64, device="cuda")
for B in (256, 4096, 65536):
    for how in ("host", "dev"):
        s = mmpc.Solver(path, kkt_solver=2, hessian=mmpc.HESSIAN_EXACT, init_states=mmpc.INIT_ZERO)
        if how == "host":
            x0, up, tr = o.synth(20250213, 0, B, N, 0.002, model=o.EXO)
            r = s.solve_batch_host(x0, up, tr, W)
            it = r["iters"]; V = r["V"]
        else:
            x0 = torch.empty((B, 8), **f); up = torch.empty((B, 4), **f); tr = torch.empty((B, N, 8), **f)
            s.synth(20250213, 0, B, x0, up, tr)
            V = torch.zeros((B, s.NV), **f); st = torch.zeros(B, dtype=torch.int32, device="cuda"); itt = torch.zeros(B, dtype=torch.int32, device="cuda")
            w = torch.tensor(W, **f)
            s.reserve_workspace(B)
            s.solve_batch(B, x0, up, tr, w, V, st, itt, None)
            torch.cuda.synchronize()
            it = itt.cpu().numpy(); V = V.cpu().numpy()
        print(B, how, "mean iters", it.mean(), "max", it.max(), "first 8", it[:8].tolist(), flush=True)
        s.close()
