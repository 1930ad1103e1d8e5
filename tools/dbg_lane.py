"""Debug: compare Riccati-kernel iterates with the oracle after k SQP iterations (GPU box)."""
import json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import mmpc, oracle_lib as o
import tempfile
td = tempfile.mkdtemp()
H = 0.002
g = json.load(open(os.path.join(REPO, "tests/golden/exo_golden.json")))
W = np.array(g["weights"])
c = [c for c in g["cases"] if c["N"] == 20][0]
cases = [("exo20", o.EXO, 20, np.array([c["x0"]]), np.array([c["u_prev"]]), np.array([c["traj"]]), W)]
x0, up, tr = o.synth(20250213, 0, 4, 30, H)
cases.append(("2link30", o.TWO_LINK, 30, x0, up, tr, np.array([10.0, 1, 5, 5, 5, 5, .01, .01])))
for name, model, N, x0, up, tr, w in cases:
    nx, nu = o.DIMS[model]
    p = mmpc.write_model_json(os.path.join(td, name + ".json"), name, nx, nu, 2000, N)
    for mi in range(0, 5):
        s = mmpc.Solver(p, max_iter=mi, kkt_solver=mmpc.KKT_RICCATI)
        r = s.solve_batch_host(x0, up, tr, w)
        q = o.solve_batch(N, H, x0, up, tr, w, max_iter=mi, model=model)
        d = np.abs(r["V"] - q["V"])
        i = int(d[0].argmax())
        print(name, "max_iter", mi, "gpu", r["status"][0], r["iters"][0], "%.3e" % r["kkt"][0], "orc", q["status"][0],
              q["iters"][0], "%.3e" % q["kkt"][0], "maxdiff %.3e at %d (stage %d, comp %d)" % (d[0].max(), i, i // (nx + nu), i % (nx + nu)))
        s.close()
