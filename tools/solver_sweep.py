#!/usr/bin/env python3
"""AUTO-policy sweep: per-solve time of each KKT solver over batch sizes and horizons (2-link arm, cfg#2
generator, cold start), 2 warmup + 10 timed launches each; writes gpurun_out/solver_sweep.json."""
import json, os, sys, tempfile
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import mmpc  # noqa: E402
nx, nu = 4, 2
res = []
for N in [int(v) for v in os.environ.get("HORIZONS", "20,30,60").split(",")]:
    d = tempfile.mkdtemp()
    path = mmpc.write_model_json(os.path.join(d, "m.json"), "m", nx, nu, 2000, N, model="two_link_arm")
    solvers = {k: mmpc.Solver(path, kkt_solver=v) for k, v in
               (("condensed", mmpc.KKT_CONDENSED), ("group", mmpc.KKT_RICCATI_GROUP), ("lane", mmpc.KKT_RICCATI))
               if not (k == "condensed" and N * nu > 64)}
    for B in [int(v) for v in os.environ.get("BATCHES", "64,512,1024,2048,4096,8192,16384").split(",")]:
        f = dict(dtype=torch.float64, device="cuda")
        x0 = torch.empty((B, nx), **f); up = torch.empty((B, nu), **f); tr = torch.empty((B, N, nx), **f)
        V = torch.zeros((B, N * 6 + 4), **f)
        w = torch.tensor([10, 1, 5, 5, 5, 5, .01, .01], **f)
        row = dict(N=N, B=B)
        for name, s in solvers.items():
            s.reserve_workspace(B)
            s.synth(20250213, 0, B, x0, up, tr)
            ev = []
            for rep in range(12):
                V.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); s.solve_batch(B, x0, up, tr, w, V, None, None, None); e1.record()
                ev.append((e0, e1))
            torch.cuda.synchronize()
            row[name] = sum(a.elapsed_time(b) for a, b in ev[2:]) / 10
        row["auto_choice"] = mmpc.Solver(path).kkt_solver_for(B)
        res.append(row)
        print(row, flush=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "solver_sweep.json"), "w"), indent=1)
