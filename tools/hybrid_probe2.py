#!/usr/bin/env python3
"""Probe: library hybrid (one call) vs manual two-stream split vs single kernels, same inputs, 20 reps each."""
import json, os, sys, tempfile
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import mmpc  # noqa: E402
B, N, nx, nu = 4096, 30, 4, 2
d = tempfile.mkdtemp()
path = mmpc.write_model_json(os.path.join(d, "m.json"), "m", nx, nu, 2000, N, model="two_link_arm")
sc = mmpc.Solver(path, kkt_solver=mmpc.KKT_CONDENSED)
sg = mmpc.Solver(path, kkt_solver=mmpc.KKT_RICCATI_GROUP)
sh = mmpc.Solver(path, kkt_solver=mmpc.KKT_HYBRID)
sg.reserve_workspace(B); sh.reserve_workspace(B)
f = dict(dtype=torch.float64, device="cuda")
x0 = torch.empty((B, nx), **f); up = torch.empty((B, nu), **f); tr = torch.empty((B, N, nx), **f)
sc.synth(20250213, 0, B, x0, up, tr)
w = torch.tensor([10, 1, 5, 5, 5, 5, .01, .01], **f)
V = torch.zeros((B, sc.NV), **f)
st = torch.zeros(B, dtype=torch.int32, device="cuda")
s1 = torch.cuda.current_stream(); s2 = torch.cuda.Stream()
Bg = 2868; Bc = B - Bg
def manual(first_group=True):
    s2.wait_stream(s1)
    if first_group:
        sg.solve_batch(Bg, x0[Bc:], up[Bc:], tr[Bc:], w, V[Bc:], st[Bc:], None, None, stream=s2.cuda_stream)
        sc.solve_batch(Bc, x0, up, tr, w, V, st, None, None, stream=s1.cuda_stream)
    else:
        sc.solve_batch(Bc, x0, up, tr, w, V, st, None, None, stream=s1.cuda_stream)
        sg.solve_batch(Bg, x0[Bc:], up[Bc:], tr[Bc:], w, V[Bc:], st[Bc:], None, None, stream=s2.cuda_stream)
    s1.wait_stream(s2)
variants = {
    "condensed": lambda: sc.solve_batch(B, x0, up, tr, w, V, st, None, None, stream=s1.cuda_stream),
    "group": lambda: sg.solve_batch(B, x0, up, tr, w, V, st, None, None, stream=s1.cuda_stream),
    "lib_hybrid": lambda: sh.solve_batch(B, x0, up, tr, w, V, st, None, None, stream=s1.cuda_stream),
    "manual_group_first": lambda: manual(True),
    "manual_condensed_first": lambda: manual(False),
}
res = {}
for sync in (True, False):
    for name, fn in variants.items():
        times = []
        for rep in range(22):
            V.zero_()
            if sync: torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s1); fn(); e1.record(s1)
            if sync: torch.cuda.synchronize()
            times.append((e0, e1))
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in times[2:]]
        res[f"{name}_sync{int(sync)}"] = dict(ms=sum(ms) / len(ms), min_ms=min(ms), conv=int((st == 0).sum()))
        print(f"{name}_sync{int(sync)}", res[f"{name}_sync{int(sync)}"], flush=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "hybrid_probe2.json"), "w"), indent=1)
