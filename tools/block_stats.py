#!/usr/bin/env python3
"""Diagnostic (not a test): per instance block of a bench workload (the blocks bench.py's timed steps solve), the
solve kernel's duration (HIP events, the library's default solve) and, from a traced solve of the same block (no
iteration-tail hand-over), the iteration counts and the line-search halvings (alpha = 2^-m) of its instances.

    python tools/block_stats.py --config cfg3 --blocks 22"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import bench  # noqa: E402
import mmpc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg3")
ap.add_argument("--blocks", type=int, default=22)
a = ap.parse_args()
cfg = bench.CONFIGS[a.config]
nx, nu, N, B = cfg["nx"], cfg["nu"], cfg["N"], cfg["B"]
path = mmpc.write_model_json(f"/tmp/block_stats_{a.config}.json", cfg["model"], nx, nu, 2000, N, model=cfg["model"])
s = mmpc.Solver(path, init_states=mmpc.INIT_ZERO, factor_fp32=1 if cfg.get("fp32") else 0, max_iter=60)
s.reserve_workspace(B)
f = dict(dtype=torch.float64, device="cuda")
x0, up, tr = torch.empty((B, nx), **f), torch.empty((B, nu), **f), torch.empty((B, N, nx), **f)
w = torch.tensor(cfg["weights"], **f)
V = torch.zeros((B, s.NV), **f)
st = torch.zeros(B, dtype=torch.int32, device="cuda")
it = torch.zeros(B, dtype=torch.int32, device="cuda")
kk = torch.zeros(B, **f)
trace = torch.zeros((B, 61, 8), **f)
L = s._L
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
for blk in range(a.blocks):
    s.synth(bench.SEED, blk * B, B, x0, up, tr)
    times = []
    for r in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s.solve_batch(B, x0, up, tr, w, V, st, it, None)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    iters = it.cpu().numpy()
    rc = L.mmpc_debug_solve_trace(s._h, B, x0.data_ptr(), up.data_ptr(), tr.data_ptr(), w.data_ptr(), 0, V.data_ptr(),
                                  st.data_ptr(), it.data_ptr(), kk.data_ptr(), trace.data_ptr(), None)
    assert rc == 0, L.mmpc_last_error()
    torch.cuda.synchronize()
    alpha = trace[:, :, 5].cpu().numpy()
    ti = it.cpu().numpy()
    taken = np.arange(61)[None, :] < ti[:, None]
    halv = np.where(taken & (alpha > 0), np.round(-np.log2(np.where(alpha > 0, alpha, 1.0))), 0).astype(int)
    tot = halv.sum(1)
    worst = int(np.argmax(tot))
    print(json.dumps({"block": blk, "kernel_ms": round(float(np.median(times)), 3), "mean_iters": round(float(iters.mean()), 4),
                      "max_iters": int(iters.max()), "iters_hist": {int(k): int(v) for k, v in zip(*np.unique(iters, return_counts=True))},
                      "max_halvings_per_instance": int(tot.max()), "instances_with_halvings": int((tot > 0).sum()),
                      "worst_instance": worst, "worst_alpha": [float(x) for x in alpha[worst, :ti[worst]]]}), flush=True)
