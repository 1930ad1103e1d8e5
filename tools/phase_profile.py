#!/usr/bin/env python3
"""Per-phase cycle breakdown of the SQP kernel (diagnostic build lib/libmmpc_timing.so).

    MMPC_LIB_PATH=mahi-mpc_amd/lib/libmmpc_timing.so python tools/phase_profile.py [--batch 4096]

Stamps serialise the instruction stream, so read the SHARES, not the absolute time."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))
import mmpc  # noqa: E402

NAMES = ["load", "stage_eval", "d_forward", "adjoint+grad+check", "lyapunov", "hessian", "gauss_jordan",
         "dx_forward", "line_search", "writeback"]
NAMES_LANE = ["load", "forward(F,c,d)", "backward(grad+riccati)", "-", "check+forward(step)", "line_search",
              "after_loop", "writeback", "-", "-"]
ap = argparse.ArgumentParser()
ap.add_argument("--config", choices=["cfg2", "cfg3"], default="cfg2")
ap.add_argument("--batch", type=int, default=None)
ap.add_argument("--horizon", type=int, default=None)
ap.add_argument("--kkt", type=int, default=0, help="kkt_solver (0 auto, 1 condensed, 2 riccati)")
ap.add_argument("--u-bound", type=float, default=None, help="control bounds |u| <= U (projected SQP)")
ap.add_argument("--hessian", type=int, default=0, help="mmpc_opts.hessian (0 auto, 1 Gauss-Newton, 2 exact)")
ap.add_argument("--x-bound", type=float, default=None, help="state bounds |qdot| <= X (interior point)")
ap.add_argument("--tol-grad", type=float, default=None, help="mmpc_opts.tol_grad (default 1e-8)")
ap.add_argument("--tol-defect", type=float, default=None, help="mmpc_opts.tol_defect (default 1e-10)")
a = ap.parse_args()
exo = a.config == "cfg3"
B = a.batch or (65536 if exo else 4096)
N = a.horizon or (50 if exo else 30)
nx, nu = (8, 4) if exo else (4, 2)
L = mmpc.lib()
L.mmpc_debug_phase_cycles.argtypes = [C.c_void_p, C.c_int]
path = mmpc.write_model_json("/tmp/mmpc_phase.json", "phase", nx, nu, 2000, N)
s = mmpc.Solver(path, kkt_solver=a.kkt, hessian=a.hessian, tol_grad=a.tol_grad, tol_defect=a.tol_defect)
if a.x_bound is not None:
    s.set_state_bounds([-np.inf] * (nx // 2) + [-a.x_bound] * (nx // 2), [np.inf] * (nx // 2) + [a.x_bound] * (nx // 2))
NAMES_GROUP = ["load", "A:evals(parallel)", "B:d+adjoint(+riccati if not DIST)", "riccati(DIST)+mu",
               "C:step(serial)+dJ", "D:line_search", "after_loop", "writeback", "update(loop top)", "check"]
ksolver = s.kkt_solver_for(B)   # the AUTO choice resolved
if ksolver == 3:
    NAMES = NAMES_GROUP
elif exo or a.kkt == 2 or N * nu > 64:
    NAMES = NAMES_LANE
f = dict(dtype=torch.float64, device="cuda")
x0 = torch.empty((B, nx), **f); up = torch.empty((B, nu), **f); tr = torch.empty((B, N, nx), **f)
s.synth(20250213, 0, B, x0, up, tr)
w = torch.tensor([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4 if exo else [10, 1, 5, 5, 5, 5, .01, .01], **f)
V = torch.zeros((B, s.NV), **f)
lb = None if a.u_bound is None else torch.full((nu,), -a.u_bound, **f)
ub = None if a.u_bound is None else torch.full((nu,), a.u_bound, **f)
it = torch.zeros(B, dtype=torch.int32, device="cuda")
s.solve_batch(B, x0, up, tr, w, V, None, it, None, u_lb=lb, u_ub=ub)
torch.cuda.synchronize()
NSLOT = 16 + 2 * 4096 + 40 * 1024 + 128 * 1024
L.mmpc_debug_phase_table.argtypes = [C.c_void_p, C.c_int, C.c_int]
buf = (C.c_ulonglong * NSLOT)()
L.mmpc_debug_phase_table(buf, NSLOT, 1)
V.zero_()
s.solve_batch(B, x0, up, tr, w, V, None, it, None, u_lb=lb, u_ub=ub)
torch.cuda.synchronize()
L.mmpc_debug_phase_table(buf, NSLOT, 1)
cyc = np.array(buf[:10], dtype=np.float64)
waves = buf[15]
iters = it.cpu().numpy()
out = {"config": a.config, "tol_grad": a.tol_grad, "tol_defect": a.tol_defect, "u_bound": a.u_bound, "x_bound": a.x_bound, "hessian": s.hessian_for(B, a.u_bound is not None), "waves": int(waves), "mean_iters": float(iters.mean()), "max_iters": int(iters.max()),
       "iters_hist": {int(k): int(v) for k, v in zip(*np.unique(iters, return_counts=True))},
       # a wave runs until its slowest instance: 4 instances per wave (16-lane kernel) or 64 (lane kernel)
       "wave_max_iters_mean": float(iters[: B // (4 if ksolver == 3 else 64) * (4 if ksolver == 3 else 64)]
                                    .reshape(-1, 4 if ksolver == 3 else 64).max(1).mean()),
       "cycles_per_wave": float(cyc.sum() / waves),
       # wall-clock extents (s_memrealtime, 100 MHz): the kernel's span from the first wave start to the last wave end,
       # the longest and the mean wave, and the mean shader clock of the waves (s_memtime cycles / duration)
       "span_us": float((buf[10] - (~buf[11] & 0xFFFFFFFFFFFFFFFF)) / 100.0),
       "longest_wave_us": float(buf[12] / 100.0),
       "mean_wave_us": float(buf[13] / 100.0 / waves),
       "mean_clock_ghz": float(buf[14] / buf[13] * 0.1) if buf[13] else None,
       "per_phase_cycles_per_wave_iteration": {n: float(c / waves / (iters.mean() + 1)) for n, c in zip(NAMES, cyc)},
       "share": {n: float(c / cyc.sum()) for n, c in zip(NAMES, cyc)}}
# the slowest waves (slots 16 + blockIdx.x: one wave per block) and the iteration counts of their instances
ipw = 4 if ksolver == 3 else 64
nw = (B + ipw - 1) // ipw   # the solve kernel's waves (a lane-kernel solve's resume launch reuses the low slots)
dur = np.array(buf[16:16 + min(nw, 4096)], dtype=np.float64) / 100.0
cyc_w = np.array(buf[16 + 4096:16 + 4096 + min(nw, 4096)], dtype=np.float64)
if len(dur) and int(waves) == nw:
    ghz = cyc_w / np.maximum(dur, 1e-9) * 1e-3
    wm = np.pad(iters, (0, nw * ipw - B)).reshape(-1, ipw).max(1)[: len(dur)]
    out["wave_clock_ghz_percentiles"] = {str(q): float(np.percentile(ghz, q)) for q in (0, 10, 50, 90, 100)}
    order = np.argsort(dur)[::-1][:12]
    out["wave_us_percentiles"] = {str(q): float(np.percentile(dur, q)) for q in (0, 10, 50, 90, 99, 100)}
    wph4 = np.array(buf[16 + 2 * 4096:16 + 2 * 4096 + 40 * 1024], dtype=np.float64).reshape(1024, 4, 10)
    wph = wph4[:, 0]   # lane 0
    if len(dur) <= 1024:   # per-phase cycles of the waves, by their slowest instance's iteration count
        out["phase_cycles_by_wave_max_iters"] = {
            int(m): {n: float(v) for n, v in zip(NAMES, wph[: len(dur)][wm == m].mean(0))} for m in np.unique(wm)}
    out["slowest_waves"] = [{"block": int(b), "us": float(dur[b]), "ghz": float(ghz[b]),
                             "phases": ({n: float(v) for n, v in zip(NAMES, wph[b])} if b < 1024 else None),
                             "riccati_stage_cycles_by_group": ([np.diff(np.array(buf[16 + 2 * 4096 + 40 * 1024 + 128 * b
                                                                  + 32 * g:16 + 2 * 4096 + 40 * 1024 + 128 * b + 32 * g + N],
                                                                 dtype=np.int64)[::-1]).tolist() for g in range(4)]
                                                               if b < 1024 and N <= 32 else None),
                             "phases_by_group": ([{n: float(v) for n, v in zip(NAMES, wph4[b, g])} for g in range(4)]
                                                 if b < 1024 else None),
                             "iters": [int(v) for v in iters[b * ipw:(b + 1) * ipw]][:16]} for b in order]
    out["mean_us_by_wave_max_iters"] = {
        int(m): [float(dur[wm == m].mean()), float(ghz[wm == m].mean()), int((wm == m).sum())]
        for m in np.unique(wm)}
print(json.dumps(out, indent=1))
