"""Per-iteration trace of the cfg#2 batch (B = 4096, AUTO solver): iteration histogram and, per iteration, the
defect / gradient norms -- which iterations end with ||g|| <= tol_defect but ||grad|| > tol_grad."""
import ctypes as C
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "mahi-mpc_amd")
import mmpc  # noqa: E402

B, N = 4096, 30
path = mmpc.write_model_json("/tmp/m.json", "nonlinear_double_pendulum", 4, 2, 2000, N)
s = mmpc.Solver(path)
L = mmpc.lib()
L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
f = dict(dtype=torch.float64, device="cuda")
x0 = torch.empty((B, 4), **f); up = torch.empty((B, 2), **f); tr = torch.empty((B, N, 4), **f)
s.synth(20250213, 0, B, x0, up, tr)
w = torch.tensor([10, 1, 5, 5, 5, 5, .01, .01], **f)
V = torch.zeros((B, s.NV), **f)
st = torch.zeros(B, dtype=torch.int32, device="cuda"); it = torch.zeros(B, dtype=torch.int32, device="cuda")
kk = torch.zeros(B, **f); trc = torch.zeros((B, 51, 8), **f)
rc = L.mmpc_debug_solve_trace(s._h, B, x0.data_ptr(), up.data_ptr(), tr.data_ptr(), w.data_ptr(), 0, V.data_ptr(),
                              st.data_ptr(), it.data_ptr(), kk.data_ptr(), trc.data_ptr(), None)
torch.cuda.synchronize()
it = it.cpu().numpy(); T = trc.cpu().numpy()
hist = np.bincount(it).tolist()
small_c_not_final = 0; small_c_total = 0
rows = []
for b in range(B):
    for i in range(it[b] + 1):
        g, c = T[b, i, 0], T[b, i, 1]
        if c <= 1e-10:
            small_c_total += 1
            if i < it[b]:
                small_c_not_final += 1
worst = np.argsort(-it)[:8]
for b in worst:
    rows.append([[float(T[b, i, 0]), float(T[b, i, 1]), float(T[b, i, 5])] for i in range(it[b] + 1)])
out = dict(rc=rc, hist=hist, mean=float(it.mean()), total_passes=int((it + 1).sum()),
           small_defect_passes=small_c_total, small_defect_not_final=small_c_not_final,
           worst_idx=worst.tolist(), worst_trace_grad_defect_alpha=rows)
# per final iteration count: quantiles of the stop-test norms at the check before the last one, and how many took
# a step shorter than alpha = 1
q = {}
for n in sorted(set(it.tolist())):
    sel = it == n
    if n == 0:
        continue
    g, c = T[sel, n - 1, 0], T[sel, n - 1, 1]
    al = T[sel, :n, 5]
    q[int(n)] = dict(count=int(sel.sum()),
                     grad_before_last_q=[float(v) for v in np.quantile(g, [0.0, 0.5, 0.9, 1.0])],
                     defect_before_last_q=[float(v) for v in np.quantile(c, [0.0, 0.5, 0.9, 1.0])],
                     short_steps=int((al < 1.0).sum()),
                     grad_by_iter_median=[float(np.median(T[sel, i, 0])) for i in range(n + 1)],
                     defect_by_iter_median=[float(np.median(T[sel, i, 1])) for i in range(n + 1)])
out["by_iters"] = q
json.dump(out, open("gpurun_out/cfg2_trace.json", "w"), indent=1)
print(json.dumps({k: out[k] for k in ("rc", "hist", "mean", "total_passes", "small_defect_passes",
                                      "small_defect_not_final")}))
print(json.dumps(q, indent=1))
