"""GPU: the lane kernel's lazy step records (round 6, csrc/sqp_lane.h MMPC_LANE_LAZY_DXU).  An unbounded lane solve
stores the step (dx_k, du_k) only in its first iteration; a lane whose full step is rejected later regenerates it
before its first shorter trial.  Instances with targets far from the initial state (x 20) and a small Delta-u weight
take shorter steps in later iterations too (asserted from the per-iteration trace of the same solve, so the
regeneration runs; the iteration-tail hand-over is off, so every iteration runs in the lane kernel), and
must still match the oracle's Riccati restatement of the same SQP as every same-algorithm comparison does
(tests/test_gpu_parity.py _compare: V* within 1e-10 where the iteration counts agree)."""
import ctypes as C

import numpy as np
import pytest

from conftest import WEIGHTS_CFG
from test_gpu_parity import _compare, _rel

pytestmark = pytest.mark.gpu

H = 0.002
W_EXO = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)


# regen: whether this batch has shorter steps after the first iteration (GPU trace, round 6: 2-link Gauss-Newton 1,
# exo exact 8 instance-iterations; the exo Gauss-Newton batch takes only full steps after the first iteration).  The
# exact-Hessian lane kernel keeps storing dx / du every iteration (sqp_lane.h LAZY): its case checks that path.
@pytest.mark.parametrize("model,N,B,hess,regen", [("two_link_arm", 30, 256, "gn", True), ("exo_arm", 50, 128, "gn", False),
                                                   ("exo_arm", 50, 128, "exact", True)])
def test_lane_lazy_step_records_vs_oracle(model, N, B, hess, regen, mmpc_mod, oracle, tmp_path):
    import torch
    om = oracle.EXO if model == "exo_arm" else oracle.TWO_LINK
    w = (W_EXO if model == "exo_arm" else np.array(WEIGHTS_CFG)).copy()
    nx, nu = (8, 4) if model == "exo_arm" else (4, 2)
    w[nx:nx + nu] *= 0.01
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=om)
    tr = np.ascontiguousarray(tr * 20.0)
    p = mmpc_mod.write_model_json(str(tmp_path / f"{model}_{N}.json"), model, nx, nu, 2000, N, model=model)
    h = mmpc_mod.HESSIAN_EXACT if hess == "exact" else mmpc_mod.HESSIAN_GAUSS_NEWTON
    # no iteration-tail hand-over: every iteration runs in the lane kernel (as the trace solve below)
    s = mmpc_mod.Solver(p, kkt_solver=2, hessian=h, init_states=mmpc_mod.INIT_ZERO, max_iter=60, tail_cap=0)
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w, model=om, kkt=oracle.KKT_RICCATI, init_states=2, max_iter=60,
                           hessian=oracle.HESS_EXACT if hess == "exact" else oracle.HESS_GAUSS_NEWTON)
    assert (r["status"] == 0).all() and (o["status"] == 0).all()
    _compare(r, o)
    # the same solve with the per-iteration trace: some lane rejects its full step after the first iteration
    f64 = dict(dtype=torch.float64, device="cuda")
    t = [torch.tensor(a, **f64) for a in (x0, up, tr, w)]
    V = torch.zeros((B, s.NV), **f64)
    st = torch.zeros(B, dtype=torch.int32, device="cuda")
    it = torch.zeros(B, dtype=torch.int32, device="cuda")
    kk = torch.zeros(B, **f64)
    trace = torch.zeros((B, 61, 8), **f64)
    L = s._L
    L.mmpc_debug_solve_trace.argtypes = [C.c_void_p, C.c_int64] + [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 6
    rc = L.mmpc_debug_solve_trace(s._h, B, *(a.data_ptr() for a in t), 0, V.data_ptr(), st.data_ptr(),
                                  it.data_ptr(), kk.data_ptr(), trace.data_ptr(), None)
    assert rc == 0, L.mmpc_last_error()
    torch.cuda.synchronize()
    iters = it.cpu().numpy()
    alpha = trace[:, :, 5].cpu().numpy()
    later = (np.arange(61)[None, :] >= 1) & (np.arange(61)[None, :] < iters[:, None])
    n_short = int(((alpha < 1.0) & later).sum())
    print(f"{model} {hess}: {n_short} instance-iterations after the first with alpha < 1")
    assert (n_short > 0) == regen
    # the instances whose later steps were shorter (the regenerated records): the oracle's iterates exactly, not merely
    # inside _compare's allowance for a stop test on the other side of its threshold
    short = ((alpha < 1.0) & later).any(1)
    if short.any():
        assert (r["iters"][short] == o["iters"][short]).all(), (r["iters"][short], o["iters"][short])
        assert _rel(r["V"][short], o["V"][short]).max() <= 1e-10
    assert np.array_equal(V.cpu().numpy(), r["V"]) and np.array_equal(iters, r["iters"])   # trace: same iterates


@pytest.mark.parametrize("model,N,B,hess", [("two_link_arm", 30, 256, "gn"), ("exo_arm", 50, 128, "exact")])
def test_lane_line_search_handover_vs_oracle(model, N, B, hess, mmpc_mod, oracle, tmp_path):
    """The same batches with the default iteration-tail policy: a lane whose full step is rejected after the first
    iteration is handed to the 16-lane resume launch instead of line-searching in its wave (sqp_lane.h
    MMPC_LANE_LS_HANDOVER).  The resume launch runs the same SQP from the same iterate, count and merit weight, so the
    solutions are the oracle's (as every hand-over test: tests/test_gpu_tail.py)."""
    om = oracle.EXO if model == "exo_arm" else oracle.TWO_LINK
    w = (W_EXO if model == "exo_arm" else np.array(WEIGHTS_CFG)).copy()
    nx, nu = (8, 4) if model == "exo_arm" else (4, 2)
    w[nx:nx + nu] *= 0.01
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=om)
    tr = np.ascontiguousarray(tr * 20.0)
    p = mmpc_mod.write_model_json(str(tmp_path / f"{model}_{N}.json"), model, nx, nu, 2000, N, model=model)
    h = mmpc_mod.HESSIAN_EXACT if hess == "exact" else mmpc_mod.HESSIAN_GAUSS_NEWTON
    s = mmpc_mod.Solver(p, kkt_solver=2, hessian=h, init_states=mmpc_mod.INIT_ZERO, max_iter=60)
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w, model=om, kkt=oracle.KKT_RICCATI, init_states=2, max_iter=60,
                           hessian=oracle.HESS_EXACT if hess == "exact" else oracle.HESS_GAUSS_NEWTON)
    assert (r["status"] == 0).all() and (o["status"] == 0).all()
    _compare(r, o)
