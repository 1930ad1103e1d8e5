"""GPU parity of the Riccati (lane-per-instance) solve path, sqp_lane.h, through the C-ABI.

Covers SURVEY.md 8a A3b (exo dynamics) and the cfg#3 workload shape, plus the 2-link arm on the Riccati
path (cross-checked against the condensed kernel and the oracle).  Tolerances:
  * GPU vs oracle (same GN-SQP, different exact KKT solve: Riccati vs dense Cholesky): V* within 1e-9
    relative where iteration counts agree (>= 99 %), 1e-6 where a stop test flips (see _compare).
  * GPU vs scipy golden (independent formulation/solver): V* within 1e-8 relative, J* within 1e-11.
  * Jacobians vs complex-step golden: 1e-11 relative.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, WEIGHTS_CFG
from test_gpu_parity import _compare, _rel

pytestmark = pytest.mark.gpu

H = 0.002
W_EXO = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)  # SURVEY.md 8d cfg#3 weights


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def exo_golden():
    return json.load(open(os.path.join(GOLDEN, "exo_golden.json")))


@pytest.fixture
def exo_solver(tmp_path, mmpc_mod):
    def make(N=50, is_linear=False, **kw):
        p = mmpc_mod.write_model_json(str(tmp_path / f"exo_{N}_{int(is_linear)}.json"), "exo", 8, 4, 2000, N,
                                      is_linear=is_linear, model="exo_arm")
        return mmpc_mod.Solver(p, **kw)
    return make


def _dev(torch, *arrs):
    return [torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda") for a in arrs]


def test_exo_synth_matches_oracle(exo_solver, oracle, torch_cuda):
    torch = torch_cuda
    s = exo_solver()
    B = 1000
    x0 = torch.empty((B, 8), dtype=torch.float64, device="cuda")
    up = torch.empty((B, 4), dtype=torch.float64, device="cuda")
    tr = torch.empty((B, 50, 8), dtype=torch.float64, device="cuda")
    s.synth(20250213, 777, B, x0, up, tr)
    torch.cuda.synchronize()
    ox, ou, ot = oracle.synth(20250213, 777, B, 50, H, model=oracle.EXO)
    np.testing.assert_array_equal(x0.cpu().numpy(), ox)
    np.testing.assert_array_equal(up.cpu().numpy(), ou)
    np.testing.assert_allclose(tr.cpu().numpy(), ot, rtol=2e-14, atol=2e-15)


def test_exo_linearize_vs_complex_step(exo_golden, exo_solver, torch_cuda):
    s = exo_solver()
    pts = exo_golden["jacobian_points"]
    A, Bm, xd = s.linearize_host(np.array([p["x"] for p in pts]), np.array([p["u"] for p in pts]))
    for i, p in enumerate(pts):
        for got, ref in ((A[i], p["A"]), (Bm[i], p["B"]), (xd[i], p["xdot"])):
            ref = np.array(ref)
            assert np.abs(got - ref).max() <= 1e-11 * np.abs(ref).max()


def test_exo_nlp_eval_vs_oracle(exo_solver, oracle, torch_cuda):
    torch = torch_cuda
    B, N = 64, 50
    x0, up, tr = oracle.synth(3, 0, B, N, H, model=oracle.EXO)
    rng = np.random.default_rng(3)
    V = rng.uniform(-1, 1, (B, 8 * (N + 1) + 4 * N))
    s = exo_solver()
    Vd, upd, trd, wd = _dev(torch, V, up, tr, W_EXO)
    J = torch.zeros(B, dtype=torch.float64, device="cuda")
    d = torch.zeros(B, dtype=torch.float64, device="cuda")
    s.nlp_eval(B, Vd, upd, trd, wd, J, d)
    torch.cuda.synchronize()
    for b in range(B):
        Jo, go = oracle.nlp_eval(N, H, V[b], up[b], tr[b], W_EXO, model=oracle.EXO)
        assert J[b].item() == pytest.approx(Jo, rel=1e-12)
        assert d[b].item() == pytest.approx(np.abs(go).max(), rel=1e-12)


def test_exo_solve_vs_scipy_golden(exo_golden, exo_solver, oracle, torch_cuda):
    w = np.array(exo_golden["weights"])
    for N in sorted({c["N"] for c in exo_golden["cases"]}):
        cs = [c for c in exo_golden["cases"] if c["N"] == N]
        x0 = np.array([c["x0"] for c in cs]); up = np.array([c["u_prev"] for c in cs])
        tr = np.array([c["traj"] for c in cs]); Vg = np.array([c["V"] for c in cs])
        s = exo_solver(N=N)
        r = s.solve_batch_host(x0, up, tr, w)
        assert (r["status"] == 0).all(), r["status"]
        assert _rel(r["V"], Vg).max() <= 1e-8
        for b, c in enumerate(cs):
            J, _ = oracle.nlp_eval(N, H, r["V"][b], up[b], tr[b], w, model=oracle.EXO)
            assert J == pytest.approx(c["J"], rel=1e-11)
        o = oracle.solve_batch(N, H, x0, up, tr, w, model=oracle.EXO)
        _compare(r, o, min_same=1.0)


def test_exo_batch_vs_oracle(exo_solver, oracle, torch_cuda):
    """cfg#3 recipe, 512 instances, every one against the oracle (ragged batch: 512 = 8 full waves)."""
    B, N = 512, 50
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=oracle.EXO)
    s = exo_solver()
    r = s.solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO)
    assert (r["status"] == 0).all()
    _compare(r, o)


def test_exo_ragged_batch_and_horizons(exo_solver, oracle, torch_cuda):
    # B not a multiple of 64 (partial last wave) and short / long horizons
    for N, B in ((1, 3), (7, 65), (100, 70)):
        x0, up, tr = oracle.synth(11, 5, B, N, H, model=oracle.EXO)
        r = exo_solver(N=N).solve_batch_host(x0, up, tr, W_EXO)
        o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO)
        _compare(r, o)


def _exo_full_batch(exo_solver, oracle, torch, factor_fp32):
    """cfg#3 / cfg#5 at full size (B = 65536, N = 50) on one GPU: size-independent properties on every
    instance (all converged, KKT residual, pinned x_0, zero defects through the device nlp_eval, bitwise
    determinism) and 1024 evenly spaced instances against the oracle."""
    B, N = 65536, 50
    s = exo_solver(factor_fp32=factor_fp32)
    s.reserve_workspace(B)
    x0 = torch.empty((B, 8), dtype=torch.float64, device="cuda")
    up = torch.empty((B, 4), dtype=torch.float64, device="cuda")
    tr = torch.empty((B, N, 8), dtype=torch.float64, device="cuda")
    s.synth(20250213, 0, B, x0, up, tr)
    w = torch.tensor(W_EXO, dtype=torch.float64, device="cuda")
    outs = []
    for _ in range(2):
        V = torch.zeros((B, s.NV), dtype=torch.float64, device="cuda")
        st = torch.full((B,), -1, dtype=torch.int32, device="cuda")
        it = torch.zeros(B, dtype=torch.int32, device="cuda")
        kkt = torch.zeros(B, dtype=torch.float64, device="cuda")
        s.solve_batch(B, x0, up, tr, w, V, st, it, kkt)
        torch.cuda.synchronize()
        outs.append((V, st, it, kkt))
    V, st, it, kkt = outs[0]
    assert torch.equal(outs[0][0], outs[1][0])                   # bitwise deterministic
    stn = st.cpu().numpy()
    assert (stn == 0).all(), np.bincount(stn + 1)               # every instance converged (as the bench reports)
    assert (kkt.cpu().numpy() <= 1e-8).all()
    assert torch.equal(V[:, :8], x0)
    Jd = torch.zeros(B, dtype=torch.float64, device="cuda")
    dd = torch.zeros(B, dtype=torch.float64, device="cuda")
    s.nlp_eval(B, V, up, tr, w, Jd, dd)
    torch.cuda.synchronize()
    assert dd.cpu().numpy().max() <= 1e-10
    idx = np.arange(0, B, 64)                                    # 1024 instances against the oracle
    xo, uo, to = x0.cpu().numpy()[idx], up.cpu().numpy()[idx], tr.cpu().numpy()[idx]
    o = oracle.solve_batch(N, H, xo, uo, to, W_EXO, model=oracle.EXO)
    gpu = dict(V=V.cpu().numpy()[idx], status=stn[idx], iters=it.cpu().numpy()[idx])
    return gpu, o, Jd.cpu().numpy()[idx]


def test_exo_cfg3_full_batch_properties(exo_solver, oracle, torch_cuda):
    gpu, o, J = _exo_full_batch(exo_solver, oracle, torch_cuda, 0)
    _compare(gpu, o)
    np.testing.assert_allclose(J, o["J"], rtol=1e-10)


def test_exo_cfg5_full_batch_properties(exo_solver, oracle, torch_cuda):
    """cfg#5 (fp32 Riccati factor, fp64 residuals) at full size: the same stop test on every instance, so the
    same KKT point to the accuracy the stop test guarantees (1e-6 relative in V*, J* to 1e-9)."""
    gpu, o, J = _exo_full_batch(exo_solver, oracle, torch_cuda, 1)
    assert (o["status"] == 0).all()
    assert _rel(gpu["V"], o["V"]).max() <= 1e-6
    np.testing.assert_allclose(J, o["J"], rtol=1e-10)


def test_riccati_two_link_matches_condensed_and_oracle(model_json, mmpc_mod, oracle, torch_cuda):
    """The 2-link arm (cfg#2 recipe) through both device KKT solvers and the oracle."""
    B, N = 512, 30
    x0, up, tr = oracle.synth(20250213, 0, B, N, H)
    w = np.array(WEIGHTS_CFG)
    rc = mmpc_mod.Solver(model_json(N=N), kkt_solver=mmpc_mod.KKT_CONDENSED).solve_batch_host(x0, up, tr, w)
    rr = mmpc_mod.Solver(model_json(N=N), kkt_solver=mmpc_mod.KKT_RICCATI).solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w)
    _compare(rr, o)
    _compare(rr, rc)


@pytest.mark.parametrize("N", [33, 50, 120])
def test_riccati_two_link_long_horizons(N, model_json, mmpc_mod, oracle):
    # beyond the condensed kernel's N*nu <= 64: MMPC_KKT_AUTO selects the Riccati kernel
    x0, up, tr = oracle.synth(21, 0, 96, N, H)
    w = np.array(WEIGHTS_CFG)
    s = mmpc_mod.Solver(model_json(N=N))
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w, solver=s)
    _compare(r, o)


def test_riccati_linear_mode(model_json, exo_solver, mmpc_mod, oracle):
    x0, up, tr = oracle.synth(11, 0, 128, 25, H)
    w = np.array(WEIGHTS_CFG)
    s = mmpc_mod.Solver(model_json(N=25, name="linear_double_pendulum", is_linear=True),
                        kkt_solver=mmpc_mod.KKT_RICCATI)
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(25, H, x0, up, tr, w, is_linear=True)
    assert (r["iters"] == 1).all()
    _compare(r, o, min_same=1.0)
    x0, up, tr = oracle.synth(7, 0, 70, 50, H, model=oracle.EXO)
    r = exo_solver(is_linear=True).solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(50, H, x0, up, tr, W_EXO, is_linear=True, model=oracle.EXO)
    _compare(r, o, min_same=1.0)


def test_riccati_weights_bounds_nonfinite_warmstart(exo_solver, oracle):
    N = 50
    x0, up, tr = oracle.synth(13, 0, 64, N, H, model=oracle.EXO)
    rng = np.random.default_rng(0)
    w = np.tile(W_EXO, (64, 1)) * rng.uniform(0.5, 2.0, (64, 16))
    s = exo_solver()
    r = s.solve_batch_host(x0, up, tr, w)                       # per-instance weights
    _compare(r, oracle.solve_batch(N, H, x0, up, tr, w, model=oracle.EXO))
    r2 = s.solve_batch_host(x0, up, tr, w, V=r["V"])            # warm start = fixed point
    assert (r2["iters"] == 0).all() and (r2["status"] == 0).all()
    np.testing.assert_array_equal(r2["V"], r["V"])
    lb, ub = [-1e-3] * 4, [1e-3] * 4                             # bounds enforced
    r3 = s.solve_batch_host(x0[:8], up[:8], tr[:8], W_EXO, u_lb=lb, u_ub=ub)
    o3 = oracle.solve_batch(N, H, x0[:8], up[:8], tr[:8], W_EXO, u_lb=lb, u_ub=ub, model=oracle.EXO, solver=s)
    np.testing.assert_array_equal(r3["status"], o3["status"])
    x0b, trb = x0[:4].copy(), tr[:4].copy()                      # non-finite inputs
    x0b[1, 2] = np.nan
    trb[2, 7, 5] = np.inf
    r4 = s.solve_batch_host(x0b, up[:4], trb, W_EXO)
    assert list(r4["status"]) == [0, 3, 3, 0]
    s1 = exo_solver(max_iter=1)                                  # max_iter
    r5 = s1.solve_batch_host(x0[:4], up[:4], tr[:4], W_EXO)
    o5 = oracle.solve_batch(N, H, x0[:4], up[:4], tr[:4], W_EXO, max_iter=1, model=oracle.EXO)
    assert (r5["status"] == 1).all() and (r5["iters"] == 1).all()
    assert _rel(r5["V"], o5["V"]).max() < 1e-10


def test_fp32_factor_converges_to_the_fp64_solution(exo_solver, model_json, mmpc_mod, oracle):
    """SURVEY.md 8d cfg#5: fp32 Riccati factor, fp64 residuals.  Same KKT point to the accuracy the stop test
    guarantees (1e-6 relative in V*), every instance converged; the fp64 residual test is unchanged."""
    N = 50
    x0, up, tr = oracle.synth(20250213, 0, 256, N, H, model=oracle.EXO)
    r32 = exo_solver(factor_fp32=1).solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO)
    assert (r32["status"] == 0).all(), np.bincount(r32["status"])
    assert (r32["kkt"] <= 1e-8).all()
    assert _rel(r32["V"], o["V"]).max() <= 1e-6
    x0, up, tr = oracle.synth(5, 0, 128, 30, H)
    w = np.array(WEIGHTS_CFG)
    r32 = mmpc_mod.Solver(model_json(N=30), factor_fp32=1).solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(30, H, x0, up, tr, w)
    assert (r32["status"] == 0).all()
    assert _rel(r32["V"], o["V"]).max() <= 1e-6


def test_fp32_factor_is_riccati_only(model_json, mmpc_mod, oracle):
    x0, up, tr = oracle.synth(5, 0, 2, 30, H)
    s = mmpc_mod.Solver(model_json(N=30), factor_fp32=1, kkt_solver=mmpc_mod.KKT_CONDENSED)
    with pytest.raises(mmpc_mod.MmpcError) as ei:
        s.solve_batch_host(x0, up, tr, np.array(WEIGHTS_CFG))
    assert ei.value.code == -4


# ---- 16-lanes-per-instance Riccati kernel (sqp_group.h) ----
@pytest.mark.parametrize("N,B", [(30, 512), (1, 5), (7, 70), (33, 65), (50, 64)])
def test_group_kernel_vs_oracle(N, B, model_json, mmpc_mod, oracle):
    x0, up, tr = oracle.synth(20250213, 3, B, N, H)
    w = np.array(WEIGHTS_CFG)
    s = mmpc_mod.Solver(model_json(N=N), kkt_solver=mmpc_mod.KKT_RICCATI_GROUP)
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w, solver=s)
    _compare(r, o)


def test_group_kernel_linear_weights_bounds_nonfinite_warmstart(model_json, mmpc_mod, oracle):
    G = mmpc_mod.KKT_RICCATI_GROUP
    x0, up, tr = oracle.synth(11, 0, 64, 25, H)
    w = np.array(WEIGHTS_CFG)
    s = mmpc_mod.Solver(model_json(N=25, name="linear_double_pendulum", is_linear=True), kkt_solver=G)
    r = s.solve_batch_host(x0, up, tr, w)
    assert (r["iters"] == 1).all()
    _compare(r, oracle.solve_batch(25, H, x0, up, tr, w, is_linear=True), min_same=1.0)
    x0, up, tr = oracle.synth(13, 0, 64, 30, H)
    rng = np.random.default_rng(0)
    wi = np.tile(WEIGHTS_CFG, (64, 1)) * rng.uniform(0.5, 2.0, (64, 8))
    s = mmpc_mod.Solver(model_json(N=30), kkt_solver=G)
    r = s.solve_batch_host(x0, up, tr, wi)
    _compare(r, oracle.solve_batch(30, H, x0, up, tr, wi, solver=s))
    r2 = s.solve_batch_host(x0, up, tr, wi, V=r["V"])
    assert (r2["iters"] == 0).all() and (r2["status"] == 0).all()
    np.testing.assert_array_equal(r2["V"], r["V"])
    r3 = s.solve_batch_host(x0[:8], up[:8], tr[:8], w, u_lb=[-1e-3, -1e-3], u_ub=[1e-3, 1e-3])
    o3 = oracle.solve_batch(30, H, x0[:8], up[:8], tr[:8], w, u_lb=[-1e-3, -1e-3], u_ub=[1e-3, 1e-3], solver=s)
    np.testing.assert_array_equal(r3["status"], o3["status"])
    x0b, trb = x0[:4].copy(), tr[:4].copy()
    x0b[1, 0] = np.nan
    trb[2, 3, 1] = np.inf
    r4 = s.solve_batch_host(x0b, up[:4], trb, w)
    assert list(r4["status"]) == [0, 3, 3, 0]


@pytest.mark.parametrize("N,B", [(20, 70), (5, 9), (40, 64)])
def test_group_kernel_exo_vs_oracle(N, B, exo_solver, mmpc_mod, oracle):
    # explicit request (AUTO keeps exo on the lane kernel); stage data fits LDS up to N = 47
    x0, up, tr = oracle.synth(20250213, 7, B, N, H, model=oracle.EXO)
    r = exo_solver(N=N, kkt_solver=mmpc_mod.KKT_RICCATI_GROUP).solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO)
    _compare(r, o)


def test_group_kernel_exo_lds_limit(exo_solver, mmpc_mod, oracle):
    # N = 50 exceeds 160 KB of LDS for 4 exo instances: explicit request fails, AUTO uses lanes
    x0, up, tr = oracle.synth(1, 0, 4, 50, H, model=oracle.EXO)
    with pytest.raises(mmpc_mod.MmpcError) as ei:
        exo_solver(N=50, kkt_solver=mmpc_mod.KKT_RICCATI_GROUP).solve_batch_host(x0, up, tr, W_EXO)
    assert ei.value.code == -4
    r = exo_solver(N=50).solve_batch_host(x0, up, tr, W_EXO)
    assert (r["status"] == 0).all()
