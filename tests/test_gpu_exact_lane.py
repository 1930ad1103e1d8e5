"""GPU: the exact-Hessian SQP (mmpc_opts.hessian = EXACT; IPOPT's default Hessian, CasADi nlp_hess_l at
ModelGenerator.cpp:238) on the lane-per-instance Riccati kernel (round 4) and on the 16-lane group kernel for the
exo, against the oracle's ORACLE_HESS_EXACT (oracle_exo_hess / oracle_two_link_hess in its Riccati restatement).

Tolerance as every same-algorithm comparison (tests/test_gpu_parity.py _compare): V* within 1e-10 relative where
the iteration counts agree (>= 99 % of the instances), 1e-6 where a stop test lands on the other side of its
threshold.  The exact Hessian changes the iteration path, not the KKT point: the exact solutions also match the
Gauss-Newton ones to the stop test's accuracy."""
import numpy as np
import pytest

from conftest import WEIGHTS_CFG
from test_gpu_parity import _compare, _rel

pytestmark = pytest.mark.gpu

H = 0.002
W_EXO = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)   # SURVEY.md 8d cfg#3 weights


def _solver(mmpc_mod, tmp_path, model, N, **kw):
    nx, nu = (8, 4) if model == "exo_arm" else (4, 2)
    p = mmpc_mod.write_model_json(str(tmp_path / f"{model}_{N}.json"), model, nx, nu, 2000, N, model=model)
    return mmpc_mod.Solver(p, **kw)


@pytest.mark.parametrize("model,N,B", [("exo_arm", 50, 256), ("exo_arm", 7, 65), ("two_link_arm", 30, 256)])
def test_lane_exact_vs_oracle(model, N, B, mmpc_mod, oracle, tmp_path):
    om = oracle.EXO if model == "exo_arm" else oracle.TWO_LINK
    w = W_EXO if model == "exo_arm" else np.array(WEIGHTS_CFG)
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=om)
    s = _solver(mmpc_mod, tmp_path, model, N, kkt_solver=2, hessian=mmpc_mod.HESSIAN_EXACT,
                init_states=mmpc_mod.INIT_ZERO)
    assert s.kkt_solver_for(B) == 2 and s.hessian_for(B, False) == mmpc_mod.HESSIAN_EXACT
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w, model=om, hessian=oracle.HESS_EXACT, kkt=oracle.KKT_RICCATI,
                           init_states=2)
    assert (r["status"] == 0).all() and (o["status"] == 0).all()
    _compare(r, o)
    # same KKT point as the Gauss-Newton solve (the exact Hessian changes the path only)
    g = _solver(mmpc_mod, tmp_path, model, N, kkt_solver=2, hessian=mmpc_mod.HESSIAN_GAUSS_NEWTON,
                init_states=mmpc_mod.INIT_ZERO).solve_batch_host(x0, up, tr, w)
    assert _rel(r["V"], g["V"]).max() <= 1e-6


def test_group_exact_exo_vs_oracle(mmpc_mod, oracle, tmp_path):
    """the exo on the 16-lane kernel (N <= 24 fits its LDS) with the exact Hessian (its lane-distributed W path)"""
    N, B = 20, 70
    x0, up, tr = oracle.synth(7, 3, B, N, H, model=oracle.EXO)
    s = _solver(mmpc_mod, tmp_path, "exo_arm", N, kkt_solver=3, hessian=mmpc_mod.HESSIAN_EXACT,
                init_states=mmpc_mod.INIT_ZERO)
    r = s.solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO, hessian=oracle.HESS_EXACT,
                           kkt=oracle.KKT_RICCATI, init_states=2)
    assert (r["status"] == 0).all()
    _compare(r, o)


def test_exact_hessian_policy(mmpc_mod, tmp_path):
    """AUTO keeps Gauss-Newton for the exo (more iterations exact), on the lane kernel and for bounded
    solves; an explicit EXACT is honoured on the lane kernel with and without control bounds (round 5) and with state
    bounds (round 6), and refused with the fp32 factor."""
    s = _solver(mmpc_mod, tmp_path, "exo_arm", 50)
    assert s.hessian_for(65536, False) == mmpc_mod.HESSIAN_GAUSS_NEWTON
    e = _solver(mmpc_mod, tmp_path, "exo_arm", 50, kkt_solver=2, hessian=mmpc_mod.HESSIAN_EXACT)
    assert e.hessian_for(64, False) == mmpc_mod.HESSIAN_EXACT
    assert e.hessian_for(64, True) == mmpc_mod.HESSIAN_EXACT
    f = _solver(mmpc_mod, tmp_path, "exo_arm", 50, kkt_solver=2, hessian=mmpc_mod.HESSIAN_EXACT, factor_fp32=1)
    with pytest.raises(mmpc_mod.MmpcError):
        f.hessian_for(64, False)
    e.set_state_bounds([-np.inf] * 4 + [-1.5] * 4, [np.inf] * 4 + [1.5] * 4)
    assert e.hessian_for(64, False) == mmpc_mod.HESSIAN_EXACT
    assert s.hessian_for(64, False) == mmpc_mod.HESSIAN_GAUSS_NEWTON
    t = _solver(mmpc_mod, tmp_path, "two_link_arm", 30, kkt_solver=2)
    assert t.hessian_for(64, False) == mmpc_mod.HESSIAN_GAUSS_NEWTON
    assert _solver(mmpc_mod, tmp_path, "two_link_arm", 30, kkt_solver=2).hessian_for(64, True) == \
        mmpc_mod.HESSIAN_GAUSS_NEWTON


@pytest.mark.parametrize("model,N,B,ub", [("exo_arm", 50, 128, 0.5), ("exo_arm", 7, 65, 0.6), ("two_link_arm", 30, 128, 2.0)])
def test_lane_exact_bounded_vs_oracle(model, N, B, ub, mmpc_mod, oracle, tmp_path):
    """control bounds with the exact Hessian on the lane kernel (round 5) against the oracle's projected SQP with
    ORACLE_HESS_EXACT (dense condensed, held controls fixed in the exact QP, Gauss-Newton for the rest of an iteration
    whose exact QP is not positive definite); the bounds are active on most instances"""
    om = oracle.EXO if model == "exo_arm" else oracle.TWO_LINK
    w = W_EXO if model == "exo_arm" else np.array(WEIGHTS_CFG)
    nu = 4 if model == "exo_arm" else 2
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=om)
    lb, ub_ = np.full(nu, -ub), np.full(nu, ub)
    s = _solver(mmpc_mod, tmp_path, model, N, kkt_solver=2, hessian=mmpc_mod.HESSIAN_EXACT,
                init_states=mmpc_mod.INIT_ZERO)
    assert s.kkt_solver_for(B) == 2 and s.hessian_for(B, True) == mmpc_mod.HESSIAN_EXACT
    r = s.solve_batch_host(x0, up, tr, w, u_lb=lb, u_ub=ub_)
    o = oracle.solve_batch(N, H, x0, up, tr, w, u_lb=lb, u_ub=ub_, model=om, hessian=oracle.HESS_EXACT,
                           init_states=2)
    U = r["V"][:, :N * (nu + (8 if model == "exo_arm" else 4))].reshape(B, N, -1)[:, :, -nu:]
    active = (np.abs(np.abs(U) - ub) < 1e-9).any(axis=(1, 2))
    assert active.mean() > 0.5, active.mean()
    assert (r["status"] == 0).all() and (o["status"] == 0).all()
    _compare(r, o)
    # the same KKT point as the bounded Gauss-Newton solve
    g = _solver(mmpc_mod, tmp_path, model, N, kkt_solver=2, hessian=mmpc_mod.HESSIAN_GAUSS_NEWTON,
                init_states=mmpc_mod.INIT_ZERO).solve_batch_host(x0, up, tr, w, u_lb=lb, u_ub=ub_)
    assert _rel(r["V"], g["V"]).max() <= 1e-6


@pytest.mark.parametrize("model,N,B,rscale,tscale", [("two_link_arm", 30, 256, 0.01, 20.0), ("exo_arm", 50, 128, 1.0, 20.0)])
def test_lane_exact_gauss_newton_fallback(model, N, B, rscale, tscale, mmpc_mod, oracle, tmp_path):
    """targets far from the initial state (x 20) and a small Delta-u weight: the multiplier-weighted term makes the
    exact stage QP indefinite in some iterations (the oracle counts them), which then take the Gauss-Newton step --
    the lane kernel's restart of the sweep without W, iteration for iteration the oracle's fallback"""
    om = oracle.EXO if model == "exo_arm" else oracle.TWO_LINK
    w = (W_EXO if model == "exo_arm" else np.array(WEIGHTS_CFG)).copy()
    nx, nu = (8, 4) if model == "exo_arm" else (4, 2)
    w[nx:nx + nu] *= rscale
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=om)
    tr = np.ascontiguousarray(tr * tscale)
    s = _solver(mmpc_mod, tmp_path, model, N, kkt_solver=2, hessian=mmpc_mod.HESSIAN_EXACT,
                init_states=mmpc_mod.INIT_ZERO)
    r = s.solve_batch_host(x0, up, tr, w)
    oracle.exact_fallbacks(reset=True)
    o = oracle.solve_batch(N, H, x0, up, tr, w, model=om, hessian=oracle.HESS_EXACT, kkt=oracle.KKT_RICCATI,
                           init_states=2)
    assert oracle.exact_fallbacks() > 0   # the fallback path is exercised
    assert (r["status"] == 0).all() and (o["status"] == 0).all()
    _compare(r, o)
