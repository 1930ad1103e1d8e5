"""GPU: box-constrained controls (SURVEY.md 8a A1 bounds, ModelControl.cpp:37-50,146-157; 8f rank 1) on all
three KKT solvers, through the C-ABI.

The kernels run the oracle's projected SQP (oracle/mmpc_oracle.c solve_one; sqp_wave.h "box constraints") with
the Hessian the solver resolves (mmpc_resolve_hessian: exact on the 16-lane group kernel, Gauss-Newton elsewhere);
every oracle comparison runs that same Hessian (oracle_lib.solve_batch(solver=s)).  Tolerances:
  * vs the scipy bounded golden (independent solver, tests/golden/make_golden_bounds.py): V* within 1e-8
    relative, identical active sets, every control inside its box exactly;
  * vs the oracle (same algorithm): as test_gpu_parity._compare (V* 1e-10 where iteration counts agree);
    the Riccati solvers solve the same equality-constrained QPs by a different factorisation, 1e-8;
  * infinite bounds through the host API select the unbounded kernels: bitwise the unbounded result.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, WEIGHTS_CFG
from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu

H = 0.002
W_EXO = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
SOLVERS_2L = ["condensed", "riccati", "group"]


@pytest.fixture(scope="module")
def bounds_golden():
    return json.load(open(os.path.join(GOLDEN, "bounds_golden.json")))


def _kkt(mmpc_mod, name):
    return {"condensed": mmpc_mod.KKT_CONDENSED, "riccati": mmpc_mod.KKT_RICCATI,
            "group": mmpc_mod.KKT_RICCATI_GROUP}[name]


def _solver(tmp_path, mmpc_mod, model, N, kkt, **kw):
    nx, nu = (8, 4) if model == "exo_arm" else (4, 2)
    p = mmpc_mod.write_model_json(str(tmp_path / f"{model}_{N}_{kkt}.json"), "b", nx, nu, 2000, N, model=model)
    return mmpc_mod.Solver(p, kkt_solver=kkt, **kw)


def _u(V, N, nx, nu):
    V = np.asarray(V)
    return np.stack([V[..., (nx + nu) * k + nx:(nx + nu) * (k + 1)] for k in range(N)], axis=-2)


@pytest.mark.parametrize("solver", SOLVERS_2L)
def test_bounded_vs_scipy_golden(solver, bounds_golden, mmpc_mod, tmp_path):
    for c in bounds_golden["cases"]:
        if c["model"] == "exo_arm" and solver == "condensed":
            continue
        nx, nu = (8, 4) if c["model"] == "exo_arm" else (4, 2)
        N = c["N"]
        s = _solver(tmp_path, mmpc_mod, c["model"], N, _kkt(mmpc_mod, solver))
        r = s.solve_batch_host(np.array([c["x0"]]), np.array([c["u_prev"]]), np.array([c["traj"]]),
                               np.array(c["weights"]), u_lb=c["u_lb"], u_ub=c["u_ub"])
        assert r["status"][0] == 0, (solver, c["model"], c["index"])
        V, Vg = r["V"][0], np.array(c["V"])
        assert np.abs(V - Vg).max() <= 1e-8 * np.abs(Vg).max(), (solver, c["model"], c["index"])
        U, Ug = _u(V, N, nx, nu), _u(Vg, N, nx, nu)
        lb, ub = np.array(c["u_lb"]), np.array(c["u_ub"])
        assert ((U >= lb) & (U <= ub)).all()
        np.testing.assert_array_equal((U == lb) | (U == ub), (Ug == lb) | (Ug == ub))


@pytest.mark.parametrize("solver", SOLVERS_2L)
@pytest.mark.parametrize("bound", [10.0, 2.0, 1e-3])
def test_bounded_two_link_vs_oracle(solver, bound, mmpc_mod, oracle, tmp_path):
    N, B = 30, 256
    x0, up, tr = oracle.synth(20250213, 500, B, N, H)
    w = np.array(WEIGHTS_CFG)
    lb, ub = [-bound, -0.8 * bound], [0.9 * bound, bound]
    s = _solver(tmp_path, mmpc_mod, "two_link_arm", N, _kkt(mmpc_mod, solver))
    r = s.solve_batch_host(x0, up, tr, w, u_lb=lb, u_ub=ub)
    o = oracle.solve_batch(N, H, x0, up, tr, w, u_lb=lb, u_ub=ub, solver=s)   # the Hessian s resolves (exact: group)
    assert (o["status"] == 0).all()
    _compare(r, o)   # V* within 1e-10 (measured <= 1.2e-15, profiles/r02/gpu_vs_oracle_agreement_v1.log)
    U = _u(r["V"], N, 4, 2)
    assert (U >= np.array(lb)).all() and (U <= np.array(ub)).all()


@pytest.mark.parametrize("solver,N,B", [("riccati", 50, 256), ("group", 20, 130)])
def test_bounded_exo_vs_oracle(solver, N, B, mmpc_mod, oracle, tmp_path):
    x0, up, tr = oracle.synth(20250213, 900, B, N, H, model=oracle.EXO)
    lb, ub = [-0.5, -1.0, -0.5, -0.3], [0.6, 0.5, 1.0, 0.3]
    s = _solver(tmp_path, mmpc_mod, "exo_arm", N, _kkt(mmpc_mod, solver))
    r = s.solve_batch_host(x0, up, tr, W_EXO, u_lb=lb, u_ub=ub)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, u_lb=lb, u_ub=ub, model=oracle.EXO, solver=s)
    assert (o["status"] == 0).all()
    _compare(r, o)


@pytest.mark.parametrize("solver", SOLVERS_2L)
def test_infinite_bounds_select_the_unbounded_path(solver, mmpc_mod, oracle, tmp_path):
    N = 30
    x0, up, tr = oracle.synth(3, 0, 64, N, H)
    w = np.array(WEIGHTS_CFG)
    s = _solver(tmp_path, mmpc_mod, "two_link_arm", N, _kkt(mmpc_mod, solver))
    r0 = s.solve_batch_host(x0, up, tr, w)
    r1 = s.solve_batch_host(x0, up, tr, w, u_lb=[-1e31, -1e31], u_ub=[1e31, 1e20])  # reference defaults
    np.testing.assert_array_equal(r0["V"], r1["V"])
    np.testing.assert_array_equal(r0["iters"], r1["iters"])


@pytest.mark.parametrize("solver", SOLVERS_2L)
def test_bounded_kernel_with_infinite_device_bounds(solver, mmpc_mod, oracle, tmp_path):
    """device pointers always select the bounded kernels; with infinite bounds they solve the unbounded NLP"""
    import torch
    N, B = 30, 64
    x0, up, tr = oracle.synth(4, 0, B, N, H)
    w = np.array(WEIGHTS_CFG)
    s = _solver(tmp_path, mmpc_mod, "two_link_arm", N, _kkt(mmpc_mod, solver))
    f = dict(dtype=torch.float64, device="cuda")
    t = [torch.tensor(a, **f) for a in (x0, up, tr, w)]
    V = torch.zeros((B, s.NV), **f)
    st = torch.zeros(B, dtype=torch.int32, device="cuda")
    lb = torch.tensor([-1e31, -np.inf], **f)
    ub = torch.tensor([np.inf, 1e31], **f)
    s.solve_batch(B, *t, V, st, None, None, u_lb=lb, u_ub=ub)
    torch.cuda.synchronize()
    o = oracle.solve_batch(N, H, x0, up, tr, w, solver=s)
    assert (st.cpu().numpy() == 0).all()
    assert np.abs(V.cpu().numpy() - o["V"]).max() <= 1e-8 * np.abs(o["V"]).max()


@pytest.mark.parametrize("solver", SOLVERS_2L)
def test_warm_start_outside_the_box(solver, mmpc_mod, oracle, tmp_path):
    N = 30
    x0, up, tr = oracle.synth(9, 0, 16, N, H)
    w = np.array(WEIGHTS_CFG)
    V = np.zeros((16, 6 * N + 4))
    V[:, [6 * k + 4 for k in range(N)]] = 50.0
    V[:, [6 * k + 5 for k in range(N)]] = np.nan   # a NaN control is not silently projected
    lb, ub = [-2, -2], [2, 2]
    s = _solver(tmp_path, mmpc_mod, "two_link_arm", N, _kkt(mmpc_mod, solver))
    r = s.solve_batch_host(x0, up, tr, w, V=V, u_lb=lb, u_ub=ub)
    o = oracle.solve_batch(N, H, x0, up, tr, w, V=V, u_lb=lb, u_ub=ub, solver=s)
    np.testing.assert_array_equal(r["status"], o["status"])
    assert (r["status"] == 3).all()
    V[:, [6 * k + 5 for k in range(N)]] = -40.0
    r = s.solve_batch_host(x0, up, tr, w, V=V, u_lb=lb, u_ub=ub)
    ref = oracle.solve_batch(N, H, x0, up, tr, w, u_lb=lb, u_ub=ub, solver=s)
    assert (r["status"] == 0).all()
    assert np.abs(r["V"] - ref["V"]).max() <= 1e-8 * np.abs(ref["V"]).max()


def test_bounded_cfg3_batch_properties(mmpc_mod, oracle, tmp_path):
    """cfg#3 shape with torque limits (B = 16384): all converge, feasible, KKT (projected gradient) on samples"""
    import torch
    N, B = 50, 16384
    s = _solver(tmp_path, mmpc_mod, "exo_arm", N, mmpc_mod.KKT_RICCATI)
    f = dict(dtype=torch.float64, device="cuda")
    x0 = torch.empty((B, 8), **f); up = torch.empty((B, 4), **f); tr = torch.empty((B, N, 8), **f)
    s.synth(20250213, 0, B, x0, up, tr)
    lbn, ubn = np.array([-1.0] * 4), np.array([1.0] * 4)
    V = torch.zeros((B, s.NV), **f)
    st = torch.zeros(B, dtype=torch.int32, device="cuda")
    s.solve_batch(B, x0, up, tr, torch.tensor(W_EXO, **f), V, st, None, None,
                  u_lb=torch.tensor(lbn, **f), u_ub=torch.tensor(ubn, **f))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    Vn = V.cpu().numpy()
    U = _u(Vn, N, 8, 4)
    assert (U >= -1.0).all() and (U <= 1.0).all()
    assert ((U == -1.0) | (U == 1.0)).any()
    x0n, upn, trn = x0.cpu().numpy(), up.cpu().numpy(), tr.cpu().numpy()
    for b in range(0, B, 2048):
        g = oracle.reduced_gradient(N, H, x0n[b], U[b], upn[b], trn[b], W_EXO, model=oracle.EXO).reshape(-1)
        u = U[b].reshape(-1)
        assert np.abs(u - np.clip(u - g, np.tile(lbn, N), np.tile(ubn, N))).max() <= 1e-7


def test_rank0_batch_api_single_process(mmpc_mod, oracle, tmp_path):
    """mmpc.dist.solve_rank0_batch on one GPU without a process group (the N>1 plumbing is tested on gloo in
    tests/test_distributed.py): same result as the host API"""
    import torch
    from mmpc import dist as mdist
    N, B = 30, 100
    x0, up, tr = oracle.synth(21, 0, B, N, H)
    s = _solver(tmp_path, mmpc_mod, "two_link_arm", N, mmpc_mod.KKT_AUTO)
    f = dict(dtype=torch.float64, device="cuda")
    r = mdist.solve_rank0_batch(s, torch.tensor(x0, **f), torch.tensor(up, **f), torch.tensor(tr, **f),
                                weights=torch.tensor(WEIGHTS_CFG, **f), u_lb=torch.tensor([-2.0, -2.0], **f),
                                u_ub=torch.tensor([2.0, 2.0], **f), device="cuda")
    h = s.solve_batch_host(x0, up, tr, np.array(WEIGHTS_CFG), u_lb=[-2.0, -2.0], u_ub=[2.0, 2.0])
    np.testing.assert_array_equal(r["V"].cpu().numpy(), h["V"])
    np.testing.assert_array_equal(r["status"].cpu().numpy(), h["status"])


@pytest.mark.parametrize("bound", [2.0, 1e-3])
def test_bounded_exact_hessian_vs_oracle(bound, mmpc_mod, oracle, tmp_path):
    """mmpc_opts.hessian = EXACT with control bounds (the group kernel's BOUNDED + EXACT instantiation): the held
    controls are fixed in the exact QP, as the oracle's solve_one (oracle_set_exact_bounded); same iterates."""
    N, B = 30, 256
    x0, up, tr = oracle.synth(20250213, 500, B, N, H)
    w = np.array(WEIGHTS_CFG)
    lb, ub = [-bound, -0.8 * bound], [0.9 * bound, bound]
    s = _solver(tmp_path, mmpc_mod, "two_link_arm", N, mmpc_mod.KKT_RICCATI_GROUP, hessian=mmpc_mod.HESSIAN_EXACT)
    assert s.hessian_for(B, True) == mmpc_mod.HESSIAN_EXACT
    r = s.solve_batch_host(x0, up, tr, w, u_lb=lb, u_ub=ub)
    o = oracle.solve_batch(N, H, x0, up, tr, w, u_lb=lb, u_ub=ub, solver=s)
    assert (o["status"] == 0).all()
    _compare(r, o)
    U = _u(r["V"], N, 4, 2)
    assert (U >= np.array(lb)).all() and (U <= np.array(ub)).all()
