"""CPU: pin the oracle (oracle/mmpc_oracle.c) against the reference's own known answers and the
independent scipy solves committed in tests/golden/ (see tests/golden/make_golden.py)."""
import math

import numpy as np
import pytest

from conftest import WEIGHTS_CFG


def test_k1_f_lin_lin_test_m(golden_kat, oracle):
    """K1: lin_test.m:31-50 -- the F_lin step of ModelGenerator.cpp:47-48 reproduces the answer the
    reference authors recorded (lin_test.m:49: 0.025139, -0.025139, 12.568, -12.5677)."""
    k = golden_kat["K1"]
    A, B, xd = oracle.two_link_jac(k["x_init"], k["u_init"])
    np.testing.assert_allclose(A, k["A_init"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(B, k["B_init"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(xd, k["xdot_init"], rtol=1e-12, atol=1e-12)
    out = oracle.f_lin(k["h"], A, B, k["x"], k["u"], xd, k["x_init"], k["u_init"])
    np.testing.assert_allclose(out, k["F_lin"], rtol=1e-12, atol=1e-12)
    # the recorded 6-significant-digit answers of the reference
    np.testing.assert_allclose(out, k["recorded_standard"], rtol=0, atol=6e-4)
    looking = out - np.array(k["x_init"])
    np.testing.assert_allclose(looking, k["recorded_looking_for"], rtol=0, atol=2e-6)


def test_k2_origin(golden_kat, oracle):
    k = golden_kat["K2"]
    A, B, xd = oracle.two_link_jac(np.zeros(4), np.zeros(2))
    np.testing.assert_allclose(A, k["A"], atol=1e-14)
    np.testing.assert_allclose(B, k["B"], atol=1e-14)
    np.testing.assert_allclose(xd, k["xdot"], atol=1e-14)
    # structure recorded in SURVEY.md 4 (K2)
    np.testing.assert_allclose(B[2:], [[1, -2], [-2, 5]], atol=1e-14)
    np.testing.assert_allclose(xd, [0, 0, -9.81, 9.81], atol=1e-14)


def test_k3_random_jacobians(golden_kat, oracle):
    """K3: sympy jacobian of ex_model_generate.cpp:36-37 (itself cross-checked against the closed form
    of old/Models/DoublePendulumModel.hpp) at 12 seeded points."""
    for p in golden_kat["K3"]["points"]:
        A, B, xd = oracle.two_link_jac(p["x"], p["u"])
        np.testing.assert_allclose(A, p["A"], rtol=1e-11, atol=1e-11)
        np.testing.assert_allclose(B, p["B"], rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(xd, p["xdot"], rtol=1e-12, atol=1e-12)


def _cases(g):
    cs = g["cases"]
    return (np.array([c["x0"] for c in cs]), np.array([c["u_prev"] for c in cs]),
            np.array([c["traj"] for c in cs]), np.array([c["V"] for c in cs]), np.array([c["J"] for c in cs]))


@pytest.mark.parametrize("which", ["cfg1", "cfg2"])
def test_solve_matches_scipy(which, golden_cfg1, golden_cfg2, oracle):
    """Oracle GN-SQP vs the independent scipy single-shooting Newton solve: V* within 1e-6 relative,
    J* within 1e-8 relative."""
    g = golden_cfg1 if which == "cfg1" else golden_cfg2
    x0, up, tr, Vg, Jg = _cases(g)
    r = oracle.solve_batch(g["N"], g["h"], x0, up, tr, np.array(g["weights"]))
    assert (r["status"] == 0).all()
    rel = np.abs(r["V"] - Vg).max(1) / np.abs(Vg).max(1)
    assert rel.max() < 1e-6, rel
    np.testing.assert_allclose(r["J"], Jg, rtol=1e-8)
    assert (r["iters"] <= 10).all()


def test_solution_is_stationary(golden_cfg2, oracle):
    """At the oracle's V*, the exact single-shooting gradient (adjoint) vanishes and the multiple-shooting
    defects are zero -- a KKT certificate independent of the SQP iterates."""
    g = golden_cfg2
    x0, up, tr, _, _ = _cases(g)
    N, h, w = g["N"], g["h"], np.array(g["weights"])
    r = oracle.solve_batch(N, h, x0, up, tr, w)
    for b in range(len(x0)):
        V = r["V"][b]
        U = np.array([V[6 * k + 4:6 * k + 6] for k in range(N)])
        gr = oracle.reduced_gradient(N, h, x0[b], U, up[b], tr[b], w)
        assert np.abs(gr).max() < 1e-7
        J, defects = oracle.nlp_eval(N, h, V, up[b], tr[b], w)
        assert np.abs(defects).max() < 1e-10
        assert J == pytest.approx(r["J"][b], rel=1e-12)


def test_synth_matches_python_generator(golden_cfg2, oracle):
    """The counter-based cfg#2 generator is identical in C (oracle/HIP) and Python (make_golden.py)."""
    x0, up, tr = oracle.synth(20250213, 0, 16, 30, 0.002)
    gx, gu, gt, _, _ = _cases(golden_cfg2)
    np.testing.assert_array_equal(x0, gx)
    np.testing.assert_array_equal(up, gu)
    np.testing.assert_allclose(tr, gt, rtol=0, atol=1e-15)


def test_shard_invariance_of_generator(oracle):
    a = oracle.synth(7, 0, 64, 30, 0.002)
    b1 = oracle.synth(7, 0, 32, 30, 0.002)
    b2 = oracle.synth(7, 32, 32, 30, 0.002)
    for full, p1, p2 in zip(a, b1, b2):
        np.testing.assert_array_equal(full, np.concatenate([p1, p2]))


def test_warm_start_is_fixed_point(oracle):
    x0, up, tr = oracle.synth(20250213, 100, 8, 30, 0.002)
    w = np.array(WEIGHTS_CFG)
    r1 = oracle.solve_batch(30, 0.002, x0, up, tr, w)
    r2 = oracle.solve_batch(30, 0.002, x0, up, tr, w, V=r1["V"])
    assert (r2["iters"] == 0).all() and (r2["status"] == 0).all()
    np.testing.assert_array_equal(r1["V"], r2["V"])


def test_linear_mode_single_iteration(oracle):
    """is_linear (ModelGenerator.cpp:137-198): F_lin is affine, so GN-SQP is exact in one step."""
    x0, up, tr = oracle.synth(3, 0, 8, 25, 0.002)
    r = oracle.solve_batch(25, 0.002, x0, up, tr, np.array(WEIGHTS_CFG), is_linear=True)
    assert (r["status"] == 0).all() and (r["iters"] == 1).all()


def test_bounds_enforced(oracle):
    """u bounds are enforced (projected GN-SQP, tests/test_oracle_bounds.py); status 5 is never produced"""
    x0, up, tr = oracle.synth(20250213, 0, 4, 30, 0.002)
    w = np.array(WEIGHTS_CFG)
    r = oracle.solve_batch(30, 0.002, x0, up, tr, w)
    umax = np.abs(r["V"][:, [6 * k + 4 + c for k in range(30) for c in range(2)]]).max()
    loose = oracle.solve_batch(30, 0.002, x0, up, tr, w, u_lb=[-1e31, -1e31], u_ub=[2 * umax, 2 * umax])
    assert (loose["status"] == 0).all()
    np.testing.assert_array_equal(loose["V"], r["V"])     # inactive bounds: the unconstrained iterates
    tight = oracle.solve_batch(30, 0.002, x0, up, tr, w, u_lb=[-1e-3, -1e-3], u_ub=[1e-3, 1e-3])
    assert (tight["status"] == 0).all()
    assert np.abs(tight["V"][:, [6 * k + 4 + c for k in range(30) for c in range(2)]]).max() <= 1e-3


def test_nonfinite_input(oracle):
    x0, up, tr = oracle.synth(1, 0, 2, 30, 0.002)
    x0[1, 0] = math.nan
    r = oracle.solve_batch(30, 0.002, x0, up, tr, np.array(WEIGHTS_CFG))
    assert r["status"][0] == 0 and r["status"][1] == 3


def test_two_link_hessian_vs_finite_differences(oracle):
    """oracle_two_link_hess (hyper-dual second-order forward mode) vs central differences of the analytic
    Jacobian (K3-pinned), and symmetry."""
    rng = np.random.default_rng(1)
    for _ in range(10):
        x = rng.uniform(-1.5, 1.5, 4)
        u = rng.uniform(-5, 5, 2)
        lam = rng.normal(size=4)
        W = oracle.two_link_hess(x, u, lam)
        z = np.concatenate([x, u])
        fd = np.zeros((6, 6))
        for j in range(6):
            zp, zm = z.copy(), z.copy()
            zp[j] += 1e-6
            zm[j] -= 1e-6
            Ap, Bp, _ = oracle.two_link_jac(zp[:4], zp[4:])
            Am, Bm, _ = oracle.two_link_jac(zm[:4], zm[4:])
            fd[:, j] = lam @ ((np.hstack([Ap, Bp]) - np.hstack([Am, Bm])) / 2e-6)
        assert np.abs(W - fd).max() <= 1e-7 * max(1.0, np.abs(W).max())
        np.testing.assert_array_equal(W, W.T)


def test_exact_hessian_same_kkt_point_fewer_iterations(oracle):
    """ORACLE_HESS_EXACT (the Lagrangian Hessian, IPOPT's default) reaches the Gauss-Newton KKT point (to the stop
    test's accuracy) in fewer SQP iterations on cfg#2 instances; every instance converged."""
    N, h = 30, 0.002
    x0, up, tr = oracle.synth(20250213, 0, 512, N, h)
    w = np.array(WEIGHTS_CFG)
    gn = oracle.solve_batch(N, h, x0, up, tr, w)
    ex = oracle.solve_batch(N, h, x0, up, tr, w, hessian=oracle.HESS_EXACT)
    assert (gn["status"] == 0).all() and (ex["status"] == 0).all()
    assert ex["iters"].max() < gn["iters"].max() and ex["iters"].mean() < gn["iters"].mean() - 0.5
    rel = np.abs(ex["V"] - gn["V"]).max(1) / np.abs(gn["V"]).max(1)
    assert rel.max() < 1e-6
    for b in range(0, 512, 97):   # exact single-shooting stationarity of the exact-Hessian solutions
        U = ex["V"][b].reshape(-1)[[6 * k + 4 + c for k in range(N) for c in range(2)]]
        assert np.abs(oracle.reduced_gradient(N, h, x0[b], U, up[b], tr[b], w)).max() < 1e-7


def test_first_iteration_filter_rule(oracle):
    """IPOPT's first-iteration filter (Waechter & Biegler 2006, eqs. (18)-(21)): far from feasible (the cold start,
    theta_0 > theta_min = 1e-4 max(1, theta_0)) a trial that lowers J sufficiently is taken even when |c|_1 rises
    (up to theta_max); nearly feasible (a warm start) with the switching condition alpha (-dJ)^2.3 > theta_0^1.1
    met, it is not -- the Armijo test alone decides that iteration."""
    import ctypes as C
    f = oracle.lib().oracle_first_iter_filter_accepts
    f.argtypes = [C.c_double] * 6
    f.restype = C.c_int
    # cold start: theta_0 = 5
    assert f(100.0, 5.0, 90.0, 7.0, -50.0, 1.0) == 1     # J decreased, theta rose within theta_max
    assert f(100.0, 5.0, 101.0, 4.0, -50.0, 1.0) == 1    # theta decreased
    assert f(100.0, 5.0, 101.0, 6.0, -50.0, 1.0) == 0    # neither
    assert f(100.0, 5.0, 10.0, 6e4, -50.0, 1.0) == 0     # beyond theta_max = 1e4 max(1, theta_0)
    assert f(100.0, 5.0, math.nan, 1.0, -50.0, 1.0) == 0
    # warm start: theta_0 = 1e-9 <= theta_min and the switching condition holds -> f-type (Armijo only)
    assert f(100.0, 1e-9, 90.0, 1e-3, -50.0, 1.0) == 0
    assert f(100.0, 1e-9, 90.0, 1e-3, -50.0, 2.0 ** -20) == 0
    # nearly feasible but no descent direction for J: the switching condition fails, the filter test applies
    assert f(100.0, 1e-9, 90.0, 1e-3, 0.0, 1.0) == 1


def test_warm_start_perturbed_first_step_keeps_feasibility(oracle):
    """The reference's steady-state tick: warm start from the previous solution with a slightly moved measured
    state (ModelControl.cpp:144-145,160-161).  theta_0 is then tiny, so the first iteration is an Armijo
    (f-type) one: the accepted step must not increase the constraint violation, and the solve converges."""
    N, h = 30, 0.002
    x0, up, tr = oracle.synth(20250213, 300, 64, N, h)
    w = np.array(WEIGHTS_CFG)
    r1 = oracle.solve_batch(N, h, x0, up, tr, w, hessian=oracle.HESS_EXACT)
    assert (r1["status"] == 0).all()
    rng = np.random.default_rng(5)
    x0p = x0 + rng.uniform(-1e-7, 1e-7, x0.shape)
    Vw = r1["V"].copy()
    Vw[:, :4] = x0p
    one = oracle.solve_batch(N, h, x0p, up, tr, w, V=Vw, max_iter=1, hessian=oracle.HESS_EXACT)
    for b in range(len(x0)):
        _, c0 = oracle.nlp_eval(N, h, Vw[b], up[b], tr[b], w)
        _, c1 = oracle.nlp_eval(N, h, one["V"][b], up[b], tr[b], w)
        assert np.abs(c0).sum() <= 1e-4           # nearly feasible: theta_0 <= theta_min
        assert np.abs(c1).sum() <= np.abs(c0).sum()
    full = oracle.solve_batch(N, h, x0p, up, tr, w, V=Vw, hessian=oracle.HESS_EXACT)
    assert (full["status"] == 0).all() and full["iters"].max() <= 3


@pytest.mark.parametrize("model,hess", [("two_link", "gn"), ("two_link", "exact"), ("exo", "gn")])
def test_riccati_restatement_equals_dense(model, hess, oracle):
    """ORACLE_KKT_RICCATI (the kernels' Riccati recursion on s_k = [dx_k; du_{k-1}], the CPU baseline's
    same-algorithm leg) solves the same QP as the dense condensed Cholesky: identical iteration counts and
    statuses, V* within 1e-10 relative (same algorithm)."""
    if model == "exo":
        N, m, w, B = 50, oracle.EXO, np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4), 48
    else:
        N, m, w, B = 30, oracle.TWO_LINK, np.array(WEIGHTS_CFG), 256
    hs = oracle.HESS_EXACT if hess == "exact" else oracle.HESS_GAUSS_NEWTON
    x0, up, tr = oracle.synth(20250213, 0, B, N, 0.002, model=m)
    d = oracle.solve_batch(N, 0.002, x0, up, tr, w, model=m, hessian=hs, init_states=2)
    r = oracle.solve_batch(N, 0.002, x0, up, tr, w, model=m, hessian=hs, init_states=2, kkt=oracle.KKT_RICCATI)
    assert (d["status"] == 0).all()
    np.testing.assert_array_equal(r["status"], d["status"])
    np.testing.assert_array_equal(r["iters"], d["iters"])
    rel = np.abs(r["V"] - d["V"]).max(1) / np.abs(d["V"]).max(1)
    assert rel.max() <= 1e-10, rel.max()
