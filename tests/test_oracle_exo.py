"""Oracle checks for the exo model (SURVEY.md 8a A3b, 8d cfg#3) against the committed golden fixtures.

Parity anchors (the reference defines only M(q); parameters, gravity and damping are build-defined in
tests/golden/exo_params.json and are NOT reference-pinned):
  * exo_mass_kat.json  M(q) evaluated from the unexpanded src/inverseTest.cpp:59-74 printout (40 digits)
  * exo_golden.json    complex-step Jacobians and scipy least-squares single-shooting solutions
Tolerances are stated per test.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def mass_kat():
    return json.load(open(os.path.join(GOLDEN, "exo_mass_kat.json")))


@pytest.fixture(scope="module")
def exo_golden():
    return json.load(open(os.path.join(GOLDEN, "exo_golden.json")))


def test_mass_matrix_kat(mass_kat, oracle):
    # 1e-13 relative to max|M|: the generated polynomial vs the unexpanded printout
    assert mass_kat["min_eigenvalue_over_2000_random_q"] > 0
    for c in mass_kat["cases"]:
        M = oracle.exo_mass(np.array(c["q"]))
        Mk = np.array(c["M"])
        assert np.abs(M - Mk).max() <= 1e-13 * np.abs(Mk).max(), c["q"]
        np.testing.assert_array_equal(M, M.T)


def test_jacobian_vs_complex_step(exo_golden, oracle):
    # analytic dM/dq Jacobian vs complex-step of the unexpanded model: 1e-11 relative
    for p in exo_golden["jacobian_points"]:
        A, B, xd = oracle.exo_jac(np.array(p["x"]), np.array(p["u"]))
        for got, ref in ((A, p["A"]), (B, p["B"]), (xd, p["xdot"])):
            ref = np.array(ref)
            assert np.abs(got - ref).max() <= 1e-11 * np.abs(ref).max()


def test_synth_matches_python_generator(exo_golden, oracle):
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden_exo as mg
    x0, up, tr = oracle.synth(20250213, 0, 8, 50, 0.002, model=oracle.EXO)
    x1, u1, t1 = mg.synth_exo(20250213, 0, 8, 50, 0.002)
    np.testing.assert_array_equal(x0, x1)
    np.testing.assert_array_equal(up, u1)
    assert np.abs(tr - t1).max() <= 2e-14
    # the fixture's inputs are the generator's
    c = exo_golden["cases"][0]
    np.testing.assert_array_equal(np.array(c["x0"]), x0[0])


def test_solve_matches_scipy_golden(exo_golden, oracle):
    # same NLP, independent solver/formulation: V* within 1e-8 relative, J* within 1e-12 relative
    w = np.array(exo_golden["weights"])
    h = exo_golden["h"]
    for c in exo_golden["cases"]:
        N = c["N"]
        r = oracle.solve_batch(N, h, np.array([c["x0"]]), np.array([c["u_prev"]]), np.array([c["traj"]]), w,
                               model=oracle.EXO)
        assert r["status"][0] == 0
        V, Vg = r["V"][0], np.array(c["V"])
        assert np.abs(V - Vg).max() <= 1e-8 * np.abs(Vg).max()
        J, g = oracle.nlp_eval(N, h, V, np.array(c["u_prev"]), np.array(c["traj"]), w, model=oracle.EXO)
        assert abs(J - c["J"]) <= 1e-12 * c["J"]
        assert np.abs(g).max() <= 1e-10


def test_solution_is_stationary(oracle):
    # size-independent property: the reduced (single-shooting) gradient vanishes at the solution
    N, h = 50, 0.002
    x0, up, tr = oracle.synth(20250213, 1000, 8, N, h, model=oracle.EXO)
    w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
    r = oracle.solve_batch(N, h, x0, up, tr, w, model=oracle.EXO)
    assert (r["status"] == 0).all() and (r["iters"] <= 8).all()
    for b in range(8):
        V = r["V"][b].reshape(-1)
        U = np.array([V[12 * k + 8:12 * k + 12] for k in range(N)])
        g = oracle.reduced_gradient(N, h, x0[b], U, up[b], tr[b], w, model=oracle.EXO)
        assert np.abs(g).max() <= 1e-7


def test_linear_mode_single_iteration(oracle):
    # linear mode is one convex QP: GN-SQP converges in one step (then the stop test)
    N, h = 50, 0.002
    x0, up, tr = oracle.synth(7, 0, 4, N, h, model=oracle.EXO)
    w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
    r = oracle.solve_batch(N, h, x0, up, tr, w, model=oracle.EXO, is_linear=True)
    assert (r["status"] == 0).all() and (r["iters"] <= 2).all()


def test_exo_lagrangian_hessian_matches_jacobian_differences(oracle):
    """oracle_exo_hess (analytic: d^2 acc from M acc = w differentiated twice, symbolic dM and d^2M of
    exo_model_gen.h) equals central differences of lam^T [A | B] of the oracle's analytic exo Jacobian, and is
    symmetric (round 4: the exact-Hessian SQP on the exo, IPOPT's default nlp_hess_l, ModelGenerator.cpp:238)."""
    L = oracle.lib()
    rng = np.random.default_rng(1)
    for _ in range(10):
        x, u, lam = rng.uniform(-1, 1, 8), rng.uniform(-2, 2, 4), rng.uniform(-3, 3, 8)
        W = np.zeros(144)
        L.oracle_exo_hess(x, u, lam, W)
        W = W.reshape(12, 12)

        def g(z):
            A, B, xd = np.zeros(64), np.zeros(32), np.zeros(8)
            L.oracle_exo_jac(z[:8].copy(), z[8:].copy(), A, B, xd)
            return lam @ np.hstack([A.reshape(8, 8), B.reshape(8, 4)])
        z, h = np.concatenate([x, u]), 1e-6
        Wf = np.stack([(g(z + h * e) - g(z - h * e)) / (2 * h) for e in np.eye(12)], axis=1)
        assert np.abs(W - Wf).max() <= 1e-7 * max(1.0, np.abs(Wf).max())
        assert np.abs(W - W.T).max() <= 1e-14 * max(1.0, np.abs(W).max())
        # only the q rows/columns are nonzero past the q-q block: d^2 acc / dqd^2 = d^2 acc / dtau^2 = 0
        assert np.abs(W[4:, 4:]).max() == 0.0


def test_exo_exact_hessian_same_kkt_point(oracle):
    """Exact-Hessian SQP on the exo reaches the Gauss-Newton KKT point (the build's exo AUTO stays Gauss-Newton:
    on cfg#3 instances the exact Hessian takes more iterations)."""
    N, h = 50, 0.002
    x0, up, tr = oracle.synth(20250213, 0, 64, N, h, model=oracle.EXO)
    w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
    gn = oracle.solve_batch(N, h, x0, up, tr, w, model=oracle.EXO, init_states=2, kkt=oracle.KKT_RICCATI)
    ex = oracle.solve_batch(N, h, x0, up, tr, w, model=oracle.EXO, init_states=2, kkt=oracle.KKT_RICCATI,
                            hessian=oracle.HESS_EXACT)
    dense = oracle.solve_batch(N, h, x0, up, tr, w, model=oracle.EXO, init_states=2, hessian=oracle.HESS_EXACT)
    assert (gn["status"] == 0).all() and (ex["status"] == 0).all() and (dense["status"] == 0).all()
    scale = np.abs(gn["V"]).max(axis=1)
    assert (np.abs(ex["V"] - gn["V"]).max(axis=1) / scale).max() <= 1e-7
    # the Riccati restatement of the exact QP reproduces the dense one
    assert (ex["iters"] == dense["iters"]).all()
    assert (np.abs(ex["V"] - dense["V"]).max(axis=1) / scale).max() <= 1e-10
