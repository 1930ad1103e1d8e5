"""Oracle: box-constrained controls (SURVEY.md 8a A1 bounds, ModelControl.cpp:37-50,146-157; 8f rank 1).

The reference hands u_min/u_max to IPOPT, which returns a KKT point of the bound-constrained NLP. The oracle
(and the kernels) run a projected Gauss-Newton SQP (oracle/mmpc_oracle.c solve_one). Parity anchor:
tests/golden/bounds_golden.json, an independent scipy least_squares(trf, bounds) solve of the single-shooting
form, polished to a KKT point (make_golden_bounds.py). Tolerances: V* within 1e-8 relative, J* within 1e-12
relative, identical active sets.  Both active-set rules are checked: holds only added (the condensed and lane
kernels) and the primal-dual rule that also releases a hold whose QP multiplier points into the box (the 16-lane
Riccati kernel, bound_release).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, WEIGHTS_CFG


@pytest.fixture(scope="module")
def bounds_golden():
    return json.load(open(os.path.join(GOLDEN, "bounds_golden.json")))


def _u(V, N, nx, nu):
    return np.array([V[(nx + nu) * k + nx:(nx + nu) * (k + 1)] for k in range(N)])


@pytest.mark.parametrize("release", [False, True])
def test_bounded_solve_matches_scipy_golden(release, bounds_golden, oracle):
    h = bounds_golden["h"]
    for c in bounds_golden["cases"]:
        model = oracle.EXO if c["model"] == "exo_arm" else oracle.TWO_LINK
        nx, nu = (8, 4) if c["model"] == "exo_arm" else (4, 2)
        N = c["N"]
        r = oracle.solve_batch(N, h, np.array([c["x0"]]), np.array([c["u_prev"]]), np.array([c["traj"]]),
                               np.array(c["weights"]), u_lb=c["u_lb"], u_ub=c["u_ub"], model=model,
                               bound_release=release)
        assert r["status"][0] == 0, (c["model"], c["index"], r["status"][0])
        V, Vg = r["V"][0], np.array(c["V"])
        assert np.abs(V - Vg).max() <= 1e-8 * np.abs(Vg).max(), (c["model"], c["index"])
        J, _ = oracle.nlp_eval(N, h, V, np.array(c["u_prev"]), np.array(c["traj"]), np.array(c["weights"]),
                               model=model)
        assert abs(J - c["J"]) <= 1e-12 * c["J"]
        U, Ug = _u(V, N, nx, nu), _u(Vg, N, nx, nu)
        lb, ub = np.array(c["u_lb"]), np.array(c["u_ub"])
        assert ((U >= lb) & (U <= ub)).all()                                    # feasible exactly
        np.testing.assert_array_equal((U == lb) | (U == ub), (Ug == lb) | (Ug == ub))
        assert int(((U == lb) | (U == ub)).sum()) == c["n_active"]


@pytest.mark.parametrize("release", [False, True])
@pytest.mark.parametrize("bound", [20.0, 5.0, 1.0, 1e-3])
def test_bounded_batch_converges_to_kkt_points(bound, release, oracle):
    """size-independent properties: every instance converges, stays in the box, projected gradient ~ 0"""
    N, h = 30, 0.002
    x0, up, tr = oracle.synth(20250213, 0, 96, N, h)
    w = np.array(WEIGHTS_CFG)
    lb, ub = [-bound, -bound], [bound, bound]
    r = oracle.solve_batch(N, h, x0, up, tr, w, u_lb=lb, u_ub=ub, bound_release=release)
    assert (r["status"] == 0).all() and (r["iters"] <= 20).all()
    for b in range(0, 96, 12):
        U = _u(r["V"][b], N, 4, 2)
        assert (np.abs(U) <= bound).all()
        g = oracle.reduced_gradient(N, h, x0[b], U, up[b], tr[b], w)
        pg = np.abs(U.reshape(-1) - np.clip(U.reshape(-1) - g.reshape(-1), -bound, bound)).max()
        assert pg <= 1e-7, (b, pg)


def test_infinite_bounds_are_the_unconstrained_solve(oracle):
    x0, up, tr = oracle.synth(5, 0, 16, 30, 0.002)
    w = np.array(WEIGHTS_CFG)
    r0 = oracle.solve_batch(30, 0.002, x0, up, tr, w)
    r1 = oracle.solve_batch(30, 0.002, x0, up, tr, w, u_lb=[-1e31, -1e20], u_ub=[1e31, 1e19])
    np.testing.assert_array_equal(r0["V"], r1["V"])
    np.testing.assert_array_equal(r0["iters"], r1["iters"])


def test_warm_start_outside_the_box_is_projected(oracle):
    N, h = 30, 0.002
    x0, up, tr = oracle.synth(9, 0, 8, N, h)
    w = np.array(WEIGHTS_CFG)
    V = np.zeros((8, 6 * N + 4))
    V[:, [6 * k + 4 for k in range(N)]] = 50.0                               # far above the bound
    r = oracle.solve_batch(N, h, x0, up, tr, w, V=V, u_lb=[-2, -2], u_ub=[2, 2])
    ref = oracle.solve_batch(N, h, x0, up, tr, w, u_lb=[-2, -2], u_ub=[2, 2])
    assert (r["status"] == 0).all()
    assert np.abs(r["V"] - ref["V"]).max() <= 1e-8 * np.abs(ref["V"]).max()


def test_release_rule_shortens_the_iteration_tail(oracle):
    """cfg#2 with +-2 Nm: releasing holds whose multiplier points into the box (primal-dual active set) cuts the
    slowest instances' iterations (the batch waits for them) and reaches the same KKT points"""
    N, h, B = 30, 0.002, 512
    x0, up, tr = oracle.synth(20250213, 0, B, N, h)
    w = np.array(WEIGHTS_CFG)
    r0 = oracle.solve_batch(N, h, x0, up, tr, w, u_lb=[-2, -2], u_ub=[2, 2])
    r1 = oracle.solve_batch(N, h, x0, up, tr, w, u_lb=[-2, -2], u_ub=[2, 2], bound_release=True)
    assert (r0["status"] == 0).all() and (r1["status"] == 0).all()
    assert r1["iters"].max() < r0["iters"].max() and r1["iters"].mean() < r0["iters"].mean()
    assert np.abs(r1["V"] - r0["V"]).max() <= 1e-6 * np.abs(r0["V"]).max()
