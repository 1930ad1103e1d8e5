"""CPU: state bounds (x_k in [x_min, x_max] for k >= 1; ModelControl.cpp:37-50,146-157).

The oracle's primal-dual interior-point variant (oracle/mmpc_oracle.c solve_one_ip) against the
independent scipy SLSQP solves of tests/golden/xbounds_golden.json (single-shooting form, state bounds as
inequality constraints, polished to a KKT point): V* within 1e-6 relative, J* within 1e-8 relative, the same
active state bounds, every returned state inside its box.  Plus: the interior-point path reduces to the
unbounded solution when the bounds are inactive, and control bounds alone still take the projected method.
"""
import numpy as np
import pytest

from conftest import load_golden


@pytest.fixture(scope="module")
def golden():
    return load_golden("xbounds_golden.json")


def states(V, N, nx, nu):
    return np.array([V[k * (nx + nu):k * (nx + nu) + nx] for k in range(1, N + 1)])


def test_oracle_state_bounds_match_scipy(golden, oracle):
    h = golden["h"]
    for case in golden["cases"]:
        model = oracle.EXO if case["model"] == "exo_arm" else oracle.TWO_LINK
        nx, nu = oracle.DIMS[model]
        N = case["N"]
        r = oracle.solve_batch(N, h, np.array(case["x0"])[None], np.array(case["u_prev"])[None],
                               np.array(case["traj"])[None], np.array(case["weights"]),
                               u_lb=np.array(case["u_lb"]), u_ub=np.array(case["u_ub"]), x_lb=np.array(case["x_lb"]),
                               x_ub=np.array(case["x_ub"]), max_iter=200, model=model)
        assert r["status"][0] == 0, (case["index"], r["status"], r["iters"])
        V, Vg = r["V"][0], np.array(case["V"])
        assert np.abs(V - Vg).max() / np.abs(Vg).max() < 1e-6, (case["index"], np.abs(V - Vg).max())
        assert abs(r["J"][0] - case["J"]) / case["J"] < 1e-8
        X = states(V, N, nx, nu)
        xl, xu = np.array(case["x_lb"]), np.array(case["x_ub"])
        assert (X >= xl - 1e-12).all() and (X <= xu + 1e-12).all()
        Xg = states(Vg, N, nx, nu)
        act_g = (np.abs(Xg - xl) < 1e-9) | (np.abs(Xg - xu) < 1e-9)
        act = (np.abs(X - xl) < 1e-6) | (np.abs(X - xu) < 1e-6)
        assert act_g.sum() == case["n_active_x"] and (act == act_g).all()


def test_inactive_state_bounds_reduce_to_unbounded(oracle):
    N, h = 30, 0.002
    x0, up, tr = oracle.synth(20250213, 0, 16, N, h)
    w = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
    a = oracle.solve_batch(N, h, x0, up, tr, w)
    b = oracle.solve_batch(N, h, x0, up, tr, w, x_lb=np.full(4, -50.0), x_ub=np.full(4, 50.0), max_iter=100)
    assert (a["status"] == 0).all() and (b["status"] == 0).all()
    assert (b["iters"] > a["iters"]).all()  # the barrier path takes its own iterations ...
    assert np.abs(a["V"] - b["V"]).max() / np.abs(a["V"]).max() < 1e-7  # ... to the same solution


def test_infinite_state_bounds_keep_projected_method(oracle):
    N, h = 30, 0.002
    x0, up, tr = oracle.synth(20250213, 0, 8, N, h)
    w = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
    lb, ub = np.array([-2.0, -2.0]), np.array([2.0, 2.0])
    a = oracle.solve_batch(N, h, x0, up, tr, w, u_lb=lb, u_ub=ub)
    b = oracle.solve_batch(N, h, x0, up, tr, w, u_lb=lb, u_ub=ub, x_lb=np.full(4, -1e31), x_ub=np.full(4, 1e31))
    assert np.array_equal(a["V"], b["V"]) and np.array_equal(a["iters"], b["iters"])


@pytest.mark.parametrize("rule", [1, 2])
def test_oracle_mehrotra_rules_same_kkt_point(rule, golden, oracle):
    """The round-5 barrier-rule experiment: Mehrotra's predictor-corrector (rule 1) and its probing
    without the corrector term (rule 2) reach the scipy golden KKT points like the monotone rule, and on 256
    velocity-bounded cfg#2 instances with fewer iterations (the measured means: 13.4 monotone, 9.0 / 10.0)."""
    h = golden["h"]
    try:
        oracle.set_ip_rule(rule)
        for case in golden["cases"]:
            model = oracle.EXO if case["model"] == "exo_arm" else oracle.TWO_LINK
            r = oracle.solve_batch(case["N"], h, np.array(case["x0"])[None], np.array(case["u_prev"])[None],
                                   np.array(case["traj"])[None], np.array(case["weights"]),
                                   u_lb=np.array(case["u_lb"]), u_ub=np.array(case["u_ub"]),
                                   x_lb=np.array(case["x_lb"]), x_ub=np.array(case["x_ub"]), max_iter=200, model=model)
            assert r["status"][0] == 0, (case["index"], r["status"], r["iters"])
            Vg = np.array(case["V"])
            assert np.abs(r["V"][0] - Vg).max() / np.abs(Vg).max() < 1e-6, case["index"]
        B, N = 256, 30
        x0, up, tr = oracle.synth(20250213, 0, B, N, 0.002)
        w = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
        xl, xu = np.array([-np.inf, -np.inf, -1.5, -1.5]), np.array([np.inf, np.inf, 1.5, 1.5])
        m = oracle.solve_batch(N, 0.002, x0, up, tr, w, x_lb=xl, x_ub=xu, init_states=2)
        oracle.set_ip_rule(0)
        b = oracle.solve_batch(N, 0.002, x0, up, tr, w, x_lb=xl, x_ub=xu, init_states=2)
        assert (m["status"] == 0).all() and (b["status"] == 0).all()
        assert m["iters"].mean() < 0.85 * b["iters"].mean()
        assert (np.abs(m["V"] - b["V"]).max(1) / np.abs(b["V"]).max(1)).max() < 1e-5
    finally:
        oracle.set_ip_rule(0)


def test_oracle_state_bounds_exact_hessian_match_scipy(golden, oracle):
    """VERDICT r5 ask 4: IPOPT runs CasADi's nlp_hess_l whatever the bounds (ModelGenerator.cpp:232,238; x bounds
    through v_min/v_max, ModelControl.cpp:37-50,156-157).  The interior-point oracle with the exact Lagrangian Hessian
    (the barrier Newton matrix + the condensed W_k terms; Gauss-Newton step when not positive definite) reaches the
    same scipy golden KKT points as the Gauss-Newton one (V* 1e-6, J* 1e-8, the same active state bounds)."""
    h = golden["h"]
    try:
        oracle.lib().oracle_set_hessian(oracle.HESS_EXACT)
        for case in golden["cases"]:
            model = oracle.EXO if case["model"] == "exo_arm" else oracle.TWO_LINK
            nx, nu = oracle.DIMS[model]
            N = case["N"]
            args = (N, h, np.array(case["x0"])[None], np.array(case["u_prev"])[None], np.array(case["traj"])[None],
                    np.array(case["weights"]))
            kw = dict(u_lb=np.array(case["u_lb"]), u_ub=np.array(case["u_ub"]), x_lb=np.array(case["x_lb"]),
                      x_ub=np.array(case["x_ub"]), max_iter=200, model=model, hessian=oracle.HESS_EXACT)
            r = oracle.solve_batch(*args, **kw)
            assert r["status"][0] == 0, (case["index"], r["status"], r["iters"])
            V, Vg = r["V"][0], np.array(case["V"])
            assert np.abs(V - Vg).max() / np.abs(Vg).max() < 1e-6, (case["index"], np.abs(V - Vg).max())
            assert abs(r["J"][0] - case["J"]) / case["J"] < 1e-8
            X = states(V, N, nx, nu)
            xl, xu = np.array(case["x_lb"]), np.array(case["x_ub"])
            Xg = states(Vg, N, nx, nu)
            act_g = (np.abs(Xg - xl) < 1e-9) | (np.abs(Xg - xu) < 1e-9)
            act = (np.abs(X - xl) < 1e-6) | (np.abs(X - xu) < 1e-6)
            assert (act == act_g).all()
    finally:
        oracle.lib().oracle_set_hessian(oracle.HESS_GAUSS_NEWTON)


def test_oracle_state_bounds_exact_vs_gauss_newton_iterations(oracle):
    """Iteration histograms of the interior-point solve with both Hessians on 256 velocity-bounded cfg#2 instances
    (|qdot| <= 1.5): the same KKT points (1e-6), every instance converged with both."""
    N, h, B = 30, 0.002, 256
    x0, up, tr = oracle.synth(20250213, 0, B, N, h)
    w = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
    xl, xu = np.array([-np.inf, -np.inf, -1.5, -1.5]), np.array([np.inf, np.inf, 1.5, 1.5])
    gn = oracle.solve_batch(N, h, x0, up, tr, w, x_lb=xl, x_ub=xu)
    oracle.exact_fallbacks(reset=True)
    ex = oracle.solve_batch(N, h, x0, up, tr, w, x_lb=xl, x_ub=xu, hessian=oracle.HESS_EXACT)
    assert (gn["status"] == 0).all() and (ex["status"] == 0).all()
    rel = np.abs(gn["V"] - ex["V"]).max(1) / np.abs(gn["V"]).max(1)
    assert rel.max() < 1e-6
    print("GN", np.bincount(gn["iters"]), gn["iters"].mean(), "EXACT", np.bincount(ex["iters"]), ex["iters"].mean(),
          "fallbacks", oracle.exact_fallbacks(reset=True))
