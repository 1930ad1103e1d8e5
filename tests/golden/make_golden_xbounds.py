#!/usr/bin/env python3
"""Golden vectors for STATE bounds (x_k in [x_min, x_max] for k >= 1) -- build container only.

The reference passes x_min/x_max to IPOPT as lbx/ubx of x_1..x_N (ModelControl.cpp:37-50,146-157).  Here the same
NLP is solved independently of oracle/ and of the kernels: the SINGLE-shooting least-squares form (x_0 pinned,
states x_k(U) rolled out), with the state bounds as nonlinear inequality constraints and the control bounds as
simple bounds, by scipy SLSQP (exact objective gradient and constraint Jacobians from the forward sensitivities);
then polished by Gauss-Newton SQP on the active set SLSQP found (active state bounds as equality constraints,
active controls held).  The polished point is checked to be a KKT point: equality residual <= 1e-12,
multipliers of the right sign, inactive bounds satisfied, stationarity |grad + C^T lam| <= 1e-9.

Writes tests/golden/xbounds_golden.json: 4 two-link instances (N = 30) and 1 exo instance (N = 20).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
from scipy.optimize import minimize

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as g2  # noqa: E402
import make_golden_exo as gx  # noqa: E402


def rollout_sens(U, x0, up, tr, w, h, f, jac, nx, nu):
    """residual r, its Jacobian J (single shooting), states X and state sensitivities S_k = dx_k/dU."""
    N = tr.shape[0]
    Uk = U.reshape(N, nu)
    Q, R, Rm = w[:nx], w[nx:nx + nu], w[nx + nu:nx + 2 * nu]
    X = np.zeros((N + 1, nx)); X[0] = x0
    S = np.zeros((nx, nu * N))
    Ss = [S.copy()]
    res, rows = [], []
    for k in range(N):
        A, Bc = jac(X[k], Uk[k])
        X[k + 1] = X[k] + h * f(X[k], Uk[k])
        S = (np.eye(nx) + h * A) @ S
        S[:, nu * k:nu * k + nu] += h * Bc
        Ss.append(S.copy())
        res.append(np.sqrt(Q) * (X[k + 1] - tr[k]))
        rows.append(np.sqrt(Q)[:, None] * S)
    for k in range(N):
        um = up if k == 0 else Uk[k - 1]
        res.append(np.sqrt(R) * (Uk[k] - um))
        Jr = np.zeros((nu, nu * N)); Jr[:, nu * k:nu * k + nu] = np.diag(np.sqrt(R))
        if k > 0:
            Jr[:, nu * (k - 1):nu * k] = -np.diag(np.sqrt(R))
        rows.append(Jr)
        res.append(np.sqrt(Rm) * Uk[k])
        Jm = np.zeros((nu, nu * N)); Jm[:, nu * k:nu * k + nu] = np.diag(np.sqrt(Rm))
        rows.append(Jm)
    return np.concatenate(res), np.vstack(rows), X, Ss


def constraints(U, args, xl, xu):
    """g(U) >= 0: x_k,i - xl_i and xu_i - x_k,i for k >= 1 and finite bounds; Jacobian rows."""
    _, _, X, Ss = rollout_sens(U, *args)
    vals, rows, keys = [], [], []
    for k in range(1, X.shape[0]):
        for i in range(X.shape[1]):
            if np.isfinite(xl[i]):
                vals.append(X[k, i] - xl[i]); rows.append(Ss[k][i]); keys.append((k, i, -1))
            if np.isfinite(xu[i]):
                vals.append(xu[i] - X[k, i]); rows.append(-Ss[k][i]); keys.append((k, i, +1))
    return np.array(vals), np.array(rows), keys


def solve(x0, up, tr, w, h, f, jac, nx, nu, xl, xu, ul, uu):
    N = tr.shape[0]
    args = (x0, up, tr, w, h, f, jac, nx, nu)
    lbv, ubv = np.tile(ul, N), np.tile(uu, N)
    obj = lambda U: float(np.sum(rollout_sens(U, *args)[0] ** 2))  # noqa: E731

    def grad(U):
        r, J, _, _ = rollout_sens(U, *args)
        return 2.0 * J.T @ r

    cons = {"type": "ineq", "fun": lambda U: constraints(U, args, xl, xu)[0],
            "jac": lambda U: constraints(U, args, xl, xu)[1]}
    bnds = [(a if np.isfinite(a) else None, b if np.isfinite(b) else None) for a, b in zip(lbv, ubv)]
    sol = minimize(obj, np.clip(np.zeros(nu * N), lbv, ubv), jac=grad, bounds=bnds, constraints=[cons],
                   method="SLSQP", options=dict(maxiter=2000, ftol=1e-16))
    U = sol.x.copy()
    # polish: Gauss-Newton SQP with the active set SLSQP found as equalities
    g0, _, keys = constraints(U, args, xl, xu)
    act = [j for j, v in enumerate(g0) if v < 1e-7]
    held_u = np.where((U <= lbv + 1e-7) | (U >= ubv - 1e-7))[0]
    for _ in range(50):
        r, J, X, Ss = rollout_sens(U, *args)
        gv, C, keys = constraints(U, args, xl, xu)
        Ca = np.vstack([C[act]] + [np.eye(nu * N)[held_u]]) if (act or len(held_u)) else np.zeros((0, nu * N))
        ca = np.concatenate([gv[act], (U - np.where(U <= lbv + 1e-7, lbv, ubv))[held_u]])
        H = 2.0 * J.T @ J
        m = Ca.shape[0]
        K = np.block([[H, Ca.T], [Ca, np.zeros((m, m))]])
        rhs = np.concatenate([-2.0 * J.T @ r, -ca])
        sol_k = np.linalg.lstsq(K, rhs, rcond=None)[0]
        step, lam = sol_k[:nu * N], sol_k[nu * N:]
        U = U + step
        if np.abs(step).max() < 1e-15 * max(1.0, np.abs(U).max()):
            break
    r, J, X, Ss = rollout_sens(U, *args)
    gv, C, keys = constraints(U, args, xl, xu)
    Ca = np.vstack([C[act]] + [np.eye(nu * N)[held_u]]) if (act or len(held_u)) else np.zeros((0, nu * N))
    grad_f = 2.0 * J.T @ r
    lam = np.linalg.lstsq(Ca.T, -grad_f, rcond=None)[0] if Ca.shape[0] else np.zeros(0)
    stat = np.abs(grad_f + Ca.T @ lam).max()
    assert stat <= 1e-9, stat
    assert (lam[:len(act)] <= 1e-9).all(), lam[:len(act)]  # ineq g >= 0: grad = -C^T lam with lam <= 0
    assert gv.min() >= -1e-12, gv.min()
    Uk = U.reshape(N, nu)
    V = np.zeros(nx * (N + 1) + nu * N)
    for k in range(N):
        V[(nx + nu) * k:(nx + nu) * k + nx] = X[k]
        V[(nx + nu) * k + nx:(nx + nu) * (k + 1)] = Uk[k]
    V[(nx + nu) * N:] = X[N]
    return V, float(r @ r), float(stat), len(act), len(held_u)


def main():
    h, inf = 0.002, np.inf
    cases = []
    w2 = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
    x0, up, tr = g2.synth_two_link(20250213, 0, 13, 30, h)
    specs = [  # (instance, x_lb, x_ub, u_lb, u_ub): instances whose solutions have active state bounds
        (2, [-inf, -inf, -1.5, -1.5], [inf, inf, 1.5, 1.5], [-inf, -inf], [inf, inf]),
        (12, [-inf, -inf, -1.5, -1.5], [inf, inf, 1.5, 1.5], [-inf, -inf], [inf, inf]),
        (12, [-inf, -inf, -2.0, -2.0], [inf, inf, 2.0, 2.0], [-4.0, -4.0], [4.0, 4.0]),
        (5, [-0.6, -0.6, -3.0, -3.0], [0.6, 0.6, 3.0, 3.0], [-inf, -inf], [inf, inf]),
    ]
    for b, xl, xu, ul, uu in specs:
        xl, xu, ul, uu = map(np.array, (xl, xu, ul, uu))
        V, J, stat, na, nh = solve(x0[b], up[b], tr[b], w2, h, g2.f, g2.jac, 4, 2, xl, xu, ul, uu)
        print("two_link", b, J, stat, na, nh, flush=True)
        cases.append(dict(model="two_link_arm", N=30, index=b, x0=x0[b].tolist(), u_prev=up[b].tolist(),
                          traj=tr[b].tolist(), weights=w2.tolist(), x_lb=[float(v) for v in xl],
                          x_ub=[float(v) for v in xu], u_lb=[float(v) for v in ul], u_ub=[float(v) for v in uu],
                          V=V.tolist(), J=J, stationarity=stat, n_active_x=na, n_active_u=nh))
    wx = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
    xl = np.array([-inf] * 4 + [-0.3] * 4)
    xu = np.array([inf] * 4 + [0.3] * 4)
    x0, up, tr = gx.synth_exo(20250213, 300, 1, 20, h)
    x0[0, 4:] = np.clip(x0[0, 4:], -0.25, 0.25)  # the measured state inside the velocity box
    V, J, stat, na, nh = solve(x0[0], up[0], tr[0], wx, h, gx.f, gx.jac, 8, 4, xl, xu, np.full(4, -inf),
                               np.full(4, inf))
    print("exo", J, stat, na, nh, flush=True)
    cases.append(dict(model="exo_arm", N=20, index=300, x0=x0[0].tolist(), u_prev=up[0].tolist(),
                      traj=tr[0].tolist(), weights=wx.tolist(), x_lb=[float(v) for v in xl],
                      x_ub=[float(v) for v in xu], u_lb=[-inf] * 4, u_ub=[inf] * 4, V=V.tolist(), J=J,
                      stationarity=stat, n_active_x=na, n_active_u=nh))
    with open(os.path.join(HERE, "xbounds_golden.json"), "w") as fh:
        json.dump(dict(h=h, seed=20250213,
                       solver="scipy SLSQP on the single-shooting form (state bounds as inequality constraints, "
                              "exact sensitivities), then Gauss-Newton SQP polish on the active set; KKT checked",
                       cases=cases), fh, allow_nan=True)


if __name__ == "__main__":
    main()
