#!/usr/bin/env python3
"""Golden vectors for box-constrained controls (SURVEY.md 8a A1 bounds, 8f rank 1) -- build container only.

The reference passes u_min/u_max to IPOPT as lbx/ubx (ModelControl.cpp:37-50,146-157) and IPOPT returns a KKT
point of the bound-constrained NLP.  Here the same NLP is solved independently of oracle/ and of the kernels:
the SINGLE-shooting least-squares form (ModelGenerator.cpp:191-222, x_0 pinned) with scipy
``least_squares(method="trf", bounds=...)`` (a reflective trust-region method), then polished by Gauss-Newton
on the free controls with the controls trf drives onto a bound held there.  The polished point is checked to
be a KKT point: free controls strictly inside, projected gradient ||U - P(U - grad)||_inf <= 1e-9.

Writes tests/golden/bounds_golden.json: 4 cfg#2 instances (2-link, N = 30) and 2 exo instances (N = 20).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
from scipy.optimize import least_squares

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as g2  # noqa: E402  (2-link model: sympy Jacobians, cfg#2 generator)
import make_golden_exo as gx  # noqa: E402  (exo model: unexpanded M(q), complex-step Jacobians)


def residual_and_jac(U, x0, up, tr, w, h, f, jac, nx, nu):
    N = tr.shape[0]
    U = U.reshape(N, nu)
    Q, R, Rm = w[:nx], w[nx:nx + nu], w[nx + nu:nx + 2 * nu]
    X = np.zeros((N + 1, nx)); X[0] = x0
    S = np.zeros((nx, nu * N))
    res, rows = [], []
    for k in range(N):
        A, Bc = jac(X[k], U[k])
        X[k + 1] = X[k] + h * f(X[k], U[k])
        S = (np.eye(nx) + h * A) @ S
        S[:, nu * k:nu * k + nu] += h * Bc
        res.append(np.sqrt(Q) * (X[k + 1] - tr[k]))
        rows.append(np.sqrt(Q)[:, None] * S)
    for k in range(N):
        um = up if k == 0 else U[k - 1]
        res.append(np.sqrt(R) * (U[k] - um))
        Jr = np.zeros((nu, nu * N)); Jr[:, nu * k:nu * k + nu] = np.diag(np.sqrt(R))
        if k > 0:
            Jr[:, nu * (k - 1):nu * k] = -np.diag(np.sqrt(R))
        rows.append(Jr)
        res.append(np.sqrt(Rm) * U[k])
        Jm = np.zeros((nu, nu * N)); Jm[:, nu * k:nu * k + nu] = np.diag(np.sqrt(Rm))
        rows.append(Jm)
    return np.concatenate(res), np.vstack(rows), X


def solve_bounded(x0, up, tr, w, h, lb, ub, f, jac, nx, nu):
    N = tr.shape[0]
    lbv, ubv = np.tile(lb, N), np.tile(ub, N)
    fun = lambda U: residual_and_jac(U, x0, up, tr, w, h, f, jac, nx, nu)[0]  # noqa: E731
    jf = lambda U: residual_and_jac(U, x0, up, tr, w, h, f, jac, nx, nu)[1]  # noqa: E731
    sol = least_squares(fun, np.clip(np.zeros(nu * N), lbv, ubv), jac=jf, bounds=(lbv, ubv), method="trf",
                        xtol=1e-15, ftol=1e-15, gtol=1e-15, max_nfev=2000)
    U = sol.x.copy()
    # polish: hold what trf put on (or within 1e-7 of) a bound with the gradient pointing outward, GN on the rest
    for _ in range(60):
        r, J, _ = residual_and_jac(U, x0, up, tr, w, h, f, jac, nx, nu)
        grad = 2.0 * J.T @ r
        held = ((U <= lbv + 1e-7) & (grad > 0)) | ((U >= ubv - 1e-7) & (grad < 0))
        U[held & (grad > 0)] = lbv[held & (grad > 0)]
        U[held & (grad < 0)] = ubv[held & (grad < 0)]
        free = ~held
        step = np.zeros_like(U)
        step[free] = np.linalg.lstsq(J[:, free], -r, rcond=None)[0]
        U = np.clip(U + step, lbv, ubv)
        if np.abs(step).max() < 1e-15 * max(1.0, np.abs(U).max()):
            break
    r, J, X = residual_and_jac(U, x0, up, tr, w, h, f, jac, nx, nu)
    grad = 2.0 * J.T @ r
    pg = np.abs(U - np.clip(U - grad, lbv, ubv)).max()
    nact = int(((U == lbv) | (U == ubv)).sum())
    assert pg <= 1e-9, pg
    Uk = U.reshape(N, nu)
    V = np.zeros(nx * (N + 1) + nu * N)
    for k in range(N):
        V[(nx + nu) * k:(nx + nu) * k + nx] = X[k]
        V[(nx + nu) * k + nx:(nx + nu) * (k + 1)] = Uk[k]
    V[(nx + nu) * N:] = X[N]
    return V, float(r @ r), float(pg), nact


def main():
    h = 0.002
    cases = []
    w2 = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
    lb2, ub2 = np.array([-3.0, -4.0]), np.array([2.5, 4.0])
    x0, up, tr = g2.synth_two_link(20250213, 0, 4, 30, h)
    for b in range(4):
        V, J, pg, nact = solve_bounded(x0[b], up[b], tr[b], w2, h, lb2, ub2, g2.f, g2.jac, 4, 2)
        print("two_link", b, J, pg, nact, flush=True)
        cases.append(dict(model="two_link_arm", N=30, index=b, x0=x0[b].tolist(), u_prev=up[b].tolist(),
                          traj=tr[b].tolist(), weights=w2.tolist(), u_lb=lb2.tolist(), u_ub=ub2.tolist(),
                          V=V.tolist(), J=J, proj_grad_inf=pg, n_active=nact))
    wx = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
    lbx, ubx = np.array([-0.6, -0.5, -0.5, -0.4]), np.array([0.5, 0.6, 0.5, 0.4])
    x0, up, tr = gx.synth_exo(20250213, 200, 2, 20, h)
    for b in range(2):
        V, J, pg, nact = solve_bounded(x0[b], up[b], tr[b], wx, h, lbx, ubx, gx.f, gx.jac, 8, 4)
        print("exo", b, J, pg, nact, flush=True)
        cases.append(dict(model="exo_arm", N=20, index=200 + b, x0=x0[b].tolist(), u_prev=up[b].tolist(),
                          traj=tr[b].tolist(), weights=wx.tolist(), u_lb=lbx.tolist(), u_ub=ubx.tolist(),
                          V=V.tolist(), J=J, proj_grad_inf=pg, n_active=nact))
    with open(os.path.join(HERE, "bounds_golden.json"), "w") as fh:
        json.dump(dict(h=h, seed=20250213,
                       solver="scipy least_squares trf with bounds on the single-shooting form, then Gauss-Newton "
                              "polish on the free controls (held controls on their bound); KKT checked by the "
                              "projected gradient",
                       cases=cases), fh)


if __name__ == "__main__":
    main()
