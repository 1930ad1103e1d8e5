#!/usr/bin/env python3
"""Golden vectors for the exo model (SURVEY.md 8a A3b, 8d cfg#3) -- run in the build container only.

Independent of oracle/ and of the HIP kernels:
  * M(q) is lambdified from the UNEXPANDED CasADi printout of src/inverseTest.cpp:59-74 (parsed by
    tools/gen_exo_model.py:load_entries) with the build-defined parameters of exo_params.json;
  * f(x, u) = [qd; M(q)^-1 (tau - D qd - G(q))] with numpy.linalg.solve;
  * Jacobians by complex-step differentiation (exact to roundoff, no symbolic derivative);
  * the NLP (ModelGenerator.cpp:191-222 with the exo dynamics) is solved in SINGLE-shooting form as a
    nonlinear least-squares problem with scipy.optimize.least_squares (trust-region reflective), i.e. a
    different formulation and solver from the GN-SQP multiple-shooting path under test.

Writes tests/golden/exo_golden.json: Jacobian points and 4 cfg#3 instances (N = 50) + 1 short horizon.
The reference is read here only; the fixture is data (inputs and expected outputs).
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np
import sympy as sp
from scipy.optimize import least_squares

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tools"))
import gen_exo_model as gen  # noqa: E402

P = json.load(open(os.path.join(HERE, "exo_params.json")))
GAIN = np.array([float(v) for v in P["gravity_gain"]])
DAMP = np.array([float(v) for v in P["damping"]])


def build_mass():
    ents, q, params = gen.load_entries()
    subs = gen.param_subs(params, P)
    exprs = [ents[k].subs(subs) for k in gen.UPPER]
    fn = sp.lambdify((q[0], q[1], q[2]), exprs, "numpy")

    def M(qv):  # qv: joint angles [q0..q3] (printout q_k = joint k, k = 1..3)
        up = fn(qv[1], qv[2], qv[3])
        Mm = np.zeros((4, 4), dtype=np.result_type(qv.dtype, float))
        for (a, b), v in zip(gen.IDX, up):
            Mm[a, b] = Mm[b, a] = v
        return Mm
    return M


MASS = build_mass()


def f(x, u):
    q, qd = x[:4], x[4:]
    w = u - DAMP * qd - GAIN * np.sin(q)
    return np.concatenate([qd, np.linalg.solve(MASS(q), w)])


def jac(x, u, eps=1e-30):
    A = np.zeros((8, 8)); B = np.zeros((8, 4))
    for j in range(8):
        xc = x.astype(complex); xc[j] += 1j * eps
        A[:, j] = f(xc, u.astype(complex)).imag / eps
    for j in range(4):
        uc = u.astype(complex); uc[j] += 1j * eps
        B[:, j] = f(x.astype(complex), uc).imag / eps
    return A, B


# ---- cfg#3 generator (same recipe as oracle_synth_exo / synth_exo_kernel) ----
def splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def unit_draw_exo(seed, index, j):
    v = splitmix64(((seed + 0x3C6EF372FE94F82A) & 0xFFFFFFFFFFFFFFFF) ^ splitmix64(index * 32 + j))
    return (v >> 11) * 2.0 ** -53


def synth_exo(seed, first, B, N, h):
    x0 = np.zeros((B, 8)); up = np.zeros((B, 4)); tr = np.zeros((B, N, 8))
    for b in range(B):
        gi = first + b
        a = np.zeros(4); fr = np.zeros(4); ph = np.zeros(4)
        for j in range(4):
            x0[b, j] = -0.5 + 1.0 * unit_draw_exo(seed, gi, j)
            x0[b, 4 + j] = -0.5 + 1.0 * unit_draw_exo(seed, gi, 4 + j)
            up[b, j] = -1.0 + 2.0 * unit_draw_exo(seed, gi, 8 + j)
            a[j] = 0.1 + 0.3 * unit_draw_exo(seed, gi, 12 + j)
            fr[j] = 0.25 + 0.75 * unit_draw_exo(seed, gi, 16 + j)
            ph[j] = 0.0 + (2.0 * math.pi) * unit_draw_exo(seed, gi, 20 + j)
        for k in range(N):
            for j in range(4):
                arg = 2.0 * math.pi * fr[j] * (k * h) + ph[j]
                tr[b, k, j] = a[j] * math.sin(arg)
                tr[b, k, 4 + j] = 2.0 * math.pi * fr[j] * a[j] * math.cos(arg)
    return x0, up, tr


# ---- single-shooting least squares ----
def residual_and_jac(U, x0, up, tr, w, h):
    N = tr.shape[0]
    U = U.reshape(N, 4)
    Q, R, Rm = w[:8], w[8:12], w[12:16]
    X = np.zeros((N + 1, 8)); X[0] = x0
    S = np.zeros((8, 4 * N))
    res = []
    jac_rows = []
    for k in range(N):
        A, Bc = jac(X[k], U[k])
        X[k + 1] = X[k] + h * f(X[k], U[k])
        S = (np.eye(8) + h * A) @ S
        S[:, 4 * k:4 * k + 4] += h * Bc
        res.append(np.sqrt(Q) * (X[k + 1] - tr[k]))
        jac_rows.append(np.sqrt(Q)[:, None] * S)
    for k in range(N):
        um = up if k == 0 else U[k - 1]
        res.append(np.sqrt(R) * (U[k] - um))
        Jr = np.zeros((4, 4 * N)); Jr[:, 4 * k:4 * k + 4] = np.diag(np.sqrt(R))
        if k > 0:
            Jr[:, 4 * (k - 1):4 * k] = -np.diag(np.sqrt(R))
        jac_rows.append(Jr)
        res.append(np.sqrt(Rm) * U[k])
        Jm = np.zeros((4, 4 * N)); Jm[:, 4 * k:4 * k + 4] = np.diag(np.sqrt(Rm))
        jac_rows.append(Jm)
    return np.concatenate(res), np.vstack(jac_rows), X


def solve_ss(x0, up, tr, w, h):
    N = tr.shape[0]
    cache = {}

    def fun(U):
        r, J, _ = residual_and_jac(U, x0, up, tr, w, h)
        cache["J"] = J
        return r

    def jacf(U):
        return residual_and_jac(U, x0, up, tr, w, h)[1]

    sol = least_squares(fun, np.zeros(4 * N), jac=jacf, method="trf", xtol=1e-15, ftol=1e-15, gtol=1e-15,
                        max_nfev=500)
    # polish with MINPACK Levenberg-Marquardt from the trf point
    sol2 = least_squares(fun, sol.x, jac=jacf, method="lm", xtol=1e-15, ftol=1e-15, gtol=1e-15, max_nfev=2000)
    U = sol2.x if sol2.cost <= sol.cost else sol.x
    # Gauss-Newton polish (the fixed point is the same stationary point; it converges linearly here)
    for _ in range(30):
        r, J, X = residual_and_jac(U, x0, up, tr, w, h)
        step = np.linalg.lstsq(J, -r, rcond=None)[0]
        U = U + step
        if np.abs(step).max() < 1e-15 * max(1.0, np.abs(U).max()):
            break
    r, J, X = residual_and_jac(U, x0, up, tr, w, h)
    grad = 2.0 * J.T @ r                      # gradient of J = sum r^2 (no 1/2, ModelGenerator.cpp:208-222)
    Uk = U.reshape(N, 4)
    V = np.zeros(8 * (N + 1) + 4 * N)
    for k in range(N):
        V[12 * k:12 * k + 8] = X[k]; V[12 * k + 8:12 * k + 12] = Uk[k]
    V[12 * N:12 * N + 8] = X[N]
    return V, float(r @ r), float(np.abs(grad).max()), int(sol.nfev)


def main():
    rng = np.random.default_rng(7)
    pts = []
    for _ in range(6):
        x = np.r_[rng.uniform(-1.5, 1.5, 4), rng.uniform(-2, 2, 4)]
        u = rng.uniform(-2, 2, 4)
        A, B = jac(x, u)
        pts.append(dict(x=x.tolist(), u=u.tolist(), xdot=f(x, u).tolist(), A=A.tolist(), B=B.tolist()))
    w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
    h = 0.002
    cases = []
    for N, first, B in ((50, 0, 4), (20, 100, 1)):
        x0, up, tr = synth_exo(20250213, first, B, N, h)
        for b in range(B):
            V, J, gmax, nfev = solve_ss(x0[b], up[b], tr[b], w, h)
            print("exo", N, first + b, J, gmax, nfev, flush=True)
            cases.append(dict(N=N, index=first + b, x0=x0[b].tolist(), u_prev=up[b].tolist(), traj=tr[b].tolist(),
                              V=V.tolist(), J=J, grad_inf=gmax))
    with open(os.path.join(HERE, "exo_golden.json"), "w") as fh:
        json.dump(dict(h=h, seed=20250213, weights=w.tolist(), params="exo_params.json",
                       solver="scipy least_squares (trf, then lm polish) single shooting, complex-step Jacobians, M(q) "
                              "lambdified from the unexpanded src/inverseTest.cpp:59-74 expressions",
                       jacobian_points=pts, cases=cases), fh)


if __name__ == "__main__":
    main()
