#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/.

Run in the development container (needs sympy + scipy; NOT needed on the GPU box):
    python tests/golden/make_golden.py

Nothing here imports or executes reference code: the reference (CasADi+IPOPT) cannot
be built or run.  The fixtures pin the oracle through
  K1  lin_test.m:31-50  -- the F_lin step with the answers the reference authors
      recorded at lin_test.m:49-50 (6 significant digits), re-derived here exactly;
  K2  lin_test.m:22-28  -- A, B, x_dot of the 2-link arm at the origin (sympy, exact);
  K3  A, B, x_dot at seeded random points: symbolic Jacobian of the ODE of
      examples/ex_model_generate.cpp:36-37, cross-checked against the hand-derived
      closed form of old/Models/DoublePendulumModel.hpp:15-131 (restated below);
  S1  cfg#1 single instance (examples/ex_model_control.cpp:66-73 trajectory,
      N=20, h=2 ms, Q/R from examples/thread_model_control_example.cpp:24-25) and
  S2  16 cfg#2 instances (SURVEY.md 8d generator) solved by an independent
      scipy trust-region Newton solve of the single-shooting form of the NLP
      of src/Mahi/Mpc/ModelGenerator.cpp:191-222 (x_0 pinned, so the dynamics
      equalities determine every x_k: the two forms share their minimisers).
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import sympy as sp
from scipy.optimize import minimize

HERE = os.path.dirname(os.path.abspath(__file__))

# ---------------- symbolic model (examples/ex_model_generate.cpp:24-43) ----------------
qA, qB, dA, dB, TA, TB = sp.symbols("qA qB qA_dot qB_dot TA TB", real=True)
Ls, ms, gs = sp.Integer(1), sp.Integer(1), sp.Rational(981, 100)
cos, sin = sp.cos, sp.sin
qA_dd = -(TA - TB - TB*cos(qB) + Ls*Ls*ms*dA*dA*sin(qB) + Ls*Ls*ms*dB*dB*sin(qB) - 2*Ls*gs*ms*cos(qA)
          + Ls*Ls*ms*dA*dA*cos(qB)*sin(qB) + 2*Ls*Ls*ms*dA*dB*sin(qB) + Ls*gs*ms*cos(qA + qB)*cos(qB)) \
    / (Ls*Ls*ms*(cos(qB)*cos(qB) - 2))
qB_dd = (TA - 3*TB + TA*cos(qB) - 2*TB*cos(qB) + 2*Ls*gs*ms*cos(qA + qB) + 3*Ls*Ls*ms*dA*dA*sin(qB)
         + Ls*Ls*ms*dB*dB*sin(qB) - 2*Ls*gs*ms*cos(qA) + 2*Ls*Ls*ms*dA*dA*cos(qB)*sin(qB)
         + Ls*Ls*ms*dB*dB*cos(qB)*sin(qB) - 2*Ls*gs*ms*cos(qA)*cos(qB) + 2*Ls*Ls*ms*dA*dB*sin(qB)
         + Ls*gs*ms*cos(qA + qB)*cos(qB) + 2*Ls*Ls*ms*dA*dB*cos(qB)*sin(qB)) \
    / (Ls*Ls*ms*(cos(qB)*cos(qB) - 2))
xs = sp.Matrix([qA, qB, dA, dB])
us = sp.Matrix([TA, TB])
xdot = sp.Matrix([dA, dB, qA_dd, qB_dd])
Asym = xdot.jacobian(xs)
Bsym = xdot.jacobian(us)
f_num = sp.lambdify((xs, us), xdot, "numpy")
A_num = sp.lambdify((xs, us), Asym, "numpy")
B_num = sp.lambdify((xs, us), Bsym, "numpy")


def f(x, u):
    return np.asarray(f_num(x, u), dtype=np.float64).reshape(4)


def jac(x, u):
    return (np.asarray(A_num(x, u), dtype=np.float64).reshape(4, 4),
            np.asarray(B_num(x, u), dtype=np.float64).reshape(4, 2))


def closed_form_old(x, u, L=1.0, m=1.0, g=9.81):
    """Restatement of the hand-derived A(x,u), B(x) of old/Models/DoublePendulumModel.hpp:15-95."""
    qa, qb, da, db = x
    ta, tb = u
    t2, t3, t4 = math.cos(qb), math.sin(qa), math.sin(qb)
    t5 = qa + qb
    t6, t7, t8, t9 = L * L, da * 2.0, qb * 2.0, db * 2.0
    t10, t11 = da * da, db * db
    t17, t20 = 1.0 / L, 1.0 / m
    t12, t13, t14, t15, t16 = math.cos(t8), t2 * t2, t2 ** 3, math.sin(t8), t4 ** 3
    t18, t19 = 1.0 / t6, math.sin(t5)
    t22 = t7 + t9
    t23 = L * g * m * t3 * 2.0
    t21 = ta * t15
    t24, t25 = t12 - 3.0, t13 - 2.0
    t30 = L * g * m * t3 * t13 * 3.0
    t31 = m * t6 * t11 * t14
    t32 = m * db * t6 * t7 * t14
    t26, t27, t28, t33 = -t21, 1.0 / t24, 1.0 / t25, -t30
    t29 = t28 * t28
    A = np.zeros((4, 4))
    A[0, 2] = 1.0
    A[1, 3] = 1.0
    A[2, 0] = -g * t17 * t27 * (t3 * 3.0 - math.sin(qb + t5))
    A[2, 1] = t18 * t20 * t29 * (t23 + t26 + t31 + t32 + t33 + tb * t4 * 3.0 + tb * t15 - tb * t16
                                 - m * t6 * t10 * 2.0 + m * t6 * t10 * t13 * 3.0 + m * t6 * t10 * t14)
    A[2, 2] = -t28 * (t4 * t7 + t4 * t9 + t2 * t4 * t7)
    A[2, 3] = (t4 * t22) / (t4 * t4 + 1.0)
    A[3, 0] = g * t17 * t28 * (t3 * 2.0 - t19 * 2.0 + t2 * t3 * 2.0 - t2 * t19)
    A[3, 1] = -t18 * t20 * t29 * (t23 + t26 + t31 + t32 + t33 - ta * t4 * 3.0 + ta * t16 + tb * t4 * 6.0
                                  + tb * t15 * 3.0 - tb * t16 * 2.0 - m * t6 * t10 * 4.0 - m * t6 * t11 * 2.0
                                  - m * da * db * t6 * 4.0 + m * t6 * t10 * t13 * 6.0 + m * t6 * t10 * t14 * 3.0
                                  + m * t6 * t11 * t13 * 3.0 - L * g * m * t3 * t14 * 2.0
                                  + m * da * db * t6 * t13 * 6.0)
    A[3, 2] = t27 * (da * t4 * 1.2e1 + da * t15 * 4.0 + db * t4 * 4.0 + t9 * t15)
    A[3, 3] = t22 * t28 * (t4 + t2 * t4)
    c2 = math.cos(qb)
    s5, s6 = 1.0 / (L * L), 1.0 / m
    s3, s4 = c2 + 1.0, c2 * c2
    s8 = 1.0 / (s4 - 2.0)
    s9 = s3 * s5 * s6 * s8
    B = np.zeros((4, 2))
    B[2, 0] = -s5 * s6 * s8
    B[2, 1] = s9
    B[3, 0] = s9
    B[3, 1] = -s5 * s6 * s8 * (s3 * 2.0 + 1.0)
    return A, B


# ---------------- synthetic generator (must match oracle/HIP) ----------------
M64 = (1 << 64) - 1


def splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def unit_draw(seed, index, j):
    v = splitmix64(seed ^ splitmix64((index * 16 + j) & M64))
    return (v >> 11) * 2.0 ** -53


def synth_two_link(seed, first, B, N, h):
    x0 = np.zeros((B, 4)); up = np.zeros((B, 2)); tr = np.zeros((B, N, 4))
    for b in range(B):
        gi = first + b
        # lo + span*u, product and sum rounded separately (Python never fuses) == C/HIP affine_draw
        x0[b] = [-math.pi / 4 + (math.pi / 2) * unit_draw(seed, gi, 0),
                 -math.pi / 4 + (math.pi / 2) * unit_draw(seed, gi, 1),
                 -1.0 + 2.0 * unit_draw(seed, gi, 2), -1.0 + 2.0 * unit_draw(seed, gi, 3)]
        up[b] = [-5.0 + 10.0 * unit_draw(seed, gi, 4), -5.0 + 10.0 * unit_draw(seed, gi, 5)]
        a = 0.5 + 0.5 * unit_draw(seed, gi, 6)
        fr = 0.25 + 0.75 * unit_draw(seed, gi, 7)
        ph = 0.0 + (2.0 * math.pi) * unit_draw(seed, gi, 8)
        for k in range(N):
            arg = 2.0 * math.pi * fr * (k * h) + ph
            s, c = a * math.sin(arg), 2.0 * math.pi * fr * a * math.cos(arg)
            tr[b, k] = [s, -s, c, -c]
    return x0, up, tr


# ---------------- independent single-shooting solve ----------------
def rollout(x0, U, h):
    N = U.shape[0]
    X = np.zeros((N + 1, 4)); X[0] = x0
    for k in range(N):
        X[k + 1] = X[k] + h * f(X[k], U[k])
    return X


def objective(U, x0, up, tr, w, h):
    U = U.reshape(-1, 2)
    Q, R, Rm = w[:4], w[4:6], w[6:8]
    X = rollout(x0, U, h)
    e = X[1:] - tr
    du = np.diff(np.vstack([up, U]), axis=0)
    return float(np.sum(e * e * Q) + np.sum(du * du * R) + np.sum(U * U * Rm))


def gradient(U, x0, up, tr, w, h):
    """exact gradient by forward sensitivities (independent of the oracle's adjoint)."""
    U = U.reshape(-1, 2); N = U.shape[0]
    Q, R, Rm = w[:4], w[4:6], w[6:8]
    X = rollout(x0, U, h)
    S = np.zeros((N + 1, 4, 2 * N))           # dX_k / dU
    for k in range(N):
        A, B = jac(X[k], U[k])
        Ad = np.eye(4) + h * A
        S[k + 1] = Ad @ S[k]
        S[k + 1][:, 2 * k:2 * k + 2] += h * B
    e = X[1:] - tr
    g = np.einsum("kr,kra->a", 2 * e * Q, S[1:])
    du = np.diff(np.vstack([up, U]), axis=0)
    gu = 2 * du * R + 2 * U * Rm
    gu[:-1] -= 2 * du[1:] * R
    return g + gu.reshape(-1)


def solve_ss(x0, up, tr, w, h):
    N = tr.shape[0]
    fun = lambda U: objective(U, x0, up, tr, w, h)
    jacf = lambda U: gradient(U, x0, up, tr, w, h)

    def hess(U, eps=1e-6):
        n = U.size; Hm = np.zeros((n, n))
        for i in range(n):
            e = np.zeros(n); e[i] = eps
            Hm[:, i] = (jacf(U + e) - jacf(U - e)) / (2 * eps)
        return 0.5 * (Hm + Hm.T)

    r = minimize(fun, np.zeros(2 * N), jac=jacf, hess=hess, method="trust-exact",
                 options=dict(gtol=1e-11, maxiter=200))
    U = r.x.reshape(N, 2)
    # polish with exact-gradient Newton steps (FD Hessian is accurate to ~1e-9 relative)
    for _ in range(3):
        U = U - np.linalg.solve(hess(U.reshape(-1)), jacf(U.reshape(-1))).reshape(N, 2)
    X = rollout(x0, U, h)
    V = np.zeros(4 * (N + 1) + 2 * N)
    for k in range(N):
        V[6 * k:6 * k + 4] = X[k]; V[6 * k + 4:6 * k + 6] = U[k]
    V[6 * N:6 * N + 4] = X[N]
    gfin = jacf(U.reshape(-1))
    return V, objective(U.reshape(-1), x0, up, tr, w, h), float(np.abs(gfin).max()), int(r.nit)


def main():
    rng = np.random.default_rng(20250213)
    # K1: lin_test.m:31-50
    x_t = np.array([0.012566, -0.012566, 6.286450, -6.286450])
    x_i = np.array([0.00628315, -0.00628309, 6.28305, -6.28278])
    u_t = np.array([9451.340333, 3150.037249])
    u_i = np.array([9458.794556, 3152.724932])
    h = 0.002
    A_i, B_i = jac(x_i, u_i)
    xdot_i = f(x_i, u_i)
    xdot_lin = A_i @ (x_t - x_i) + B_i @ (u_t - u_i) + xdot_i
    k1 = dict(
        source="lin_test.m:31-50", h=h, x=x_t.tolist(), x_init=x_i.tolist(), u=u_t.tolist(), u_init=u_i.tolist(),
        A_init=A_i.tolist(), B_init=B_i.tolist(), xdot_init=xdot_i.tolist(),
        F_lin=(x_t + h * xdot_lin).tolist(),
        recorded_standard=[0.025139, -0.025139, 12.568, -12.5677],          # lin_test.m:49
        recorded_looking_for=[0.018856, -0.018855, 6.284949, -6.284949],     # lin_test.m:50
        x_minus_xinit_plus_h_xdotlin=(x_t - x_i + h * xdot_lin).tolist(),
    )
    assert np.allclose(k1["F_lin"], k1["recorded_standard"], rtol=0, atol=6e-4)
    assert np.allclose(k1["x_minus_xinit_plus_h_xdotlin"], k1["recorded_looking_for"], rtol=0, atol=2e-6)
    # K2: origin
    A0, B0 = jac(np.zeros(4), np.zeros(2))
    k2 = dict(source="lin_test.m:22-28", A=A0.tolist(), B=B0.tolist(), xdot=f(np.zeros(4), np.zeros(2)).tolist())
    # K3: random points; closed form of old/Models/DoublePendulumModel.hpp must agree with sympy
    pts = []
    for _ in range(12):
        x = np.r_[rng.uniform(-math.pi, math.pi, 2), rng.uniform(-3, 3, 2)]
        u = rng.uniform(-20, 20, 2)
        A, B = jac(x, u)
        Ao, Bo = closed_form_old(x, u)
        assert np.allclose(A, Ao, rtol=1e-10, atol=1e-10), (A, Ao)
        assert np.allclose(B, Bo, rtol=1e-12, atol=1e-12)
        pts.append(dict(x=x.tolist(), u=u.tolist(), A=A.tolist(), B=B.tolist(), xdot=f(x, u).tolist()))
    k3 = dict(source="examples/ex_model_generate.cpp:36-37 (sympy jacobian); "
                     "cross-checked vs old/Models/DoublePendulumModel.hpp:15-95", points=pts)
    with open(os.path.join(HERE, "two_link_kat.json"), "w") as fh:
        json.dump(dict(K1=k1, K2=k2, K3=k3), fh, indent=1)

    w = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
    # S1: cfg#1 (N=20) single instance, t=0 trajectory of ex_model_control.cpp:66-73
    N = 20
    tr = np.array([[math.sin(2 * math.pi * k * h), -math.sin(2 * math.pi * k * h),
                    2 * math.pi * math.cos(2 * math.pi * k * h), -2 * math.pi * math.cos(2 * math.pi * k * h)]
                   for k in range(N)])
    cases = []
    x0s = [np.zeros(4), np.array([0.3, -0.2, 0.5, -0.4])]
    ups = [np.zeros(2), np.array([2.0, -1.0])]
    for x0, up in zip(x0s, ups):
        V, J, gmax, nit = solve_ss(x0, up, tr, w, h)
        cases.append(dict(x0=x0.tolist(), u_prev=up.tolist(), traj=tr.tolist(), V=V.tolist(), J=J,
                          grad_inf=gmax, scipy_nit=nit))
        print("cfg1", J, gmax)
    with open(os.path.join(HERE, "nlp_cfg1.json"), "w") as fh:
        json.dump(dict(N=N, h=h, weights=w.tolist(), solver="scipy trust-exact single shooting + Newton polish",
                       cases=cases), fh)
    # S2: cfg#2 16 instances
    N = 30
    x0, up, tr = synth_two_link(20250213, 0, 16, N, h)
    cases = []
    for b in range(16):
        V, J, gmax, nit = solve_ss(x0[b], up[b], tr[b], w, h)
        cases.append(dict(index=b, x0=x0[b].tolist(), u_prev=up[b].tolist(), traj=tr[b].tolist(), V=V.tolist(),
                          J=J, grad_inf=gmax, scipy_nit=nit))
        print("cfg2", b, J, gmax)
    with open(os.path.join(HERE, "nlp_cfg2_16.json"), "w") as fh:
        json.dump(dict(N=N, h=h, seed=20250213, weights=w.tolist(),
                       solver="scipy trust-exact single shooting + Newton polish", cases=cases), fh)


if __name__ == "__main__":
    main()
