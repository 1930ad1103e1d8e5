"""Exact-Hessian checks on the CPU: nlp_hess_l of the oracle, and a second-order KKT certificate
of the committed golden solutions.

* oracle_nlp_hess (the (x_k, u_k) stage blocks of the Hessian of lam_f J + lam_g^T g, ModelGenerator.cpp:238) against
  central differences of an independent numpy gradient of the same Lagrangian, built from the oracle's analytic
  (K3-pinned) Jacobians: 1e-6 relative.
* Certificate at every golden V* (scipy solves of the identical NLP, tests/golden/make_golden*.py): the multipliers
  lam_g follow from stationarity in x_1..x_N; the reduced gradient (stationarity in u) vanishes to 1e-9; the reduced
  Hessian Z^T (d^2 L) Z on the null space of the constraint Jacobian (Z = [Gamma; I], x_0 pinned) is positive
  definite -- V* is a strict local minimiser of the reference NLP.  Stage Hessians: oracle_nlp_hess for the 2-link
  arm, central differences of the analytic Jacobian for the exo (no second derivatives in its oracle model).
"""
import numpy as np
import pytest

from conftest import load_golden


def _jac(oracle, model, x, u):
    return (oracle.exo_jac if model == oracle.EXO else oracle.two_link_jac)(x, u)


def _stage_blocks(oracle, model, N, h, V, up, tr, w, lam):
    """(x_k, u_k) Hessian blocks of J + lam^T g"""
    nx, nu = oracle.DIMS[model]
    if model == oracle.TWO_LINK:
        return oracle.nlp_hess(N, h, V, up, tr, w, 1.0, lam, model=model)
    K = nx + nu
    out = np.zeros((N, K, K))
    Q, R, Rm = w[:nx], w[nx:nx + nu], w[nx + nu:]
    Vs = V[:-nx].reshape(N, K)
    for k in range(N):
        x, u = Vs[k, :nx], Vs[k, nx:]
        A, B, xd = _jac(oracle, model, x, u)
        JF = np.hstack([np.eye(nx) + h * A, h * B])
        nu_ = h * (2 * Q * (x + h * xd - tr[k]) + lam[k])
        z = np.concatenate([x, u])
        W = np.zeros((K, K))
        for j in range(K):
            zp, zm = z.copy(), z.copy()
            zp[j] += 1e-6
            zm[j] -= 1e-6
            Ap, Bp, _ = _jac(oracle, model, zp[:nx], zp[nx:])
            Am, Bm, _ = _jac(oracle, model, zm[:nx], zm[nx:])
            W[:, j] = nu_ @ ((np.hstack([Ap, Bp]) - np.hstack([Am, Bm])) / 2e-6)
        out[k] = 0.5 * (W + W.T) + 2 * JF.T @ (Q[:, None] * JF)
        out[k, nx:, nx:] += np.diag(2 * R + 2 * Rm + (2 * R if k + 1 < N else 0))
    return out


def _lagrangian_grad(oracle, model, N, h, V, up, tr, w, lam):
    """d(J + lam^T g)/dV in the V layout (numpy restatement from the analytic Jacobians)"""
    nx, nu = oracle.DIMS[model]
    K = nx + nu
    Q, R, Rm = w[:nx], w[nx:nx + nu], w[nx + nu:]
    Vs = V[:-nx].reshape(N, K)
    g = np.zeros_like(V)
    for k in range(N):
        x, u = Vs[k, :nx], Vs[k, nx:]
        A, B, xd = _jac(oracle, model, x, u)
        JF = np.hstack([np.eye(nx) + h * A, h * B])
        e = x + h * xd - tr[k]
        g[k * K:(k + 1) * K] += JF.T @ (2 * Q * e + lam[k])
        g[(k + 1) * K:(k + 1) * K + nx] -= lam[k]
        um = up if k == 0 else Vs[k - 1, nx:]
        g[k * K + nx:(k + 1) * K] += 2 * R * (u - um) + 2 * Rm * u
        if k > 0:
            g[(k - 1) * K + nx:k * K] -= 2 * R * (u - um)
    return g


def test_oracle_nlp_hess_vs_finite_differences(oracle):
    N, h = 6, 0.002
    w = np.array([10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01])
    rng = np.random.default_rng(4)
    x0, up, tr = oracle.synth(3, 0, 1, N, h)
    V = rng.uniform(-1, 1, 4 * (N + 1) + 2 * N) * np.tile([1, 1, 1, 1, 5, 5], N + 1)[:4 * (N + 1) + 2 * N]
    lam = rng.normal(size=(N, 4))
    blocks = oracle.nlp_hess(N, h, V, up[0], tr[0], w, 1.0, lam)
    Hfd = np.zeros((V.size, V.size))
    for j in range(V.size):
        Vp, Vm = V.copy(), V.copy()
        Vp[j] += 1e-6
        Vm[j] -= 1e-6
        Hfd[:, j] = (_lagrangian_grad(oracle, oracle.TWO_LINK, N, h, Vp, up[0], tr[0], w, lam)
                     - _lagrangian_grad(oracle, oracle.TWO_LINK, N, h, Vm, up[0], tr[0], w, lam)) / 2e-6
    H = np.zeros_like(Hfd)
    for k in range(N):
        H[k * 6:(k + 1) * 6, k * 6:(k + 1) * 6] = blocks[k]
        if k > 0:   # the constant Delta-u coupling
            for c in range(2):
                H[k * 6 + 4 + c, (k - 1) * 6 + 4 + c] = H[(k - 1) * 6 + 4 + c, k * 6 + 4 + c] = -2 * w[4 + c]
    assert np.abs(H - Hfd).max() <= 1e-6 * np.abs(H).max()


def _certify(oracle, model, N, h, x0, up, tr, w, V):
    nx, nu = oracle.DIMS[model]
    K = nx + nu
    Q = w[:nx]
    Vs = V[:-nx].reshape(N, K)
    A, B, e = [], [], []
    for k in range(N):
        Ac, Bc, xd = _jac(oracle, model, Vs[k, :nx], Vs[k, nx:])
        A.append(np.eye(nx) + h * Ac)
        B.append(h * Bc)
        e.append(Vs[k, :nx] + h * xd - tr[k])
    # stationarity in x_{k+1}: lam_k = A_{k+1}^T (2 Q e_{k+1} + lam_{k+1}), lam_{N-1} = 0 (x_N enters only g_{N-1})
    lam = np.zeros((N, nx))
    for k in range(N - 2, -1, -1):
        lam[k] = A[k + 1].T @ (2 * Q * e[k + 1] + lam[k + 1])
    grad = _lagrangian_grad(oracle, model, N, h, V, up, tr, w, lam)
    red = np.array([grad[k * K + nx:(k + 1) * K] for k in range(N)]).ravel()   # d L / du at the multipliers
    scale = max(1.0, np.abs(2 * Q * np.array(e)).max())
    blocks = _stage_blocks(oracle, model, N, h, V, up, tr, w, lam)
    # null space of the linearised constraints (x_0 pinned): dx_{k+1} = A_k dx_k + B_k du_k
    M = N * nu
    S = np.zeros((N, K, M))   # [dx_k; du_k] as a function of du
    dx = np.zeros((nx, M))
    for k in range(N):
        S[k, :nx] = dx
        S[k, nx + np.arange(nu), k * nu + np.arange(nu)] = 1.0
        dx = A[k] @ dx + B[k] @ S[k, nx:]
    Hred = sum(S[k].T @ blocks[k] @ S[k] for k in range(N))
    for k in range(1, N):
        for c in range(nu):
            i, j = k * nu + c, (k - 1) * nu + c
            Hred[i, j] -= 2 * w[nx + c]
            Hred[j, i] -= 2 * w[nx + c]
    Hred = 0.5 * (Hred + Hred.T)
    ev = np.linalg.eigvalsh(Hred)
    return np.abs(red).max() / scale, ev.min() / ev.max(), ev.min()


@pytest.mark.parametrize("fixture", ["nlp_cfg1.json", "nlp_cfg2_16.json", "exo_golden.json"])
def test_golden_solutions_are_certified_local_minima(fixture, oracle):
    g = load_golden(fixture)
    model = oracle.EXO if fixture.startswith("exo") else oracle.TWO_LINK
    w = np.array(g["weights"])
    for c in g["cases"][:6]:
        N = c.get("N", g.get("N"))
        stat, cond, lmin = _certify(oracle, model, N, g["h"], np.array(c["x0"]), np.array(c["u_prev"]),
                                    np.array(c["traj"]), w, np.array(c["V"]))
        assert stat < 1e-9, stat           # first order: stationary on the null space (measured <= 5e-15)
        assert lmin > 0 and cond > 1e-10   # second order: reduced exact Hessian positive definite
