"""GPU: mmpc_nlp_derivs_batch -- nlp_grad_f and nlp_jac_g of the reference's generated NLP (ModelGenerator.cpp:238,
CasADi generate_dependencies) for the built-in 2-link arm and exo, nonlinear and linear mode, and for an
SX-generated model.  Checked against (a) the same formulas in numpy on the oracle's model Jacobians (1e-12) and
(b) central differences of the oracle's J (1e-6 relative): the gradient of J with respect to every entry of V,
the defect Jacobian blocks [I + h f_x | h f_u], and J itself against mmpc_nlp_eval_batch."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, WEIGHTS_CFG

pytestmark = pytest.mark.gpu


def numpy_derivs(jacf, V, up, tr, w, N, h, nx, nu):
    ND = nx + nu
    Q, R, Rm = w[:nx], w[nx:nx + nu], w[nx + nu:]
    grad = np.zeros_like(V)
    blocks = np.zeros((N, nx, ND))
    J = 0.0
    for k in range(N):
        x, u = V[k * ND:k * ND + nx], V[k * ND + nx:(k + 1) * ND]
        A, Bc, xd = jacf(x, u)
        e = x + h * xd - tr[k]
        J += e @ (Q * e)
        Ad, Bd = np.eye(nx) + h * A, h * Bc
        blocks[k] = np.hstack([Ad, Bd])
        grad[k * ND:k * ND + nx] = 2 * Ad.T @ (Q * e)
        um = up if k == 0 else V[(k - 1) * ND + nx:k * ND]
        g = 2 * Bd.T @ (Q * e) + 2 * R * (u - um) + 2 * Rm * u
        if k + 1 < N:
            g -= 2 * R * (V[(k + 1) * ND + nx:(k + 2) * ND] - u)
        grad[k * ND + nx:(k + 1) * ND] = g
        J += (u - um) @ (R * (u - um)) + u @ (Rm * u)
    return J, grad, blocks


@pytest.mark.parametrize("model", ["two_link_arm", "exo_arm", "two_link_linear"])
def test_nlp_derivs(model, mmpc_mod, oracle, tmp_path):
    exo = model == "exo_arm"
    linear = model == "two_link_linear"
    model = "two_link_arm" if linear else model
    nx, nu, N, h, B = (8, 4, 12, 0.002, 16) if exo else (4, 2, 20, 0.002, 16)
    s = mmpc_mod.Solver(mmpc_mod.write_model_json(str(tmp_path / "m.json"), "m", nx, nu, 2000, N, is_linear=linear,
                                                  model=model))
    om = oracle.EXO if exo else oracle.TWO_LINK
    x0, up, tr = oracle.synth(20250213, 0, B, N, h, model=om)
    w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4) if exo else np.array(WEIGHTS_CFG)
    rng = np.random.default_rng(1)
    V = rng.uniform(-0.5, 0.5, (B, s.NV))
    f = dict(dtype=torch.float64, device="cuda")
    t = lambda a: torch.tensor(np.ascontiguousarray(a), **f)  # noqa: E731
    J = torch.zeros(B, **f); G = torch.zeros((B, s.NV), **f); JB = torch.zeros((B, N, nx, nx + nu), **f)
    s.nlp_derivs(B, t(V), t(up), t(tr), t(w), J, G, JB)
    J2 = torch.zeros(B, **f); gi = torch.zeros(B, **f)
    s.nlp_eval(B, t(V), t(up), t(tr), t(w), J2, gi)
    torch.cuda.synchronize()
    J, G, JB = J.cpu().numpy(), G.cpu().numpy(), JB.cpu().numpy()
    np.testing.assert_allclose(J, J2.cpu().numpy(), rtol=1e-14)
    for b in range(B):
        jacf = oracle.exo_jac if exo else oracle.two_link_jac
        if linear:  # F_lin: model linearised at (x_0, u_prev) (ModelGenerator.cpp:160-175)
            A0, B0, xd0 = oracle.two_link_jac(V[b, :nx], up[b])
            jacf = lambda x, u, A0=A0, B0=B0, xd0=xd0, x0=V[b, :nx], u0=up[b]: (  # noqa: E731
                A0, B0, xd0 + A0 @ (x - x0) + B0 @ (u - u0))
        Jn, gn, bn = numpy_derivs(jacf, V[b], up[b], tr[b], w, N, h, nx, nu)
        assert abs(J[b] - Jn) <= 1e-12 * abs(Jn)
        np.testing.assert_allclose(G[b], gn, rtol=1e-12, atol=1e-12 * np.abs(gn).max())
        np.testing.assert_allclose(JB[b], bn, rtol=1e-12, atol=1e-14)
    if linear:
        return  # the oracle's nlp_eval is the nonlinear NLP
    # central differences of the oracle's J on instance 0
    eps = 1e-6
    for i in range(0, s.NV, 7):
        Vp, Vm = V[0].copy(), V[0].copy()
        Vp[i] += eps; Vm[i] -= eps
        fd = (oracle.nlp_eval(N, h, Vp, up[0], tr[0], w, model=om)[0]
              - oracle.nlp_eval(N, h, Vm, up[0], tr[0], w, model=om)[0]) / (2 * eps)
        assert abs(fd - G[0, i]) <= 1e-6 * (1 + abs(fd)), (i, fd, G[0, i])


def test_nlp_derivs_generated_model(mmpc_mod, oracle):
    path = os.path.join(ROOT, "mahi-mpc_amd", "lib", "user", "motor_pendulum.json")
    if not os.path.exists(path):
        pytest.skip("generated model missing")
    s = mmpc_mod.Solver(path)
    m = oracle.UserModelHost("motor_pendulum")
    B, N, h, nx, nu = 8, s.N, s.h, s.nx, s.nu
    rng = np.random.default_rng(4)
    V = rng.uniform(-0.5, 0.5, (B, s.NV)); up = rng.uniform(-1, 1, (B, nu)); tr = rng.uniform(-1, 1, (B, N, nx))
    w = np.concatenate([np.full(nx, 5.0), np.full(nu, 0.5), np.full(nu, 0.01)])
    f = dict(dtype=torch.float64, device="cuda")
    t = lambda a: torch.tensor(np.ascontiguousarray(a), **f)  # noqa: E731
    J = torch.zeros(B, **f); G = torch.zeros((B, s.NV), **f); JB = torch.zeros((B, N, nx, nx + nu), **f)
    s.nlp_derivs(B, t(V), t(up), t(tr), t(w), J, G, JB)
    torch.cuda.synchronize()
    for b in range(B):
        Jn, gn, bn = numpy_derivs(m.jac, V[b], up[b], tr[b], w, N, h, nx, nu)
        assert abs(J[b].item() - Jn) <= 1e-12 * abs(Jn)
        np.testing.assert_allclose(G[b].cpu().numpy(), gn, rtol=1e-12, atol=1e-12 * np.abs(gn).max())
        np.testing.assert_allclose(JB[b].cpu().numpy(), bn, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("model", ["two_link_arm", "cart_pole", "exo_arm"])
def test_nlp_hess(model, mmpc_mod, oracle, tmp_path):
    """mmpc_nlp_hess_batch (nlp_hess_l, ModelGenerator.cpp:238): the (x_k, u_k) stage blocks of the Hessian of
    lam_f J + lam_g^T g against the oracle's (its own hyper-dual second derivatives for the 2-link arm; the host build
    of the generated header, itself pinned to sympy, for cart-pole; round 4: the exo's analytic Hessian, oracle_exo_hess,
    itself checked against differences of the analytic Jacobian) at 1e-12 relative; symmetric."""
    B, lam_f = 24, 0.7
    if model == "cart_pole":
        path = os.path.join(ROOT, "mahi-mpc_amd", "lib", "user", "cart_pole.json")
        if not os.path.exists(path):
            pytest.skip("cart_pole not generated")
        s = mmpc_mod.Solver(path)
        om = oracle.use_user_model("cart_pole")
    else:
        nx, nu = (8, 4) if model == "exo_arm" else (4, 2)
        s = mmpc_mod.Solver(mmpc_mod.write_model_json(str(tmp_path / "m.json"), "m", nx, nu, 2000, 12, model=model))
        om = oracle.EXO if model == "exo_arm" else oracle.TWO_LINK
    nx, nu, N, K = s.nx, s.nu, s.N, s.nx + s.nu
    rng = np.random.default_rng(9)
    V = rng.uniform(-0.8, 0.8, (B, s.NV))
    up = rng.uniform(-1, 1, (B, nu))
    tr = rng.uniform(-1, 1, (B, N, nx))
    lam = rng.normal(size=(B, N * nx))
    w = np.concatenate([np.full(nx, 5.0), np.full(nu, 0.5), np.full(nu, 0.01)])
    f = dict(dtype=torch.float64, device="cuda")
    t = lambda a: torch.tensor(np.ascontiguousarray(a), **f)  # noqa: E731
    out = torch.zeros((B, N, K, K), **f)
    s.nlp_hess(B, t(V), t(up), t(tr), t(w), lam_f, t(lam), out)
    torch.cuda.synchronize()
    H = out.cpu().numpy()
    for b in range(B):
        ref = oracle.nlp_hess(N, s.h, V[b], up[b], tr[b], w, lam_f, lam[b], model=om)
        assert np.abs(H[b] - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max()), b
        np.testing.assert_array_equal(H[b], H[b].transpose(0, 2, 1))
