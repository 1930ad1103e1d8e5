"""GPU: solves of models defined as SX expressions and generated through ModelGenerator.

Each generated <name>.so (mahi-mpc_amd/lib/user, built by __graft_entry__.build()) carries the gfx950 solver
kernels compiled for that model; mmpc.Solver / ModelControl load it through the JSON's dll_filepath, as the
reference loads <name>.so (ModelControl.cpp:62, ModelGenerator.cpp:254-259).  Checked against:
  * the oracle's GN-SQP on the same dynamics (host build of the same generated header, itself pinned to sympy
    in tests/test_sx_models.py): V* within 1e-10 relative where the iteration counts agree (>= 90 %), 1e-6
    everywhere (a stop test landing within roundoff of its threshold), every instance converged;
  * for the reference's double pendulum, the built-in 2-link kernels of libmmpc.so on cfg#2-recipe instances;
  * every KKT solver the generated library has (16-lane group Riccati, lane Riccati), bounded controls,
    linear mode (exactly one SQP iteration), the device linearisation, and the closed-loop C++ example.
Models: double pendulum (nq = 2), cart-pole (nq = 2, nu = 1), unicycle (first order, nq = 0),
motor-driven pendulum (nq = 1, na = 2)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, WEIGHTS_CFG

pytestmark = pytest.mark.gpu
USER = os.path.join(ROOT, "mahi-mpc_amd", "lib", "user")
HOST = os.path.join(ROOT, "mahi-mpc_amd", "host")
MODELS = ["nonlinear_double_pendulum", "cart_pole", "unicycle", "motor_pendulum"]


def instances(nx, nu, B, N, h, seed=7):
    rng = np.random.default_rng(seed)
    x0 = rng.uniform(-0.3, 0.3, (B, nx))
    up = rng.uniform(-0.5, 0.5, (B, nu))
    t = np.arange(N) * h
    a = rng.uniform(0.1, 0.4, (B, 1, nx))
    f = rng.uniform(0.25, 1.0, (B, 1, nx))
    ph = rng.uniform(0, 2 * np.pi, (B, 1, nx))
    return x0, up, a * np.sin(2 * np.pi * f * t[None, :, None] + ph)


def weights(nx, nu):
    return np.concatenate([np.full(nx, 5.0), np.full(nu, 0.5), np.full(nu, 0.01)])


def compare(g, o, tight=1e-10):
    assert (g["status"] == 0).all(), np.bincount(g["status"])
    assert (o["status"] == 0).all()
    same = g["iters"] == o["iters"]
    assert same.mean() >= 0.9, (g["iters"], o["iters"])
    rel = np.abs(g["V"] - o["V"]).max(axis=1) / np.abs(o["V"]).max()
    assert rel[same].max() < tight, rel[same].max()
    assert rel.max() < 1e-6


def solver(mmpc_mod, name, **kw):
    path = os.path.join(USER, f"{name}.json")
    if not os.path.exists(path):
        pytest.skip(f"{name} not generated")
    return mmpc_mod.Solver(path, **kw)


@pytest.mark.parametrize("kkt", ["auto", "riccati", "group"])
@pytest.mark.parametrize("name", MODELS)
def test_generated_model_solve_matches_oracle(name, kkt, mmpc_mod, oracle):
    ks = {"auto": mmpc_mod.KKT_AUTO, "riccati": mmpc_mod.KKT_RICCATI, "group": mmpc_mod.KKT_RICCATI_GROUP}[kkt]
    s = solver(mmpc_mod, name, kkt_solver=ks)
    assert s.info.model_id == mmpc_mod.MODEL_USER
    mid = oracle.use_user_model(name)
    B = 96
    x0, up, tr = instances(s.nx, s.nu, B, s.N, s.h)
    w = weights(s.nx, s.nu)
    g = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(s.N, s.h, x0, up, tr, w, model=mid, solver=s)
    compare(g, o)
    assert np.array_equal(g["V"][:, :s.nx], x0)  # x_0 pinned (ModelControl.cpp:144-145)
    s.close()


def test_generated_double_pendulum_equals_builtin(mmpc_mod, oracle, tmp_path):
    """The reference's SX double pendulum through its generated library vs the built-in 2-link kernels."""
    s = solver(mmpc_mod, "nonlinear_double_pendulum")
    builtin = mmpc_mod.Solver(mmpc_mod.write_model_json(str(tmp_path / "dp.json"), "dp", 4, 2, 2000, s.N,
                                                        model="two_link_arm"), kkt_solver=mmpc_mod.KKT_RICCATI_GROUP)
    x0, up, tr = oracle.synth(20250213, 0, 256, s.N, s.h)
    w = np.array(WEIGHTS_CFG)
    a = s.solve_batch_host(x0, up, tr, w)
    b = builtin.solve_batch_host(x0, up, tr, w)
    compare(a, b)


def test_generated_model_bounded(mmpc_mod, oracle):
    s = solver(mmpc_mod, "cart_pole")
    mid = oracle.use_user_model("cart_pole")
    x0, up, tr = instances(s.nx, s.nu, 64, s.N, s.h, seed=11)
    tr *= 4.0  # targets the force bound keeps out of reach
    w = weights(s.nx, s.nu)
    lb, ub = np.array([-1.5]), np.array([1.5])
    g = s.solve_batch_host(x0, up, tr, w, u_lb=lb, u_ub=ub)
    o = oracle.solve_batch(s.N, s.h, x0, up, tr, w, model=mid, u_lb=lb, u_ub=ub, solver=s)
    compare(g, o, tight=1e-8)
    U = g["V"][:, :-s.nx].reshape(64, s.N, s.nx + s.nu)[:, :, s.nx:]
    assert U.min() >= -1.5 and U.max() <= 1.5
    assert (np.abs(np.abs(U) - 1.5) < 1e-12).any()  # some bounds are active


def test_generated_linear_model(mmpc_mod, oracle):
    s = solver(mmpc_mod, "linear_double_pendulum")
    assert s.info.is_linear == 1
    mid = oracle.use_user_model("linear_double_pendulum")
    x0, up, tr = oracle.synth(20250213, 0, 64, s.N, s.h)
    w = np.array(WEIGHTS_CFG)
    g = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(s.N, s.h, x0, up, tr, w, model=mid, is_linear=True)
    assert (g["iters"] == 1).all()  # a convex QP: one Gauss-Newton step is exact
    compare(g, o)


@pytest.mark.parametrize("name", MODELS)
def test_generated_linearize(name, mmpc_mod, oracle):
    s = solver(mmpc_mod, name)
    m = oracle.UserModelHost(name)
    rng = np.random.default_rng(2)
    x = rng.uniform(-1, 1, (32, s.nx))
    u = rng.uniform(-1, 1, (32, s.nu))
    A, Bm, xd = s.linearize_host(x, u)
    for b in range(32):
        A0, B0, xd0 = m.jac(x[b], u[b])
        np.testing.assert_allclose(A[b], A0, rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(Bm[b], B0, rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(xd[b], xd0, rtol=1e-13, atol=1e-13)


def test_closed_loop_example_on_generated_model(tmp_path):
    """model_control_example through ModelControl + the generated library (dll_filepath) equals the same closed
    loop on the built-in model."""
    exe = os.path.join(HOST, "bin", "model_control_example")
    model = os.path.join(USER, "nonlinear_double_pendulum")
    if not os.path.exists(exe) or not os.path.exists(model + ".so"):
        pytest.skip("example or generated model missing")
    run = lambda *a: subprocess.run([exe, "20", "0.1", "n", *a], cwd=tmp_path, capture_output=True, text=True,
                                    timeout=120)
    r_sx, r_builtin = run(model), run()
    assert r_sx.returncode == 0, r_sx.stderr
    assert r_builtin.returncode == 0, r_builtin.stderr
    rows = lambda out: np.array([[float(v) for v in l.split(",")] for l in out.splitlines() if l[:1].isdigit()])
    a, b = rows(r_sx.stdout), rows(r_builtin.stdout)
    assert a.shape == b.shape and a.shape[0] == 50
    assert (a[:, 7] == 0).all()
    np.testing.assert_allclose(a[:, :7], b[:, :7], rtol=1e-8, atol=1e-9)


@pytest.mark.parametrize("kkt", ["group", "riccati"])
def test_generated_model_state_bounds(kkt, mmpc_mod, oracle):
    """State bounds on a generated model (interior-point variant compiled into <name>.so): cart-pole with the
    cart position in [-0.2, 0.2] m and the pole rate in [-1, 1] rad/s, against the oracle on the same dynamics."""
    ks = mmpc_mod.KKT_RICCATI_GROUP if kkt == "group" else mmpc_mod.KKT_RICCATI
    s = solver(mmpc_mod, "cart_pole", kkt_solver=ks, max_iter=100)
    mid = oracle.use_user_model("cart_pole")
    xl, xu = np.array([-0.2, -np.inf, -np.inf, -1.0]), np.array([0.2, np.inf, np.inf, 1.0])
    s.set_state_bounds(xl, xu)
    x0, up, tr = instances(s.nx, s.nu, 64, s.N, s.h, seed=5)
    x0[:, 0] = np.clip(x0[:, 0], -0.15, 0.15)
    x0[:, 3] = np.clip(x0[:, 3], -0.9, 0.9)
    tr *= 3.0
    w = weights(s.nx, s.nu)
    g = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(s.N, s.h, x0, up, tr, w, model=mid, x_lb=xl, x_ub=xu, max_iter=100)
    compare(g, o)
    X = np.stack([g["V"][:, k * 5:k * 5 + 4] for k in range(1, s.N + 1)], 1)
    assert (X >= xl - 1e-12).all() and (X <= xu + 1e-12).all()
    assert (np.abs(np.abs(X[:, :, 0]) - 0.2) < 1e-6).any()  # the position bound is active somewhere
