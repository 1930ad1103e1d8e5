"""GPU parity: the HIP solve path (through the C-ABI) against the CPU oracle and the committed golden
fixtures, plus size-independent properties at the full cfg#2 size (B = 4096).

Tolerances (stated per test):
  * GPU vs oracle, same algorithm: V* within 1e-10 relative to max|V| and identical iteration counts
    for >= 99 % of instances; where the counts differ (a stop test landing on either side of its
    threshold after roundoff) within the solution accuracy the stop test guarantees, 1e-6.
  * GPU vs scipy golden (independent solver): V* within 1e-6 relative, J* within 1e-8 relative.
"""
import math
import os

import numpy as np
import pytest

from conftest import WEIGHTS_CFG

pytestmark = pytest.mark.gpu

H = 0.002


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _cases(g):
    cs = g["cases"]
    return (np.array([c["x0"] for c in cs]), np.array([c["u_prev"] for c in cs]),
            np.array([c["traj"] for c in cs]), np.array([c["V"] for c in cs]), np.array([c["J"] for c in cs]))


def _rel(a, b):
    return np.abs(a - b).max(1) / np.maximum(np.abs(b).max(1), 1e-300)


def _compare(gpu, orc, tol_same=1e-10, tol_diff=1e-6, min_same=0.99, dump=None):
    """Same algorithm on both sides: identical iteration counts except where a stop test lands within
    roundoff of its threshold (allowed for max(2, 1 %) of the instances); V* within tol_same (SURVEY.md A9:
    1e-10 relative, same algorithm) where the counts agree and within the stop test's accuracy (tol_diff)
    where they differ.  MMPC_TEST_DUMP=1 saves the inputs of status mismatches under gpurun_out/."""
    same = gpu["iters"] == orc["iters"]
    bad_status = gpu["status"] != orc["status"]
    if os.environ.get("MMPC_TEST_LOG"):   # diagnostics: the achieved agreement of every comparison
        with open(os.environ["MMPC_TEST_LOG"], "a") as f:
            r = _rel(gpu["V"], orc["V"])
            f.write(f"{os.environ.get('PYTEST_CURRENT_TEST', '?')} n={len(same)} same={int(same.sum())} "
                    f"max_rel_same={r[same].max() if same.any() else 0:.3e} max_rel={r.max():.3e}\n")
    if dump is not None and bad_status.any() and os.environ.get("MMPC_TEST_DUMP"):
        os.makedirs(os.path.dirname(dump), exist_ok=True)
        np.savez(dump, idx=np.where(bad_status)[0], gpu_status=gpu["status"][bad_status],
                 orc_status=orc["status"][bad_status], gpu_iters=gpu["iters"][bad_status],
                 orc_iters=orc["iters"][bad_status], **{k: v[bad_status] for k, v in dump_inputs.items()})
    n = len(same)
    assert (~same).sum() <= max(2, int((1.0 - min_same) * n)), (gpu["iters"][~same], orc["iters"][~same])
    rel = _rel(gpu["V"], orc["V"])
    assert rel[same].max() <= tol_same, rel[same].max()
    if (~same).any():
        assert rel[~same].max() <= tol_diff
    np.testing.assert_array_equal(gpu["status"], orc["status"])


dump_inputs = {}


def test_linearize_vs_golden(golden_kat, model_json, mmpc_mod, torch_cuda):
    """mmpc_linearize_batch (replaces <name>_get_A/_get_B/_get_x_dot_init) vs the sympy fixtures."""
    s = mmpc_mod.Solver(model_json())
    pts = golden_kat["K3"]["points"] + [dict(x=[0, 0, 0, 0], u=[0, 0], A=golden_kat["K2"]["A"],
                                             B=golden_kat["K2"]["B"], xdot=golden_kat["K2"]["xdot"])]
    A, Bm, xd = s.linearize_host([p["x"] for p in pts], [p["u"] for p in pts])
    for i, p in enumerate(pts):
        np.testing.assert_allclose(A[i], p["A"], rtol=1e-11, atol=1e-11)
        np.testing.assert_allclose(Bm[i], p["B"], rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(xd[i], p["xdot"], rtol=1e-12, atol=1e-12)


def test_linearize_column_major(model_json, mmpc_mod, torch_cuda):
    """raw device call returns CasADi column-major order (ModelControl.cpp:127-129)"""
    torch = torch_cuda
    s = mmpc_mod.Solver(model_json())
    x = torch.tensor([[0.3, -0.2, 0.5, 0.1]], dtype=torch.float64, device="cuda")
    u = torch.tensor([[1.0, -2.0]], dtype=torch.float64, device="cuda")
    A = torch.zeros(16, dtype=torch.float64, device="cuda")
    Bm = torch.zeros(8, dtype=torch.float64, device="cuda")
    s.linearize(1, x, u, A, Bm, None)
    torch.cuda.synchronize()
    import oracle_lib
    Ao, Bo, _ = oracle_lib.two_link_jac(x.cpu().numpy()[0], u.cpu().numpy()[0])
    np.testing.assert_allclose(A.cpu().numpy(), Ao.T.reshape(-1), rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(Bm.cpu().numpy(), Bo.T.reshape(-1), rtol=1e-12, atol=1e-13)


def test_synth_matches_oracle(model_json, mmpc_mod, oracle, torch_cuda):
    torch = torch_cuda
    s = mmpc_mod.Solver(model_json())
    B = 1000
    x0 = torch.empty((B, 4), dtype=torch.float64, device="cuda")
    up = torch.empty((B, 2), dtype=torch.float64, device="cuda")
    tr = torch.empty((B, 30, 4), dtype=torch.float64, device="cuda")
    s.synth(20250213, 12345, B, x0, up, tr)
    torch.cuda.synchronize()
    ox, ou, ot = oracle.synth(20250213, 12345, B, 30, H)
    np.testing.assert_array_equal(x0.cpu().numpy(), ox)
    np.testing.assert_array_equal(up.cpu().numpy(), ou)
    # sin/cos of the trajectory differ between OCML and glibc by a few ulp (transcendental, not bitwise)
    np.testing.assert_allclose(tr.cpu().numpy(), ot, rtol=2e-14, atol=2e-15)


@pytest.mark.parametrize("which", ["cfg1", "cfg2"])
def test_solve_vs_scipy_golden(which, golden_cfg1, golden_cfg2, model_json, mmpc_mod, oracle, torch_cuda):
    g = golden_cfg1 if which == "cfg1" else golden_cfg2
    x0, up, tr, Vg, Jg = _cases(g)
    s = mmpc_mod.Solver(model_json(N=g["N"]))
    r = s.solve_batch_host(x0, up, tr, np.array(g["weights"]))
    assert (r["status"] == 0).all(), r["status"]
    assert _rel(r["V"], Vg).max() < 1e-6
    J, dinf = oracle.nlp_eval(g["N"], g["h"], r["V"][0], up[0], tr[0], np.array(g["weights"]))
    assert J == pytest.approx(Jg[0], rel=1e-8)
    o = oracle.solve_batch(g["N"], g["h"], x0, up, tr, np.array(g["weights"]), solver=s)
    _compare(r, o, min_same=1.0)


def test_cfg2_full_batch_vs_oracle(model_json, mmpc_mod, oracle, torch_cuda):
    """Headline config (B = 4096, N = 30): every instance against the oracle on the same inputs."""
    torch = torch_cuda
    B, N = 4096, 30
    s = mmpc_mod.Solver(model_json(N=N))
    x0 = torch.empty((B, 4), dtype=torch.float64, device="cuda")
    up = torch.empty((B, 2), dtype=torch.float64, device="cuda")
    tr = torch.empty((B, N, 4), dtype=torch.float64, device="cuda")
    s.synth(20250213, 0, B, x0, up, tr)
    w = torch.tensor(WEIGHTS_CFG, dtype=torch.float64, device="cuda")
    V = torch.zeros((B, s.NV), dtype=torch.float64, device="cuda")
    st = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    it = torch.zeros(B, dtype=torch.int32, device="cuda")
    kkt = torch.zeros(B, dtype=torch.float64, device="cuda")
    s.solve_batch(B, x0, up, tr, w, V, st, it, kkt)
    torch.cuda.synchronize()
    gpu = dict(V=V.cpu().numpy(), status=st.cpu().numpy(), iters=it.cpu().numpy(), kkt=kkt.cpu().numpy())
    xo, uo, to = x0.cpu().numpy(), up.cpu().numpy(), tr.cpu().numpy()
    orc = oracle.solve_batch(N, H, xo, uo, to, np.array(WEIGHTS_CFG), solver=s)
    nc = np.where((gpu["status"] != 0) | (orc["status"] != 0))[0]
    if len(nc) and os.environ.get("MMPC_TEST_DUMP"):
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez("gpurun_out/cfg2_nonconverged.npz", idx=nc, x0=xo[nc], u_prev=uo[nc], traj=to[nc],
                 gpu_status=gpu["status"][nc], gpu_iters=gpu["iters"][nc], gpu_kkt=gpu["kkt"][nc],
                 orc_status=orc["status"][nc], orc_iters=orc["iters"][nc], orc_kkt=orc["kkt"][nc])
    assert (gpu["status"] == 0).all(), [(int(i), int(gpu["status"][i]), int(gpu["iters"][i]), float(gpu["kkt"][i]),
                                         int(orc["status"][i]), int(orc["iters"][i]), float(orc["kkt"][i])) for i in nc]
    assert (gpu["kkt"] <= 1e-8).all()
    dump_inputs.update(x0=xo, u_prev=uo, traj=to)
    _compare(gpu, orc, dump="gpurun_out/cfg2_status_mismatch.npz")
    dump_inputs.clear()
    # size-independent properties on every instance: pinned x_0, zero defects, stationarity
    assert np.array_equal(gpu["V"][:, :4], xo)
    Jg = torch.zeros(B, dtype=torch.float64, device="cuda")
    dg = torch.zeros(B, dtype=torch.float64, device="cuda")
    s.nlp_eval(B, V, up, tr, w, Jg, dg)
    torch.cuda.synchronize()
    assert dg.cpu().numpy().max() <= 1e-10
    np.testing.assert_allclose(Jg.cpu().numpy(), orc["J"], rtol=1e-10)
    for b in range(0, B, 257):
        U = gpu["V"][b].reshape(-1)[[6 * k + 4 + c for k in range(N) for c in range(2)]]
        gr = oracle.reduced_gradient(N, H, xo[b], U, uo[b], to[b], np.array(WEIGHTS_CFG))
        assert np.abs(gr).max() < 1e-7


def test_warm_start_fixed_point_and_determinism(model_json, mmpc_mod, oracle):
    x0, up, tr = oracle.synth(99, 0, 256, 30, H)
    s = mmpc_mod.Solver(model_json())
    w = np.array(WEIGHTS_CFG)
    r1 = s.solve_batch_host(x0, up, tr, w)
    r1b = s.solve_batch_host(x0, up, tr, w)
    np.testing.assert_array_equal(r1["V"], r1b["V"])          # bitwise deterministic
    r2 = s.solve_batch_host(x0, up, tr, w, V=r1["V"])          # ModelControl.cpp:160-161 warm start
    assert (r2["iters"] == 0).all() and (r2["status"] == 0).all()
    np.testing.assert_array_equal(r2["V"], r1["V"])


@pytest.mark.parametrize("N", [1, 2, 16, 20, 25, 31, 32])
def test_horizons(N, model_json, mmpc_mod, oracle):
    """ragged horizons incl. N = 1 and the kernel maximum N*nu = 64"""
    x0, up, tr = oracle.synth(5, 0, 64, N, H)
    s = mmpc_mod.Solver(model_json(N=N))
    w = np.array(WEIGHTS_CFG)
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w, solver=s)
    _compare(r, o)


def test_horizon_too_long_for_condensed_is_api_error(model_json, mmpc_mod, oracle):
    # N*nu > 64 does not fit the condensed kernel: an explicit request is an API error (no fallback);
    # MMPC_KKT_AUTO routes it to the Riccati kernel (tests/test_gpu_riccati.py)
    x0, up, tr = oracle.synth(5, 0, 2, 33, H)
    s = mmpc_mod.Solver(model_json(N=33), kkt_solver=mmpc_mod.KKT_CONDENSED)
    with pytest.raises(mmpc_mod.MmpcError) as ei:
        s.solve_batch_host(x0, up, tr, np.array(WEIGHTS_CFG))
    assert ei.value.code == -4


def test_linear_mode(model_json, mmpc_mod, oracle):
    x0, up, tr = oracle.synth(11, 0, 128, 25, H)
    s = mmpc_mod.Solver(model_json(N=25, name="linear_double_pendulum", is_linear=True))
    w = np.array(WEIGHTS_CFG)
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(25, H, x0, up, tr, w, is_linear=True)
    assert (r["iters"] == 1).all()
    _compare(r, o, min_same=1.0)


def test_per_instance_weights(model_json, mmpc_mod, oracle):
    x0, up, tr = oracle.synth(13, 0, 64, 30, H)
    rng = np.random.default_rng(0)
    w = np.tile(WEIGHTS_CFG, (64, 1)) * rng.uniform(0.5, 2.0, (64, 8))
    s = mmpc_mod.Solver(model_json())
    r = s.solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(30, H, x0, up, tr, w, solver=s)
    _compare(r, o)


def test_bounds_enforced(model_json, mmpc_mod, oracle):
    """u bounds are enforced (projected SQP; tests/test_gpu_bounds.py covers them in depth)"""
    x0, up, tr = oracle.synth(20250213, 0, 32, 30, H)
    s = mmpc_mod.Solver(model_json())
    w = np.array(WEIGHTS_CFG)
    r = s.solve_batch_host(x0, up, tr, w, u_lb=[-1e31, -1e31], u_ub=[1e31, 1e31])
    assert (r["status"] == 0).all()
    r = s.solve_batch_host(x0, up, tr, w, u_lb=[-1e-3, -1e-3], u_ub=[1e-3, 1e-3])
    o = oracle.solve_batch(30, H, x0, up, tr, w, u_lb=[-1e-3, -1e-3], u_ub=[1e-3, 1e-3], solver=s)
    _compare(r, o)
    assert (r["status"] == 0).all()
    assert np.abs(r["V"][:, [6 * k + 4 + c for k in range(30) for c in range(2)]]).max() <= 1e-3


def test_nonfinite_and_max_iter(model_json, mmpc_mod, oracle):
    x0, up, tr = oracle.synth(1, 0, 4, 30, H)
    x0[1, 0] = math.nan
    tr[2, 3, 1] = math.inf
    s = mmpc_mod.Solver(model_json())
    r = s.solve_batch_host(x0, up, tr, np.array(WEIGHTS_CFG))
    assert list(r["status"]) == [0, 3, 3, 0]
    s2 = mmpc_mod.Solver(model_json(), max_iter=1)
    r2 = s2.solve_batch_host(x0[[0, 3]], up[[0, 3]], tr[[0, 3]], np.array(WEIGHTS_CFG))
    o2 = oracle.solve_batch(30, H, x0[[0, 3]], up[[0, 3]], tr[[0, 3]], np.array(WEIGHTS_CFG), max_iter=1, solver=s2)
    assert (r2["status"] == 1).all() and (r2["iters"] == 1).all()
    assert _rel(r2["V"], o2["V"]).max() < 1e-10


def test_warm_start_perturbed_state(model_json, mmpc_mod, oracle):
    """The reference's steady-state tick (ModelControl.cpp:144-145,160-161): warm start from the previous solution
    with a slightly moved measured state.  theta_0 is then below IPOPT's theta_min, so the first iteration is an
    Armijo (f-type) one in the kernels as in the oracle (sqp_wave.h first_iter_filter_accepts); GPU = oracle, and
    the first accepted step does not increase the constraint violation."""
    N, B = 30, 256
    x0, up, tr = oracle.synth(20250213, 300, B, N, H)
    w = np.array(WEIGHTS_CFG)
    s = mmpc_mod.Solver(model_json(N=N))
    r1 = s.solve_batch_host(x0, up, tr, w)
    assert (r1["status"] == 0).all()
    x0p = x0 + np.random.default_rng(5).uniform(-1e-7, 1e-7, x0.shape)
    Vw = r1["V"].copy()
    Vw[:, :4] = x0p
    g = s.solve_batch_host(x0p, up, tr, w, V=Vw)
    o = oracle.solve_batch(N, H, x0p, up, tr, w, V=Vw, solver=s)
    assert (g["status"] == 0).all()
    _compare(g, o)
    s1 = mmpc_mod.Solver(model_json(N=N), max_iter=1)
    g1 = s1.solve_batch_host(x0p, up, tr, w, V=Vw)
    o1 = oracle.solve_batch(N, H, x0p, up, tr, w, V=Vw, max_iter=1, solver=s1)
    assert _rel(g1["V"], o1["V"]).max() < 1e-10
    for b in range(0, B, 17):
        _, c0 = oracle.nlp_eval(N, H, Vw[b], up[b], tr[b], w)
        _, c1 = oracle.nlp_eval(N, H, g1["V"][b], up[b], tr[b], w)
        assert np.abs(c1).sum() <= np.abs(c0).sum() <= 1e-4
