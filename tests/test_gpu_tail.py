"""GPU: the iteration-tail hand-over of lane-kernel solves: instances still unconverged at the stop
test of iteration `cap` stop in the lane kernel and continue in a 16-lane resume launch from the same iterate,
iteration count and l1-merit weight.  Same algorithm in both kernels, so the results match the oracle as every
same-algorithm comparison does (tests/test_gpu_parity.py _compare: V* within 1e-10 where the iteration counts agree,
>= 99 % of the instances) and match a solve without hand-over to roundoff.  MMPC_TAIL_CAP (read at handle creation)
forces the cap; 2 hands over most cfg#3 instances, and B = 4096 exceeds the resume launch's slots (3072 on 256 CUs),
so the overflow path (instances that keep iterating in the lane kernel) runs too."""
import numpy as np
import pytest

from test_gpu_parity import _compare, _rel

pytestmark = pytest.mark.gpu

H = 0.002
W_EXO = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)


def _solve(mmpc_mod, tmp_path, monkeypatch, cap, B, N=50, seed=20250213, **kw):
    monkeypatch.setenv("MMPC_TAIL_CAP", str(cap))
    p = mmpc_mod.write_model_json(str(tmp_path / f"exo_{cap}_{N}.json"), "exo", 8, 4, 2000, N, model="exo_arm")
    s = mmpc_mod.Solver(p, kkt_solver=2, init_states=mmpc_mod.INIT_ZERO, **kw)
    monkeypatch.delenv("MMPC_TAIL_CAP")
    return s


@pytest.mark.parametrize("cap,B,hess", [(2, 4096, 1), (3, 640, 1), (4, 512, 2)])
def test_tail_handover_vs_oracle(cap, B, hess, mmpc_mod, oracle, tmp_path, monkeypatch):
    N = 50
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=oracle.EXO)
    s = _solve(mmpc_mod, tmp_path, monkeypatch, cap, B, hessian=hess)
    r = s.solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO, kkt=oracle.KKT_RICCATI, init_states=2,
                           hessian=oracle.HESS_EXACT if hess == 2 else oracle.HESS_GAUSS_NEWTON)
    assert (r["status"] == 0).all() and (o["status"] == 0).all()
    assert (r["iters"] > cap).sum() > 0   # some instances did continue past the cap
    _compare(r, o)
    off = _solve(mmpc_mod, tmp_path, monkeypatch, 0, B, hessian=hess).solve_batch_host(x0, up, tr, W_EXO)
    assert (off["iters"] == r["iters"]).mean() >= 0.99
    same = off["iters"] == r["iters"]
    assert _rel(r["V"][same], off["V"][same]).max() <= 1e-10


def test_tail_handover_device_api_and_u0(mmpc_mod, oracle, tmp_path, monkeypatch):
    """the device-pointer entry with u_0* in host-mapped memory: handed-over instances' u_0*, status and iterations
    come from the resume launch"""
    import torch
    B, N = 300, 50
    x0, up, tr = oracle.synth(7, 11, B, N, H, model=oracle.EXO)
    s = _solve(mmpc_mod, tmp_path, monkeypatch, 2, B)
    d = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda:0")
    V = torch.zeros((B, s.NV), dtype=torch.float64, device="cuda:0")
    st = torch.full((B,), -1, dtype=torch.int32, device="cuda:0")
    it = torch.zeros_like(st)
    hb = mmpc_mod.HostBuffer(B * 4 * 8)
    u0 = hb.view(0, np.float64, B * 4)
    s.solve_batch(B, d(x0), d(up), d(tr), d(W_EXO), V, st, it, None, u0=u0)
    torch.cuda.synchronize()
    Vh = V.cpu().numpy()
    assert (st.cpu().numpy() == 0).all() and (it.cpu().numpy() >= 3).all()
    assert np.array_equal(u0.reshape(B, 4), Vh[:, 8:12])
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO, kkt=oracle.KKT_RICCATI, init_states=2)
    _compare(dict(V=Vh, status=st.cpu().numpy(), iters=it.cpu().numpy()), o)
    hb.close()


def test_tail_handover_fp32_factor_escalates_to_fp64(mmpc_mod, oracle, tmp_path, monkeypatch):
    """cfg#5 (fp32 Riccati factor): the handed-over tail continues with the fp64 factor from the same iterate, so
    the stop test (fp64 residuals, unchanged) holds on every instance and V* is the fp64 solution to the stop test's
    accuracy (1e-6 relative, as tests/test_gpu_riccati.py's fp32 tests)"""
    B, N = 768, 50
    x0, up, tr = oracle.synth(20250213, 3, B, N, H, model=oracle.EXO)
    r = _solve(mmpc_mod, tmp_path, monkeypatch, 2, B, factor_fp32=1).solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO, kkt=oracle.KKT_RICCATI, init_states=2)
    assert (r["status"] == 0).all(), np.bincount(r["status"])
    assert (r["kkt"] <= 1e-8).all()
    assert (r["iters"] > 2).sum() > B // 2
    assert _rel(r["V"], o["V"]).max() <= 1e-6
    off = _solve(mmpc_mod, tmp_path, monkeypatch, 0, B, factor_fp32=1).solve_batch_host(x0, up, tr, W_EXO)
    assert _rel(r["V"], off["V"]).max() <= 1e-6


def test_tail_handover_wave_rule_loose_tolerance(mmpc_mod, oracle, tmp_path, monkeypatch):
    """the wave rule (hand over from iteration 2 once at most MMPC_TAIL_WAVE lanes of a wave are left) at the
    reference's IPOPT tolerance (tol 1e-5, defects 1e-7), where the stragglers need the 4th iteration: same iterates
    as without hand-over, against the oracle with the same tolerances"""
    B, N, tg, td = 1024, 50, 1e-5, 1e-7
    x0, up, tr = oracle.synth(20250213, 5, B, N, H, model=oracle.EXO)
    monkeypatch.setenv("MMPC_TAIL_WAVE", "16")
    s = _solve(mmpc_mod, tmp_path, monkeypatch, 9, B, tol_grad=tg, tol_defect=td)
    monkeypatch.delenv("MMPC_TAIL_WAVE")
    r = s.solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO, kkt=oracle.KKT_RICCATI, init_states=2,
                           tol_grad=tg, tol_defect=td)
    assert (r["status"] == 0).all()
    _compare(r, o)
    off = _solve(mmpc_mod, tmp_path, monkeypatch, 0, B, tol_grad=tg, tol_defect=td).solve_batch_host(x0, up, tr, W_EXO)
    assert (off["iters"] == r["iters"]).mean() >= 0.99
    same = off["iters"] == r["iters"]
    assert _rel(r["V"][same], off["V"][same]).max() <= 1e-10


@pytest.mark.parametrize("model,wave,B", [("exo", 8, 512), ("exo", 40, 320), ("two_link", 24, 768)])
def test_tail_handover_state_bounds(model, wave, B, mmpc_mod, oracle, tmp_path, monkeypatch):
    """state-bounded (interior-point) lane solves hand over by the wave rule: the resume launch reads the duals from
    the lane launch's workspace and continues with the same barrier parameter and merit weight -- same iterates as
    without hand-over and as the oracle's interior-point solve (oracle solve_one_ip)"""
    from conftest import WEIGHTS_CFG
    if model == "exo":
        nx, nu, N, w, mname, om = 8, 4, 50, W_EXO, "exo_arm", oracle.EXO
        xl, xu = [-np.inf] * 4 + [-1.5] * 4, [np.inf] * 4 + [1.5] * 4
    else:
        nx, nu, N, w, mname, om = 4, 2, 30, np.array(WEIGHTS_CFG), "two_link_arm", oracle.TWO_LINK
        xl, xu = [-np.inf] * 2 + [-1.5] * 2, [np.inf] * 2 + [1.5] * 2
    x0, up, tr = oracle.synth(20250213, 9, B, N, H, model=om)

    def solver(wave_max):
        monkeypatch.setenv("MMPC_TAIL_WAVE", str(wave_max))
        p = mmpc_mod.write_model_json(str(tmp_path / f"{model}_xb_{wave_max}.json"), model, nx, nu, 2000, N, model=mname)
        s = mmpc_mod.Solver(p, kkt_solver=2, init_states=mmpc_mod.INIT_ZERO)
        monkeypatch.delenv("MMPC_TAIL_WAVE")
        s.set_state_bounds(xl, xu)
        return s

    r = solver(wave).solve_batch_host(x0, up, tr, w)
    o = oracle.solve_batch(N, H, x0, up, tr, w, model=om, kkt=oracle.KKT_RICCATI, init_states=2, x_lb=xl, x_ub=xu)
    assert (r["status"] == 0).all() and (o["status"] == 0).all()
    _compare(r, o)
    off = solver(0).solve_batch_host(x0, up, tr, w)
    assert (off["iters"] == r["iters"]).mean() >= 0.99
    same = off["iters"] == r["iters"]
    assert _rel(r["V"][same], off["V"][same]).max() <= 1e-10


@pytest.mark.parametrize("model,ub,cap,B,hess", [("exo", 0.5, 3, 640, 1), ("exo", 2.0, 2, 512, 2),
                                                 ("two_link", 2.0, 3, 768, 1)])
def test_tail_handover_control_bounds(model, ub, cap, B, hess, mmpc_mod, oracle, tmp_path, monkeypatch):
    """control-bounded (projected SQP) lane solves: the resume launch runs the 16-lane kernel with the lane kernel's
    active-set rule (holds only added, four QP solves; SolveParams.no_release) from the handed-over iterate, merit
    weight and hold epsilon -- same iterates as the oracle's projected SQP without releases and as no hand-over"""
    from conftest import WEIGHTS_CFG
    if model == "exo":
        nx, nu, N, w, mname, om = 8, 4, 50, W_EXO, "exo_arm", oracle.EXO
    else:
        nx, nu, N, w, mname, om = 4, 2, 30, np.array(WEIGHTS_CFG), "two_link_arm", oracle.TWO_LINK
    lb, ubv = [-ub] * nu, [ub] * nu
    x0, up, tr = oracle.synth(20250213, 17, B, N, H, model=om)

    def solver(c):
        monkeypatch.setenv("MMPC_TAIL_CAP", str(c))
        p = mmpc_mod.write_model_json(str(tmp_path / f"{model}_ub_{c}.json"), model, nx, nu, 2000, N, model=mname)
        s = mmpc_mod.Solver(p, kkt_solver=2, init_states=mmpc_mod.INIT_ZERO, hessian=hess)
        monkeypatch.delenv("MMPC_TAIL_CAP")
        return s

    s = solver(cap)
    r = s.solve_batch_host(x0, up, tr, w, u_lb=lb, u_ub=ubv)
    o = oracle.solve_batch(N, H, x0, up, tr, w, model=om, u_lb=lb, u_ub=ubv, init_states=2, solver=s)
    assert (r["iters"] > cap).sum() > 0
    np.testing.assert_array_equal(r["status"], o["status"])
    _compare(r, o)
    off = solver(0).solve_batch_host(x0, up, tr, w, u_lb=lb, u_ub=ubv)
    assert (off["iters"] == r["iters"]).mean() >= 0.99
    same = off["iters"] == r["iters"]
    assert _rel(r["V"][same], off["V"][same]).max() <= 1e-10


@pytest.mark.parametrize("B", [1, 3, 65])
def test_tail_handover_tiny_and_ragged_batches(B, mmpc_mod, oracle, tmp_path, monkeypatch):
    """one partial wave (B < 64) and a ragged last wave (65): the wave rule counts only the lanes of real instances
    (the others left the kernel at its first line), the resume launch's slots are clamped to B -- unbounded and
    state-bounded exo lane solves, against the oracle"""
    N = 50
    x0, up, tr = oracle.synth(20250213, 31, B, N, H, model=oracle.EXO)
    s = _solve(mmpc_mod, tmp_path, monkeypatch, 4, B)
    r = s.solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO, kkt=oracle.KKT_RICCATI, init_states=2)
    assert (r["status"] == 0).all()
    _compare(r, o)
    xl, xu = [-np.inf] * 4 + [-1.5] * 4, [np.inf] * 4 + [1.5] * 4
    s.set_state_bounds(xl, xu)
    r = s.solve_batch_host(x0, up, tr, W_EXO)
    o = oracle.solve_batch(N, H, x0, up, tr, W_EXO, model=oracle.EXO, kkt=oracle.KKT_RICCATI, init_states=2,
                           x_lb=xl, x_ub=xu)
    assert (r["status"] == 0).all()
    _compare(r, o)


def test_batch_composition_single_instance_vs_full_batch(mmpc_mod, oracle, tmp_path):
    """VERDICT r5 ask 7: the hand-over decides by an instance's wave-mates (the wave rule) and by the slots, so the same
    instance solved alone (B = 1, ModelControl::calc_u's call, ModelControl.cpp:159) -- where from iteration 2 on it is
    the only lane of its wave and continues in the 16-lane resume launch -- and inside the full cfg#3 batch agree to
    1e-10 relative in V* with identical iteration counts on >= 99 % of the instances, not bit for bit (include/mmpc.h,
    mmpc_opts.tail_cap).  With the hand-over off (opts.tail_cap = 0) every lane is independent: bit for bit."""
    N, B = 50, 65536
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=oracle.EXO)
    p = mmpc_mod.write_model_json(str(tmp_path / "exo_comp.json"), "exo", 8, 4, 2000, N, model="exo_arm")
    full = mmpc_mod.Solver(p, kkt_solver=2, init_states=mmpc_mod.INIT_ZERO).solve_batch_host(x0, up, tr, W_EXO)
    assert (full["status"] == 0).all()
    pick = np.linspace(0, B - 1, 128).astype(int)
    one = mmpc_mod.Solver(p, kkt_solver=2, init_states=mmpc_mod.INIT_ZERO)
    alone = [one.solve_batch_host(x0[i:i + 1], up[i:i + 1], tr[i:i + 1], W_EXO) for i in pick]
    it1 = np.array([a["iters"][0] for a in alone])
    V1 = np.stack([a["V"][0] for a in alone])
    assert all(a["status"][0] == 0 for a in alone)
    same = it1 == full["iters"][pick]
    assert same.mean() >= 0.99, (it1[~same], full["iters"][pick][~same])
    assert _rel(V1[same], full["V"][pick][same]).max() <= 1e-10
    assert (it1 >= 2).all()   # every single-instance solve reached the wave rule's iteration
    # hand-over off through the options (ABI 6): the lane kernel alone, bit for bit in and out of the batch
    off = mmpc_mod.Solver(p, kkt_solver=2, init_states=mmpc_mod.INIT_ZERO, tail_cap=0)
    sub = np.arange(0, B, 4096)
    offb = off.solve_batch_host(x0[:4096 * 2], up[:4096 * 2], tr[:4096 * 2], W_EXO)
    for i in sub[:2]:
        a = off.solve_batch_host(x0[i:i + 1], up[i:i + 1], tr[i:i + 1], W_EXO)
        np.testing.assert_array_equal(a["V"][0], offb["V"][i])
        assert a["iters"][0] == offb["iters"][i]
