"""GPU: mmpc_solve_batch_u0 -- u_0* (the control ModelControl::calc_u returns, ModelControl.cpp:174-190) written
by the solve kernel, to device memory or straight into pinned host memory from mmpc_host_alloc (mmpc.HostBuffer).

* every KKT solver (condensed, 16-lane group, lane Riccati), unbounded and with control bounds, and the exo model:
  u0 equals V[:, nx:nx+nu] of the same solve bit for bit, status / iterations stored into host memory equal the
  device-memory ones, and V equals a plain mmpc_solve_batch solve bit for bit;
* a solve into host memory is visible to the host after a stream synchronisation (no copy issued).
"""
import numpy as np
import pytest
import torch

from conftest import WEIGHTS_CFG

pytestmark = pytest.mark.gpu


def _inputs(s, B, N, nx, nu, seed=20250213):
    f = dict(dtype=torch.float64, device="cuda")
    x0 = torch.empty((B, nx), **f)
    up = torch.empty((B, nu), **f)
    tr = torch.empty((B, N, nx), **f)
    s.synth(seed, 0, B, x0, up, tr)
    return x0, up, tr


@pytest.mark.parametrize("solver,bounded", [("condensed", False), ("condensed", True), ("group", False),
                                            ("group", True), ("lane", False), ("lane", True)])
def test_u0_host_and_device_match_V(solver, bounded, model_json, mmpc_mod):
    N, B, nx, nu = 30, 256, 4, 2
    ks = {"condensed": mmpc_mod.KKT_CONDENSED, "group": mmpc_mod.KKT_RICCATI_GROUP,
          "lane": mmpc_mod.KKT_RICCATI}[solver]
    s = mmpc_mod.Solver(model_json(N=N), kkt_solver=ks)
    x0, up, tr = _inputs(s, B, N, nx, nu)
    w = torch.tensor(WEIGHTS_CFG, dtype=torch.float64, device="cuda")
    lb = torch.tensor([-3.0, -3.0], dtype=torch.float64, device="cuda") if bounded else None
    ub = torch.tensor([3.0, 3.0], dtype=torch.float64, device="cuda") if bounded else None
    i32 = dict(dtype=torch.int32, device="cuda")
    # reference: the plain entry point
    V0 = torch.zeros((B, s.NV), dtype=torch.float64, device="cuda")
    st0, it0 = torch.zeros(B, **i32), torch.zeros(B, **i32)
    s.solve_batch(B, x0, up, tr, w, V0, st0, it0, u_lb=lb, u_ub=ub)
    # u0 to device memory
    V1 = torch.zeros_like(V0)
    u0d = torch.full((B, nu), np.nan, dtype=torch.float64, device="cuda")
    s.solve_batch(B, x0, up, tr, w, V1, st0.clone(), it0.clone(), u_lb=lb, u_ub=ub, u0=u0d)
    # u0 / status / iters straight into pinned host memory
    hb = mmpc_mod.HostBuffer(B * (8 * nu + 8))
    u0h = hb.view(0, np.float64, B * nu)
    sth = hb.view(B * nu * 8, np.int32, B)
    ith = hb.view(B * nu * 8 + 4 * B, np.int32, B)
    u0h[:] = np.nan
    sth[:] = -1
    ith[:] = -1
    V2 = torch.zeros_like(V0)
    s.solve_batch(B, x0, up, tr, w, V2, sth, ith, u_lb=lb, u_ub=ub, u0=u0h)
    torch.cuda.synchronize()
    Vr = V0.cpu().numpy()
    assert (st0.cpu().numpy() == 0).all()
    assert np.array_equal(V1.cpu().numpy(), Vr) and np.array_equal(V2.cpu().numpy(), Vr)
    assert np.array_equal(u0d.cpu().numpy(), Vr[:, nx:nx + nu])
    assert np.array_equal(u0h.reshape(B, nu), Vr[:, nx:nx + nu])
    assert np.array_equal(sth, st0.cpu().numpy()) and np.array_equal(ith, it0.cpu().numpy())
    if bounded:
        assert (np.abs(u0h) <= 3.0).all()
    hb.close()
    s.close()


def test_u0_exo_lane(mmpc_mod, tmp_path):
    N, B, nx, nu = 50, 128, 8, 4
    path = mmpc_mod.write_model_json(str(tmp_path / "exo.json"), "exo", nx, nu, 2000, N, model="exo_arm")
    s = mmpc_mod.Solver(path)
    assert s.kkt_solver_for(B) == mmpc_mod.KKT_RICCATI
    x0, up, tr = _inputs(s, B, N, nx, nu)
    w = torch.tensor([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4, dtype=torch.float64, device="cuda")
    V = torch.zeros((B, s.NV), dtype=torch.float64, device="cuda")
    hb = mmpc_mod.HostBuffer(B * (8 * nu + 8))
    u0h = hb.view(0, np.float64, B * nu)
    sth = hb.view(B * nu * 8, np.int32, B)
    ith = hb.view(B * nu * 8 + 4 * B, np.int32, B)
    s.solve_batch(B, x0, up, tr, w, V, sth, ith, u0=u0h)
    torch.cuda.synchronize()
    Vr = V.cpu().numpy()
    assert (sth == 0).all() and (ith >= 1).all()
    assert np.array_equal(u0h.reshape(B, nu), Vr[:, nx:nx + nu])
    hb.close()
    s.close()
