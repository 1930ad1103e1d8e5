"""GPU: the one-process multi-device C-ABI (mmpc_multi_*).  On the 1-GPU pool the device list repeats
device 0 (each entry gets its own handle, stream, workspace and staging, so the shard / concurrent-solve / in-place
assembly logic runs exactly as on G devices); results must equal a single-handle solve of the whole batch bit for
bit, for ragged splits, per-instance weights (weights_stride), control bounds and warm starts."""
import numpy as np
import pytest

from conftest import WEIGHTS_CFG

pytestmark = pytest.mark.gpu
H = 0.002


@pytest.mark.parametrize("G", [1, 3, 8])
def test_multi_device_equals_single_device(G, model_json, mmpc_mod, oracle):
    B, N = 1001, 30
    x0, up, tr = oracle.synth(20250213, 0, B, N, H)
    path = model_json(N=N)
    single = mmpc_mod.Solver(path)
    multi = mmpc_mod.MultiSolver(path, [0] * G)
    assert multi.num_devices() == G
    w = np.array(WEIGHTS_CFG)
    a = single.solve_batch_host(x0, up, tr, w)
    b = multi.solve_batch_host(x0, up, tr, w)
    for k in ("V", "status", "iters", "kkt"):
        np.testing.assert_array_equal(a[k], b[k])
    assert (b["status"] == 0).all()
    # per-instance weights, bounds, warm start: the shard offsets apply to every strided input
    rng = np.random.default_rng(3)
    wi = np.tile(WEIGHTS_CFG, (B, 1)) * rng.uniform(0.5, 2.0, (B, 8))
    lb, ub = np.array([-20.0, -20.0]), np.array([20.0, 20.0])
    a = single.solve_batch_host(x0, up, tr, wi, V=a["V"], u_lb=lb, u_ub=ub)
    b = multi.solve_batch_host(x0, up, tr, wi, V=b["V"], u_lb=lb, u_ub=ub)
    for k in ("V", "status", "iters", "kkt"):
        np.testing.assert_array_equal(a[k], b[k])
    multi.close()


def test_multi_device_errors(model_json, mmpc_mod):
    with pytest.raises(mmpc_mod.MmpcError):
        mmpc_mod.MultiSolver(model_json(), [])
    with pytest.raises(mmpc_mod.MmpcError):
        mmpc_mod.MultiSolver(model_json(), [0, -1])


def test_multi_device_lane_solver_exo_ragged_shards(tmp_path, mmpc_mod, oracle):
    """the lane (RICCATI) solver's iteration-tail hand-over makes an instance's bits depend on its 64-lane
    wave, so ragged shards (G = 3: shard boundaries off the 64-instance waves) agree with a single-device solve of the
    whole batch to 1e-10 relative in V* with identical iteration counts on >= 99 % -- the contract include/mmpc.h
    states -- while each shard equals a single-handle solve of that shard bit for bit; with the hand-over off
    (opts.tail_cap = 0) the multi-device result equals the whole-batch solve bit for bit."""
    B, N, G = 3000, 50, 3
    x0, up, tr = oracle.synth(20250213, 0, B, N, H, model=oracle.EXO)
    w = np.array([10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4)
    p = mmpc_mod.write_model_json(str(tmp_path / "exo_multi.json"), "exo", 8, 4, 2000, N, model="exo_arm")
    single = mmpc_mod.Solver(p, kkt_solver=2).solve_batch_host(x0, up, tr, w)
    multi = mmpc_mod.MultiSolver(p, [0] * G, kkt_solver=2)
    m = multi.solve_batch_host(x0, up, tr, w)
    assert (m["status"] == 0).all() and (single["status"] == 0).all()
    same = m["iters"] == single["iters"]
    assert same.mean() >= 0.99
    rel = np.abs(m["V"] - single["V"]).max(1) / np.abs(single["V"]).max(1)
    assert rel[same].max() <= 1e-10
    shard_solver = mmpc_mod.Solver(p, kkt_solver=2)
    for g in range(G):
        f, c = mmpc_mod.shard(B, G, g)
        r = shard_solver.solve_batch_host(x0[f:f + c], up[f:f + c], tr[f:f + c], w)
        np.testing.assert_array_equal(r["V"], m["V"][f:f + c])
        np.testing.assert_array_equal(r["iters"], m["iters"][f:f + c])
    multi.close()
    off_single = mmpc_mod.Solver(p, kkt_solver=2, tail_cap=0).solve_batch_host(x0, up, tr, w)
    off_multi = mmpc_mod.MultiSolver(p, [0] * G, kkt_solver=2, tail_cap=0)
    om = off_multi.solve_batch_host(x0, up, tr, w)
    for k in ("V", "status", "iters", "kkt"):
        np.testing.assert_array_equal(om[k], off_single[k])
    off_multi.close()
