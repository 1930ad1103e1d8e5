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
