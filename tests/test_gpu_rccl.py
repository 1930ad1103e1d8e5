"""GPU: the RCCL leg of the multi-GPU path, run on the one-GPU pool.

RCCL rejects two ranks on one GPU (profiles/r03/rccl/), but a ONE-rank "nccl" process group is legal, and with
``mmpc.dist.force_collectives`` the helpers issue their collectives even at world size 1.  So every RCCL call the
8-GPU run makes executes here on real RCCL over HIP device memory:
  * all_gather_into_tensor of the per-instance result table (bench.py's rank-0 gather),
  * broadcast of the shared weights / bounds (broadcast_shared),
  * scatter of the instances and gather of the results around a real device solve (solve_rank0_batch, the
    batched counterpart of the per-tick call ModelControl.cpp:159),
  * all_reduce MAX / SUM (bench.py's timing and convergence reductions),
and ``bench.py --rccl`` takes the N > 1 code path (table gathered through RCCL) at N = 1.
The test ids carry the RCCL version the process group ran on."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, WEIGHTS_CFG

pytestmark = pytest.mark.gpu


def _rccl_version():
    try:
        import torch
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return "unknown"


RCCL = _rccl_version()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def rccl_group():
    import torch
    import torch.distributed as dist
    from mmpc import dist as mdist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    prev = mdist.force_collectives(True)
    try:
        yield dist
    finally:
        mdist.force_collectives(prev)
        dist.destroy_process_group()


@pytest.mark.parametrize("rccl", [RCCL])
def test_rccl_collectives_one_rank(rccl, rccl_group):
    import torch
    from mmpc import dist as mdist
    dist = rccl_group
    info = mdist.rccl_info()
    assert info["backend"] == "nccl" and info["world_size"] == 1 and info["rccl_version"] == rccl
    dev = torch.device("cuda", 0)
    # the result-table gather of bench.py (uint8 rows of u_0* | status | iters)
    res = torch.arange(4096 * 24, dtype=torch.int64, device=dev).to(torch.uint8)
    table = torch.empty_like(res)
    dist.all_gather_into_tensor(table, res, async_op=True).wait()
    assert torch.equal(table, res)
    # broadcast of the shared weights and bounds
    w = torch.tensor(WEIGHTS_CFG, dtype=torch.float64, device=dev)
    lb = torch.tensor([-2.0, -3.0], dtype=torch.float64, device=dev)
    mdist.broadcast_shared(w, lb, None)
    assert w.tolist() == WEIGHTS_CFG and lb.tolist() == [-2.0, -3.0]
    # ragged rows through all_gather_into_tensor; scatter back
    rows = torch.arange(37 * 3, dtype=torch.float64, device=dev).view(37, 3)
    assert torch.equal(mdist.gather_rows(rows, 37), rows)
    assert torch.equal(mdist.scatter_rows(rows, 37, (3,), torch.float64, dev), rows)
    assert mdist.max_over_ranks(3.5, device=dev) == 3.5
    assert mdist.sum_over_ranks(7, device=dev) == 7
    torch.cuda.synchronize()


@pytest.mark.parametrize("rccl", [RCCL])
def test_rccl_rank0_scatter_solve_gather(rccl, rccl_group, model_json, mmpc_mod, oracle):
    """solve_rank0_batch on real RCCL and the HIP solver equals a direct device solve of the batch bit for bit
    (37 instances, per-instance weights, control bounds and a warm start)."""
    import torch
    from mmpc import dist as mdist
    dev = torch.device("cuda", 0)
    N, B = 30, 37
    x0, up, tr = oracle.synth(20250213, 0, B, N, 0.002)
    solver = mmpc_mod.Solver(model_json(N=N))
    NV = solver.NV
    f64 = dict(dtype=torch.float64, device=dev)
    w = np.tile(WEIGHTS_CFG, (B, 1)) * np.linspace(0.5, 2.0, B)[:, None]
    args = dict(x0=torch.tensor(x0, **f64), u_prev=torch.tensor(up, **f64), traj=torch.tensor(tr, **f64),
                weights=torch.tensor(w, **f64), weights_stride=8, V=torch.full((B, NV), 0.1, **f64),
                u_lb=torch.tensor([-20.0, -20.0], **f64), u_ub=torch.tensor([20.0, 20.0], **f64))
    r = mdist.solve_rank0_batch(solver, device=dev, **{k: (v.clone() if torch.is_tensor(v) else v)
                                                        for k, v in args.items()})
    V = args["V"].clone()
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    kk = torch.empty(B, **f64)
    solver.solve_batch(B, args["x0"], args["u_prev"], args["traj"], args["weights"], V, st, it, kk,
                       weights_stride=8, u_lb=args["u_lb"], u_ub=args["u_ub"])
    torch.cuda.synchronize()
    assert torch.equal(r["V"], V) and torch.equal(r["status"], st) and torch.equal(r["iters"], it)
    assert torch.equal(r["kkt"], kk) and bool((st == 0).all())
    solver.close()


@pytest.mark.parametrize("rccl", [RCCL])
def test_bench_rccl_flag(rccl):
    """bench.py --rccl: the default cfg#2 step at N = 1 with the last step's table gathered through RCCL."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--rccl", "--steps", "3", "--warmup", "2",
                        "--no-cpu-baseline", "--no-secondary", "--no-sweep"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["process_group"] == {"backend": "nccl", "world_size": 1, "rccl_version": rccl}
    assert out["gathered_results_match"] is True and out["converged"] == 4096
    assert out["zero_copy_results_checked"] is True


# ---- the C-ABI's own RCCL path: one process over the listed devices (mmpc_multi_solve_batch_rccl) ----

def _multi_model(mmpc_mod, tmp_path):
    return mmpc_mod.write_model_json(str(tmp_path / "m.json"), "two_link_arm", 4, 2, 2000, 30, model="two_link_arm")


@pytest.mark.parametrize("variant", ["shared", "bounded", "per_instance", "warm"])
def test_multi_rccl_equals_single_device(variant, mmpc_mod, oracle, tmp_path):
    """ncclCommInitAll over device 0, the shard sent to itself by ncclSend/ncclRecv, weights and bounds by
    ncclBroadcast, results gathered back: bit for bit the single-handle device solve of the same instances"""
    import torch
    path = _multi_model(mmpc_mod, tmp_path)
    B, N = 333, 30
    x0, up, tr = oracle.synth(5, 0, B, N, 0.002)
    w = np.array(WEIGHTS_CFG, dtype=np.float64)
    if variant == "per_instance":
        w = np.tile(w, (B, 1)) * (1.0 + 0.01 * np.arange(B))[:, None]
    d = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda:0")
    lb = ub = None
    if variant == "bounded":
        lb, ub = d(np.full(2, -2.0)), d(np.full(2, 2.0))
    V0 = np.zeros((B, 30 * 6 + 4))
    if variant == "warm":
        V0 = np.ascontiguousarray(mmpc_mod.Solver(path).solve_batch_host(x0, up, tr, w)["V"] * (1.0 + 1e-3))
    m = mmpc_mod.MultiSolver(path, [0])
    V = d(V0)
    st = torch.zeros(B, dtype=torch.int32, device="cuda:0")
    it = torch.zeros_like(st)
    kk = torch.zeros(B, dtype=torch.float64, device="cuda:0")
    m.solve_batch_rccl(d(x0), d(up), d(tr), d(w), V, st, it, kk, u_lb=lb, u_ub=ub)
    s = mmpc_mod.Solver(path)
    V1 = d(V0)
    st1, it1, kk1 = torch.zeros_like(st), torch.zeros_like(it), torch.zeros_like(kk)
    s.solve_batch(B, d(x0), d(up), d(tr), d(w), V1, st1, it1, kk1, weights_stride=8 if w.ndim == 2 else 0,
                  u_lb=lb, u_ub=ub)
    torch.cuda.synchronize()
    assert torch.equal(V, V1) and torch.equal(st, st1) and torch.equal(it, it1) and torch.equal(kk, kk1)
    assert (st == 0).all()
    m.close()


def test_multi_rccl_rejects_a_repeated_device(mmpc_mod, tmp_path):
    """RCCL refuses two ranks on one device: the RCCL entry point says so instead of hanging"""
    import torch
    m = mmpc_mod.MultiSolver(_multi_model(mmpc_mod, tmp_path), [0, 0])
    t = lambda *s: torch.zeros(*s, dtype=torch.float64, device="cuda:0")
    with pytest.raises(mmpc_mod.MmpcError):
        m.solve_batch_rccl(t(4, 4), t(4, 2), t(4, 30, 4), t(8), t(4, 184))
    m.close()


def _rccl_vs_single(mmpc_mod, oracle, tmp_path, B, weights_rows=None, stride=None):
    import torch
    path = _multi_model(mmpc_mod, tmp_path)
    N = 30
    x0, up, tr = oracle.synth(11, 0, max(B, 1), N, 0.002)
    x0, up, tr = x0[:B], up[:B], tr[:B]
    d = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda:0")
    w = d(np.array(WEIGHTS_CFG)) if weights_rows is None else d(weights_rows)
    m = mmpc_mod.MultiSolver(path, [0])
    V = torch.full((B, 30 * 6 + 4), 0.0, dtype=torch.float64, device="cuda:0")
    st = torch.full((B,), -7, dtype=torch.int32, device="cuda:0")
    it, kk = torch.zeros_like(st), torch.zeros(B, dtype=torch.float64, device="cuda:0")
    m.solve_batch_rccl(d(x0), d(up), d(tr), w, V, st, it, kk, weights_stride=stride)
    s = mmpc_mod.Solver(path)
    V1, st1 = torch.zeros_like(V), torch.full_like(st, -7)
    it1, kk1 = torch.zeros_like(it), torch.zeros_like(kk)
    if B:
        s.solve_batch(B, d(x0), d(up), d(tr), w, V1, st1, it1, kk1, weights_stride=stride or 0)
    torch.cuda.synchronize()
    m.close()
    return (V, st, it, kk), (V1, st1, it1, kk1)


@pytest.mark.parametrize("B", [0, 1])
def test_multi_rccl_tiny_batches(B, mmpc_mod, oracle, tmp_path):
    """B = 0 returns at once (nothing enqueued, outputs untouched); B = 1 is one shard of one instance: bit for bit the
    single-handle solve"""
    import torch
    a, b = _rccl_vs_single(mmpc_mod, oracle, tmp_path, B)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    if B:
        assert int(a[1][0]) == 0


def test_multi_rccl_strided_weights_not_over_read(mmpc_mod, oracle, tmp_path):
    """per-instance weights at weights_stride 11 > nx + 2 nu = 8 in a buffer of exactly (B - 1) 11 + 8 doubles: the
    scatter sends the last row only up to its 8 entries, and the solve equals the single-handle solve"""
    import torch
    B = 37
    rows = np.zeros((B - 1) * 11 + 8)
    for i in range(B):
        rows[i * 11:i * 11 + 8] = np.array(WEIGHTS_CFG) * (1.0 + 0.02 * i)
    a, b = _rccl_vs_single(mmpc_mod, oracle, tmp_path, B, weights_rows=rows, stride=11)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert (a[1] == 0).all()


def test_multi_rccl_rejects_a_short_weights_stride(mmpc_mod, tmp_path):
    """weights_stride in (0, nx + 2 nu) is refused before any RCCL operation is issued"""
    import torch
    m = mmpc_mod.MultiSolver(_multi_model(mmpc_mod, tmp_path), [0])
    t = lambda *s: torch.zeros(*s, dtype=torch.float64, device="cuda:0")
    with pytest.raises(mmpc_mod.MmpcError, match="weights_stride"):
        m.solve_batch_rccl(t(4, 4), t(4, 2), t(4, 30, 4), t(4 * 5), t(4, 184), weights_stride=5)
    m.close()


def test_multi_rccl_orders_after_the_callers_stream(mmpc_mod, oracle, tmp_path):
    """inputs produced on a side stream the call is given (no host synchronisation in between): the first RCCL send
    waits for that stream, so the solve sees the inputs; results equal the single-handle solve"""
    import torch
    path = _multi_model(mmpc_mod, tmp_path)
    B, N = 256, 30
    x0, up, tr = oracle.synth(13, 0, B, N, 0.002)
    side = torch.cuda.Stream(device="cuda:0")
    hx, hu, ht = (torch.tensor(a, dtype=torch.float64).pin_memory() for a in (x0, up, tr))
    with torch.cuda.stream(side):
        torch.cuda._sleep(20_000_000)   # the copies below land well after the call is made
        dx, du, dt = (h.to("cuda:0", non_blocking=True) for h in (hx, hu, ht))
        w = torch.tensor(WEIGHTS_CFG, dtype=torch.float64, device="cuda:0")
        V = torch.zeros((B, 30 * 6 + 4), dtype=torch.float64, device="cuda:0")
        st = torch.full((B,), -7, dtype=torch.int32, device="cuda:0")
    m = mmpc_mod.MultiSolver(path, [0])
    m.solve_batch_rccl(dx, du, dt, w, V, st, stream=side.cuda_stream)
    torch.cuda.synchronize()
    m.close()
    ref = mmpc_mod.Solver(path).solve_batch_host(x0, up, tr, np.array(WEIGHTS_CFG))
    assert np.array_equal(V.cpu().numpy(), ref["V"]) and (st.cpu().numpy() == 0).all()
