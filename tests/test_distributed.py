"""CPU, world_size 2 (gloo): the batch shards into independent instances -- each rank generates and solves
its own range from (seed, global index) -- so the union of the ranks' results equals the single-process
result bit for bit, and the only collectives are bench.py's reporting reductions (max time, sum)."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, WEIGHTS_CFG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "mahi-mpc_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import oracle_lib
    from mmpc import dist as mdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = mdist.shard(B, rank)
    x0, up, tr = oracle_lib.synth(20250213, first, n, 30, 0.002)
    r = oracle_lib.solve_batch(30, 0.002, x0, up, tr, np.array(WEIGHTS_CFG), nthreads=2)
    tmax = mdist.max_over_ranks(float(rank + 1))
    nconv = mdist.sum_over_ranks(int((r["status"] == 0).sum()))
    import torch
    Vs = [torch.zeros((n, r["V"].shape[1]), dtype=torch.float64) for _ in range(world)]
    dist.all_gather(Vs, torch.from_numpy(r["V"]))
    if rank == 0:
        q.put((np.concatenate([v.numpy() for v in Vs]), tmax, nconv))
    dist.destroy_process_group()


@pytest.mark.slow
def test_two_rank_shards_equal_single_process(oracle):
    import torch.multiprocessing as mp
    B, world = 48, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    V, tmax, nconv = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x0, up, tr = oracle.synth(20250213, 0, B * world, 30, 0.002)
    ref = oracle.solve_batch(30, 0.002, x0, up, tr, np.array(WEIGHTS_CFG))
    np.testing.assert_array_equal(V, ref["V"])
    assert tmax == 2.0 and nconv == B * world


def test_shard_arithmetic():
    import mmpc.dist as mdist
    assert mdist.shard(4096, 0) == (0, 4096) and mdist.shard(4096, 7) == (7 * 4096, 4096)
    for T, W in [(4096, 8), (10, 3), (7, 8), (0, 2)]:
        parts = [mdist.shard_strong(T, r, W) for r in range(W)]
        assert sum(n for _, n in parts) == T
        assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(W - 1))
    with pytest.raises(ValueError):
        mdist.shard(-1, 0)


class _OracleShardSolver:
    """test stand-in for mmpc.Solver on CPU tensors: solve_batch through the oracle (the C restatement), so
    the scatter / broadcast / gather plumbing of mmpc.dist.solve_rank0_batch runs on gloo without a GPU"""

    def __init__(self, N):
        self.nx, self.nu, self.N, self.NV = 4, 2, N, 6 * N + 4

    def solve_batch(self, B, x0, u_prev, traj, weights, V, status, iters, kkt, weights_stride=0, u_lb=None,
                    u_ub=None):
        import oracle_lib
        r = oracle_lib.solve_batch(self.N, 0.002, x0.numpy(), u_prev.numpy(), traj.numpy(),
                                   weights.numpy().reshape(B, -1) if weights_stride else weights.numpy(),
                                   V=V.numpy(), u_lb=None if u_lb is None else u_lb.numpy(),
                                   u_ub=None if u_ub is None else u_ub.numpy(), nthreads=1)
        V.copy_(__import__("torch").from_numpy(r["V"]))
        status.copy_(__import__("torch").from_numpy(r["status"]))
        iters.copy_(__import__("torch").from_numpy(r["iters"]))
        kkt.copy_(__import__("torch").from_numpy(r["kkt"]))


def _rank0_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "mahi-mpc_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    import oracle_lib
    from mmpc import dist as mdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, B = 30, 37
    solver = _OracleShardSolver(N)
    out = []
    for case in range(2):
        if rank == 0:
            x0, up, tr = (torch.from_numpy(a) for a in oracle_lib.synth(11, 0, B, N, 0.002))
            if case == 0:   # shared weights, bounds, cold start
                kw = dict(weights=torch.tensor(WEIGHTS_CFG, dtype=torch.float64),
                          u_lb=torch.tensor([-3.0, -2.0], dtype=torch.float64),
                          u_ub=torch.tensor([2.0, 3.0], dtype=torch.float64))
            else:           # per-instance weights, warm start
                w = np.tile(WEIGHTS_CFG, (B, 1)) * np.linspace(0.5, 2.0, B)[:, None]
                kw = dict(weights=torch.from_numpy(w), weights_stride=8,
                          V=torch.full((B, 6 * N + 4), 0.1, dtype=torch.float64))
            r = mdist.solve_rank0_batch(solver, x0, up, tr, **kw)
        else:
            r = mdist.solve_rank0_batch(solver)
        out.append(None if r is None else {k: v.numpy().copy() for k, v in r.items()})
    # gather_rows: ragged rank-major rows to rank 0 (the results leg of solve_rank0_batch)
    total = sum(r + 2 for r in range(world))
    lo, n = mdist.shard_strong(total, rank, world)
    mine = (torch.arange(total, dtype=torch.float64)[lo:lo + n, None] * 10)
    last = mdist.gather_rows(mine, total)
    if rank == 0:
        q.put((out, last.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 3])
def test_rank0_batch_scatter_solve_gather(world, oracle):
    """a rank-0 batch is scattered in contiguous shards (37 instances over 2 / 3 ranks, ragged),
    weights/bounds broadcast, results gathered -- equal to the single-process solve bit for bit"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank0_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out, last = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    N, B = 30, 37
    x0, up, tr = oracle.synth(11, 0, B, N, 0.002)
    ref0 = oracle.solve_batch(N, 0.002, x0, up, tr, np.array(WEIGHTS_CFG), u_lb=[-3.0, -2.0], u_ub=[2.0, 3.0])
    w = np.tile(WEIGHTS_CFG, (B, 1)) * np.linspace(0.5, 2.0, B)[:, None]
    ref1 = oracle.solve_batch(N, 0.002, x0, up, tr, w, V=np.full((B, 6 * N + 4), 0.1))
    for got, ref in ((out[0], ref0), (out[1], ref1)):
        np.testing.assert_array_equal(got["V"], ref["V"])
        np.testing.assert_array_equal(got["status"], ref["status"])
        np.testing.assert_array_equal(got["iters"], ref["iters"])
    # gather_rows: every rank's shard_strong rows, in global order, on rank 0
    total = sum(r + 2 for r in range(world))
    np.testing.assert_array_equal(last[:, 0], np.arange(total) * 10.0)
