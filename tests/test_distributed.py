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
