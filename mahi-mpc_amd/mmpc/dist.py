"""Batch sharding across ranks (one process per GPU, torch.distributed).

The path partitions into independent instances.  Synthetic batches (bench.py): rank r solves
the instances with global indices [r*B, (r+1)*B) generated on its GPU from (seed, global index), so results do
not depend on the number of ranks and inputs never cross xGMI; the per-instance results (u_0*, status,
iterations) are gathered to rank 0 (gather_rows).  Batches resident on rank 0 (a controller's calc_u, batched):
solve_rank0_batch broadcasts the shared weights/bounds, scatters the instances and gathers the results.
Process group: RCCL over xGMI on GPUs ("nccl"), gloo in the CPU tests."""
from __future__ import annotations


# Collectives even with one rank: the helpers below skip the collective at world size 1 (nothing to exchange).
# force_collectives(True) makes them issue it anyway, so the RCCL path (all_gather_into_tensor, broadcast, scatter)
# can be exercised on a one-GPU box (tests/test_gpu_rccl.py, bench.py --rccl).
_FORCE = False


def force_collectives(flag: bool = True) -> bool:
    """issue the collectives at world size 1 too; returns the previous setting"""
    global _FORCE
    prev, _FORCE = _FORCE, bool(flag)
    return prev


def _multi():
    """a process group whose collectives must run: world size > 1, or forced"""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or _FORCE)


def rccl_info():
    """backend and, on GPUs, the RCCL version the process group runs on (None without a process group)"""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None
    info = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    if info["backend"] == "nccl":
        try:
            v = torch.cuda.nccl.version()
            info["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception as e:   # pragma: no cover - reported, not fatal
            info["rccl_version"] = f"unknown ({e})"
    return info


def shard(batch_per_rank: int, rank: int) -> tuple[int, int]:
    """(first global instance index, count) of this rank (weak scaling: fixed work per rank)."""
    if batch_per_rank < 0 or rank < 0:
        raise ValueError("negative batch or rank")
    return rank * batch_per_rank, batch_per_rank


def shard_strong(total: int, rank: int, world: int) -> tuple[int, int]:
    """contiguous split of a fixed total: rank r gets [floor(r T / W), floor((r+1) T / W))."""
    lo = (rank * total) // world
    hi = ((rank + 1) * total) // world
    return lo, hi - lo


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not _multi():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    import torch
    import torch.distributed as dist
    if not _multi():
        return value
    t = torch.tensor([value], dtype=torch.float64 if isinstance(value, float) else torch.int64, device=device)
    dist.all_reduce(t)
    return t.item()


# ---------------- collectives of SURVEY.md 8(e) ----------------
# A controller that holds the whole batch on rank 0 (the reference's calc_u caller, batched) needs a real
# exchange: the shared weights/bounds are broadcast (< 1 KB), the instances scattered in contiguous shards
# (shard_strong), and every rank's results gathered back to rank 0.  On GPUs the process group is RCCL over
# xGMI ("nccl"); the CPU tests run the same code on gloo.

def _pg_ready():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def broadcast_shared(*tensors, src: int = 0):
    """Broadcast the shared (per-batch) solve parameters in place (weights [nx+2nu], u_lb/u_ub [nu]); None
    entries are skipped (every rank must pass the same pattern)."""
    import torch.distributed as dist
    if _multi():
        for t in tensors:
            if t is not None:
                dist.broadcast(t, src=src)
    return tensors


def gather_rows(local, total_rows: int, dst: int = 0):
    """Concatenate every rank's [n_r, ...] rows (shard_strong order) on rank ``dst`` (None elsewhere).

    One all_gather_into_tensor of equal-sized, padded chunks (RCCL over xGMI on GPUs, gloo on CPUs)."""
    import torch
    import torch.distributed as dist
    if not _multi():
        return local
    world, rank = dist.get_world_size(), dist.get_rank()
    chunk = -(-total_rows // world)
    lo, n = shard_strong(total_rows, rank, world)
    pad = torch.zeros((chunk,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:n] = local
    out = torch.empty((world * chunk,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad)
    parts = [out[r * chunk:(r + 1) * chunk] for r in range(world)]
    if rank != dst:
        return None
    return torch.cat([parts[r][:shard_strong(total_rows, r, world)[1]] for r in range(world)])


def scatter_rows(full, total_rows: int, row_shape, dtype, device, src: int = 0):
    """Rank ``src`` holds ``full`` [total_rows, *row_shape]; every rank receives its shard_strong rows."""
    import torch
    import torch.distributed as dist
    if not _multi():
        return full
    world, rank = dist.get_world_size(), dist.get_rank()
    chunk = -(-total_rows // world)
    recv = torch.empty((chunk,) + tuple(row_shape), dtype=dtype, device=device)
    parts = None
    if rank == src:
        parts = []
        for r in range(world):
            lo, n = shard_strong(total_rows, r, world)
            p = torch.zeros((chunk,) + tuple(row_shape), dtype=dtype, device=device)
            p[:n] = full[lo:lo + n]
            parts.append(p)
    dist.scatter(recv, parts, src=src)
    return recv[:shard_strong(total_rows, rank, world)[1]]


def solve_rank0_batch(solver, x0=None, u_prev=None, traj=None, weights=None, V=None, u_lb=None, u_ub=None,
                      device=None, weights_stride: int = 0):
    """Strong-scaled solve of a batch resident on rank 0: broadcast the shared weights and
    bounds, scatter the instances (and the warm start V) in contiguous shards, solve each shard on its GPU
    with ``solver.solve_batch`` (device pointers, stream-ordered), gather V / status / iters / kkt to rank 0.

    Rank 0 passes the full batch as tensors on ``device``; the other ranks pass only ``solver`` and ``device``.
    Per-instance weights (weights_stride > 0) are scattered like the instances.  Returns dict(V, status,
    iters, kkt) on rank 0 and None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size() if _pg_ready() else 1
    rank = dist.get_rank() if _pg_ready() else 0
    nx, nu, N, NV = solver.nx, solver.nu, solver.N, solver.NV
    meta = torch.zeros(5, dtype=torch.int64, device=device)
    if rank == 0:
        meta[0] = x0.shape[0]
        meta[1] = int(V is not None)
        meta[2] = int(u_lb is not None)
        meta[3] = int(u_ub is not None)
        meta[4] = int(weights_stride)
    if _multi():
        dist.broadcast(meta, src=0)
    B, has_V, has_lb, has_ub, ws = (int(v) for v in meta.tolist())
    f64 = dict(dtype=torch.float64, device=device)
    if rank != 0:
        weights = None if ws else torch.empty(nx + 2 * nu, **f64)
        u_lb = torch.empty(nu, **f64) if has_lb else None
        u_ub = torch.empty(nu, **f64) if has_ub else None
    broadcast_shared(None if ws else weights, u_lb, u_ub)
    w_loc = scatter_rows(weights, B, (ws,), torch.float64, device) if ws else weights
    x_loc = scatter_rows(x0, B, (nx,), torch.float64, device)
    u_loc = scatter_rows(u_prev, B, (nu,), torch.float64, device)
    t_loc = scatter_rows(traj, B, (N, nx), torch.float64, device)
    n = x_loc.shape[0]
    V_loc = scatter_rows(V, B, (NV,), torch.float64, device) if has_V else torch.zeros((n, NV), **f64)
    V_loc = V_loc.contiguous()
    st = torch.empty(n, dtype=torch.int32, device=device)
    it = torch.empty(n, dtype=torch.int32, device=device)
    kk = torch.empty(n, **f64)
    if n:
        solver.solve_batch(n, x_loc.contiguous(), u_loc.contiguous(), t_loc.contiguous(), w_loc.contiguous(),
                           V_loc, st, it, kk, weights_stride=ws, u_lb=u_lb, u_ub=u_ub)
    res = torch.cat([V_loc, st.double()[:, None], it.double()[:, None], kk[:, None]], 1)
    full = gather_rows(res, B)
    if full is None:
        return None
    return dict(V=full[:, :NV], status=full[:, NV].to(torch.int32), iters=full[:, NV + 1].to(torch.int32),
                kkt=full[:, NV + 2])
