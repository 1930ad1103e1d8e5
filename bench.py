#!/usr/bin/env python3
"""Benchmark of the MI355X batched NMPC solve path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg5] [--batch B] [--horizon N]

One "step" = one cold-started batched SQP solve of B independent instances per GPU (cfg#2: 2-link arm, nx=4,
nu=2, N=30, h=2 ms, fp64), i.e. what the reference does per control tick in ModelControl::calc_u
(src/Mahi/Mpc/ModelControl.cpp:116-172) -- from V = 0 with x_0 pinned, the reference's first-call state -- for
B instances at once, FROM INPUT STAGING THROUGH RESULTS ON HOST: every step first generates its B
instances on the device (mmpc_synth_batch from (seed, global instance index), the per-tick packing of
ModelControl.cpp:118-157) and ends with the per-instance results the
reference consumes (u_0*, status, iterations; ModelControl.cpp:160-190) in pinned host memory -- stored there
by the solve kernel itself (mmpc_solve_batch_u0 into mmpc_host_alloc memory, each rank into its own process's
host memory); with N > 1 the last step's results of all ranks are also gathered to rank 0 (RCCL
all_gather_into_tensor, then D2H) and checked there.  Step k of the timed region solves the instance block
max(K - 2 - k, 0) (global instances block * B_total + [r B, (r+1) B) on rank r, weak scaling): the steps solve
distinct instances, and the last two the block 0 that the CPU baseline and the N > 1 zero-copy check compare
against; results do not depend on the GPU count.  `value_solve_only` beside `value` is a second timed loop of the
same K solves on resident inputs (no generation): its HIP-event bracket is also the kernel time of the roofline.

Multi-GPU: ``--gpus N`` with N > 1 and no WORLD_SIZE in the environment makes this process a launcher that
starts N rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each) before anything touches
the GPU, forwards rank 0's JSON line and exits with the worst rank exit code.  Under torchrun (WORLD_SIZE set)
the process is a rank itself.

Prints ONE JSON line on rank 0 (driver contract) with two extra objects:
  roofline      the dominant kernel's achieved FP64 rate (its own algorithmic flop count) vs the MI355X FP64
                vector peak; kernel time from HIP events on the launch stream;
  cpu_baseline  the oracle/ CPU restatement (same NLP and SQP, fp64) on a bounded sample, rank 0 at N = 1 only,
                with its agreement with the GPU solutions and both iteration histograms.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mahi-mpc_amd"))

METRIC = "MPC solves/sec (whole node), nx=4 N=30 batch, at 1/2/4/8 MI355X"
SEED = 20250213
WEIGHTS = [10.0, 1.0, 5.0, 5.0, 5.0, 5.0, 0.01, 0.01]
# SURVEY.md 8d cfg#3 (exo): Q = [10 x4, 1 x4], R = 1 x4, Rm = 0.01 x4
WEIGHTS_EXO = [10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4
_EXO_METRIC = "MPC solves/sec (whole node), exo nx=8 N=50 batch (SURVEY.md 8d cfg#3/#4)"
CONFIGS = {
    "cfg2": dict(model="two_link_arm", nx=4, nu=2, N=30, B=4096, weights=WEIGHTS, metric=METRIC, fp32=False,
                 workload="cfg#2: 2-link arm nx=4 nu=2, N=30, h=2 ms, cold-start SQP (exact or Gauss-Newton Hessian: config.hessian) to "
                          "||grad||<=1e-8, ||g||<=1e-10"),
    "cfg3": dict(model="exo_arm", nx=8, nu=4, N=50, B=65536, weights=WEIGHTS_EXO, metric=_EXO_METRIC, fp32=False,
                 workload="cfg#3: 4-DoF exo nx=8 nu=4 (build-defined parameters), N=50, h=2 ms, cold-start GN-SQP "
                          "(Riccati KKT, lane per instance; instances unconverged after iteration 4 continue in a "
                          "16-lane resume launch, same iterates) to ||grad||<=1e-8, ||g||<=1e-10"),
    "cfg5": dict(model="exo_arm", nx=8, nu=4, N=50, B=65536, weights=WEIGHTS_EXO, fp32=True,
                 metric="MPC solves/sec (whole node), exo nx=8 N=50 batch, fp32 KKT factor + fp64 residuals "
                        "(SURVEY.md 8d cfg#5)",
                 workload="cfg#5: cfg#3 with the Riccati matrix recursion in fp32 and every right-hand side, "
                          "residual, model evaluation and merit in fp64 (each SQP iteration = one refinement "
                          "step; the iteration tail continues with the fp64 factor in the 16-lane resume launch), "
                          "to ||grad||<=1e-8, ||g||<=1e-10"),
}
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector peak (AMD spec); FP64 matrix peak is the same
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md chip table)
HBM_PEAK_TBS = 8.0        # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg2",
                    help="cfg2 = headline (BASELINE.json); cfg3 / cfg5 = exo workloads of SURVEY.md 8d")
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU (cfg#2: 4096, cfg#3/#5: 65536)")
    ap.add_argument("--kkt", choices=["auto", "condensed", "riccati", "group"], default="auto",
                    help="KKT solver (mmpc_opts.kkt_solver); auto = the library's choice")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--tol", type=float, default=None,
                    help="outer tolerance: tol_grad = tol, tol_defect = tol/100 (default: 1e-8 / 1e-10)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0,
                    help="target wall time of each CPU-baseline leg (Riccati, dense condensed)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="cfg2 only: skip the cfg#3 / cfg#5 lines the default invocation attaches as 'secondary'")
    ap.add_argument("--no-sweep", action="store_true", help="skip the tolerance sweeps (cfg5's, and cfg2's / cfg3's at the reference's IPOPT tol 1e-5 / "
                                                            "SURVEY A9's 1e-6)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --batch (default: the config's B) is the GLOBAL batch, split over the ranks "
                         "in contiguous shards (mmpc.dist.shard_strong); default: weak scaling, B per GPU")
    ap.add_argument("--x-bound", type=float, default=None,
                    help="state bounds |qdot_i| <= X on the velocity half of x (x_min/x_max, ModelControl.cpp:37-50): "
                         "the primal-dual interior-point variant (DESIGN.md 3c)")
    ap.add_argument("--u-bound", type=float, default=None,
                    help="control bounds |u| <= U on every instance (update_control_limits, ModelControl.cpp:205-209): "
                         "the projected GN-SQP (DESIGN.md 3b)")
    ap.add_argument("--init", choices=["zero", "as_given", "hold_x0"], default="zero",
                    help="mmpc_opts.init_states: the reference's cold start V = 0 (zero: MMPC_INIT_ZERO, V not read; "
                         "as_given: V zeroed every step), or x_1..x_N = x_0 (DESIGN 3d)")
    ap.add_argument("--hessian", choices=["auto", "gauss_newton", "exact"], default="auto",
                    help="mmpc_opts.hessian: AUTO = exact Lagrangian Hessian where supported (DESIGN.md 3e)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per launch per config (tools/pmc.sh + tools/pmc_summary.py)")
    ap.add_argument("--rccl", action="store_true",
                    help="N = 1 too: initialise the RCCL process group (\"nccl\") and gather the last step's result "
                         "table through all_gather_into_tensor as the N > 1 path does, so the RCCL leg runs on a "
                         "one-GPU box (the line then reports the RCCL version)")
    ap.add_argument("--standin", action="store_true",
                    help="TEST ONLY: CPU tensors, gloo and a trivial stand-in solver, to exercise the launcher / "
                         "rank / gather plumbing without a GPU (tests/test_bench_launch.py); never a measurement")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher (N > 1, no torchrun)
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv) -> int:
    """Start one rank process per GPU and wait for all of them.  Nothing here initialises the GPU (no torch,
    no mmpc import): each child is a fresh interpreter that sees every device and picks LOCAL_RANK."""
    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):   # one rank failed: the others would hang in a collective
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.kill()
                    rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc]
    return (bad[0] if bad[0] > 0 else 1) if bad else 0


# ------------------------------------------------------------------ CPU baseline (rank 0, N = 1 only)
def _cpu_leg(o, cfg, N, h, target_s, kw, kkt):
    """one timed oracle leg on a bounded sample: a small calibration solve sizes the sample to ~target_s"""
    model = kw["model"]
    w = np.array(cfg["weights"])
    n0 = 2 * kw["nthreads"]
    x0, up, tr = o.synth(SEED, 0, n0, N, h, model=model)
    t = time.perf_counter()
    o.solve_batch(N, h, x0, up, tr, w, kkt=kkt, **kw)
    dt = time.perf_counter() - t
    n = int(max(n0, min(200000, n0 * target_s / max(dt, 1e-6))))
    x0, up, tr = o.synth(SEED, 0, n, N, h, model=model)
    t = time.perf_counter()
    r = o.solve_batch(N, h, x0, up, tr, w, kkt=kkt, **kw)
    return n, time.perf_counter() - t, r


def cpu_baseline(cfg, N, h, target_s, gpu_V, gpu_iters, tol_grad, tol_defect, hessian=1, u_bound=None,
                 x_bound=None, kkt_solver=0):
    """The oracle (oracle/liboracle.so: the same NLP and SQP in plain C + OpenMP, cold start V = 0) timed on a
    bounded sample of the same seeded workload, in two legs:
      riccati          the Riccati recursion the GPU kernels run (ORACLE_KKT_RICCATI: same algorithm, same iterates)
                       -- the reported value;
      dense_condensed  explicit condensing + dense Cholesky of the N*nu Hessian (the oracle's default checker).
    Each leg's agreement with the GPU on the shared instances is reported beside it."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as o
    model = o.EXO if cfg["model"] == "exo_arm" else o.TWO_LINK
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    # the same SQP as the GPU: the Hessian the library resolved (mmpc_resolve_hessian: 1 Gauss-Newton, 2 exact)
    kw = dict(nthreads=threads, model=model, tol_grad=tol_grad, tol_defect=tol_defect, init_states=2,
              hessian=o.HESS_EXACT if hessian == 2 else o.HESS_GAUSS_NEWTON)
    nu = cfg["nu"]
    if u_bound is not None:   # the oracle's projected GN-SQP (its Riccati restatement covers unbounded solves only)
        # with the active-set rule of the kernel that ran (the 16-lane kernel also releases holds)
        kw.update(u_lb=np.full(nu, -u_bound), u_ub=np.full(nu, u_bound), bound_release=kkt_solver == 3)
    if x_bound is not None:   # the oracle's interior-point variant (solve_one_ip, dense)
        half = cfg["nx"] // 2
        kw.update(x_lb=np.array([-np.inf] * half + [-x_bound] * half), x_ub=np.array([np.inf] * half + [x_bound] * half))
    hist = lambda a: {int(k): int(v) for k, v in zip(*np.unique(a, return_counts=True))}  # noqa: E731
    legs = {}
    legs_spec = [("riccati", o.KKT_RICCATI, "Riccati recursion on [dx_k; du_{k-1}] (the GPU's algorithm)"),
                 ("dense_condensed", o.KKT_DENSE, "DENSE condensed KKT (Cholesky of the N*nu Hessian)")]
    if u_bound is not None or x_bound is not None:   # bounded: the oracle's bounded solves are dense only
        legs_spec = legs_spec[1:]
    for name, kkt, what in legs_spec:
        n, dt, r = _cpu_leg(o, cfg, N, h, target_s, kw, kkt)
        m = min(n, gpu_V.shape[0])
        ref = r["V"][:m]
        scale = np.maximum(np.abs(ref).max(axis=1), 1e-300)
        rel = np.abs(gpu_V[:m] - ref).max(axis=1) / scale
        same_it = r["iters"][:m] == gpu_iters[:m]
        legs[name] = dict(
            value=n / dt, unit="solves/s", cores=threads,
            sample=f"first {n} {cfg['workload'].split(':')[0]} instances (seed {SEED}), cold start, {dt:.1f} s wall, "
                   f"{int((r['status'] == 0).sum())}/{n} converged; oracle SQP with a {what}, "
                   f"{'exact' if hessian == 2 else 'Gauss-Newton'} Hessian as the GPU, {threads} OpenMP threads",
            vs_gpu=dict(instances=int(m), max_rel_diff_V=float(rel.max()),
                        max_rel_diff_V_same_iters=float(rel[same_it].max()) if same_it.any() else None,
                        same_iteration_count=int(same_it.sum())),
            iters_hist_cpu=hist(r["iters"]))
    ric = legs.get("riccati") or legs["dense_condensed"]
    return dict(value=ric["value"], unit="solves/s", cores=threads, kind="port",
                sample=ric["sample"] + (" (the dense-condensed leg is reported beside it)" if "riccati" in legs else ""),
                vs_gpu=ric["vs_gpu"], iters_hist_cpu=ric["iters_hist_cpu"], iters_hist_gpu=hist(gpu_iters), **legs)


def lib_sha256(path: str) -> str:
    """sha256 of the solver library a run loaded: the key that ties a PMC summary to the build it measured"""
    import hashlib
    hsh = hashlib.sha256()
    with open(path, "rb") as fh:
        for chunk in iter(lambda: fh.read(1 << 20), b""):
            hsh.update(chunk)
    return hsh.hexdigest()


# ------------------------------------------------------------------ test stand-in (no GPU)
class _StandInSolver:
    """--standin only: a CPU 'solver' with the mmpc.Solver call shape whose outputs are a fixed function of the
    synthetic inputs (u_0* := x0[:, :nu], status 0, iters 1), so the launcher / rank / gather plumbing can be
    tested on gloo.  It is not the solve path and never produces a reported number."""

    def __init__(self, nx, nu, N):
        self.nx, self.nu, self.N, self.NV = nx, nu, N, nx * (N + 1) + nu * N

    def synth(self, seed, first, B, x0, up, tr, stream=None):
        import torch
        idx = torch.arange(first, first + B, dtype=torch.float64)[:, None]
        x0.copy_(idx + torch.arange(self.nx, dtype=torch.float64) / 10)
        up.zero_()
        tr.zero_()

    def solve_batch(self, B, x0, up, tr, w, V, st, it, kkt, stream=None, u_lb=None, u_ub=None):
        V.zero_()
        V[:, self.nx:self.nx + self.nu] = x0[:, :self.nu]
        st.zero_()
        it.fill_(1)
        if kkt is not None:
            kkt.zero_()


# ------------------------------------------------------------------ one rank
def run_rank(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    pg = world > 1 or args.rccl
    if pg:
        # MMPC_BENCH_BACKEND / MMPC_BENCH_SAME_DEVICE: test hooks that rehearse the N > 1 GPU path on a one-GPU box
        # (gloo ranks sharing device 0; RCCL rejects two ranks on one GPU) -- never set for measurements
        if world == 1:   # --rccl at N = 1: a one-rank group (legal on one GPU), not launched by torchrun
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.rccl:
            import mmpc.dist as mdist
            mdist.force_collectives(True)
        if not args.standin:   # RCCL binds the communicator to the current device
            import torch
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) if not os.environ.get("MMPC_BENCH_SAME_DEVICE") else 0)
        dist.init_process_group(os.environ.get("MMPC_BENCH_BACKEND") or ("gloo" if args.standin else "nccl"))
    out = run_config(args, args.config, world, rank, primary=True)
    if pg:
        import mmpc.dist as mdist
        out["process_group"] = mdist.rccl_info()
    # the default (headline) invocation also measures the exo workloads of SURVEY.md 8d inside the same run, so the
    # driver's clock covers them: cfg#3 (at N > 1 ranks: cfg#4, weak-scaled 65536 instances per GPU) and cfg#5
    if args.config == "cfg2" and not args.no_secondary and not args.standin and args.batch is None \
            and args.horizon is None:
        out["secondary"] = {c: run_config(args, c, world, rank, primary=False) for c in ("cfg3", "cfg5")}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg:
        dist.destroy_process_group()


def run_config(args, name, world, rank, primary=True):
    """W warm-up + K timed steps of config `name` on this rank; returns the JSON object of the line (rank 0)."""
    import torch
    import torch.distributed as dist
    import mmpc.dist as mdist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    standin = args.standin
    cfg = CONFIGS[name]
    B = (args.batch if primary else None) or cfg["B"]
    N = (args.horizon if primary else None) or cfg["N"]
    # rows of this rank: weak scaling -- B per rank, global instances [r B, (r+1) B); strong -- the global batch B split
    # in contiguous shards; Bc = result-table rows per rank (equal for the gather; strong shards may be ragged)
    strong = args.strong and primary
    coll = world > 1 or args.rccl   # the last step's result table goes through the collective gather
    if strong and B < world:
        raise SystemExit(f"--strong needs --batch >= the rank count ({B} < {world}): a rank would get no instances")
    Bt = B if strong else B * world
    Bc = -(-B // world) if strong else B
    first, n = mdist.shard_strong(B, rank, world) if strong else mdist.shard(B, rank)
    nrows = [mdist.shard_strong(B, r, world)[1] for r in range(world)] if strong else [B] * world
    nx, nu, h_us = cfg["nx"], cfg["nu"], 2000
    h = h_us * 1e-6
    tol_grad = 1e-8 if args.tol is None else args.tol
    tol_defect = 1e-10 if args.tol is None else args.tol / 100

    if standin:
        dev = torch.device("cpu")
        solver = _StandInSolver(nx, nu, N)
        ksolver = 0
        hess = 1
        stream = None
    else:
        import mmpc
        if os.environ.get("MMPC_BENCH_SAME_DEVICE"):
            local = 0
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        tmpdir = tempfile.mkdtemp(prefix="mmpc_bench_")
        path = mmpc.write_model_json(os.path.join(tmpdir, f"{cfg['model']}.json"), cfg["model"], nx, nu, h_us, N,
                                     model=cfg["model"])
        ksolver = {"auto": 0, "condensed": 1, "riccati": 2, "group": 3}[args.kkt if primary else "auto"]
        solver = mmpc.Solver(path, device=local, kkt_solver=ksolver, factor_fp32=cfg["fp32"],
                             tol_grad=tol_grad, tol_defect=tol_defect,
                             init_states={"zero": mmpc.INIT_ZERO, "as_given": mmpc.INIT_AS_GIVEN,
                                          "hold_x0": mmpc.INIT_HOLD_X0}[args.init],
                             hessian={"auto": mmpc.HESSIAN_AUTO, "gauss_newton": mmpc.HESSIAN_GAUSS_NEWTON,
                                      "exact": mmpc.HESSIAN_EXACT}[args.hessian if primary else "auto"])
        if args.x_bound is not None and primary:
            half = nx // 2
            solver.set_state_bounds([-np.inf] * half + [-args.x_bound] * half, [np.inf] * half + [args.x_bound] * half)
        solver.reserve_workspace(n)
        ksolver = solver.kkt_solver_for(n)   # the AUTO choice, resolved by the library
        hess = solver.hessian_for(n, bool(args.u_bound is not None and primary))
        stream = torch.cuda.current_stream(dev)
    NV = solver.NV
    f64 = dict(dtype=torch.float64, device=dev)
    x0 = torch.empty((n, nx), **f64)
    up = torch.empty((n, nu), **f64)
    tr = torch.empty((n, N, nx), **f64)
    w = torch.tensor(cfg["weights"], **f64)
    ulb = uub = None
    if args.u_bound is not None and primary:
        ulb = torch.full((nu,), -args.u_bound, **f64)
        uub = torch.full((nu,), args.u_bound, **f64)
    V = torch.zeros((n, NV), **f64)
    # results the reference consumes per tick: u_0* (ModelControl.cpp:174-190), status, iterations -- one byte
    # buffer per rank, [B][nu] f64 u_0* | [B] i32 status | [B] i32 iterations.
    # Every step: the solve kernel stores them straight into pinned host memory of the rank's own process
    #   (mmpc_solve_batch_u0 into an mmpc_host_alloc buffer, two buffers alternating): no copy kernel, no D2H --
    #   each GPU process serves its own controllers (weak scaling).
    # N > 1, last step (and last warm-up step): the rank-0 table instead -- the solve writes status and iterations
    #   into a device buffer, u_0* is one strided copy out of V, one all_gather_into_tensor (RCCL over xGMI) to
    #   rank 0's device, then one D2H there; rank 0 checks it against every rank's own results.
    nbytes = Bc * (8 * nu + 8)
    zero_copy = not standin
    hbuf = None
    if zero_copy:
        hbuf = [mmpc.HostBuffer(nbytes) for _ in range(2)]
        hviews = [(hb.view(0, np.float64, Bc * nu), hb.view(Bc * nu * 8, np.int32, Bc),
                   hb.view(Bc * nu * 8 + 4 * Bc, np.int32, Bc)) for hb in hbuf]
    res = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    res.zero_()
    u0 = res[:Bc * nu * 8].view(torch.float64).view(Bc, nu)
    st = res[Bc * nu * 8:Bc * nu * 8 + 4 * Bc].view(torch.int32)
    it = res[Bc * nu * 8 + 4 * Bc:].view(torch.int32)
    sh = stream.cuda_stream if stream is not None else None
    solver.synth(SEED, first, n, x0, up, tr, stream=sh)
    mdist.broadcast_shared(w)   # shared weights from rank 0 (identical here by construction)

    table = torch.empty(world * nbytes, dtype=torch.uint8, device=dev) if coll else res
    pin = dict(pin_memory=True) if not standin else {}
    host = [torch.empty(world * nbytes, dtype=torch.uint8, **pin) for _ in range(2)]
    # MMPC_INIT_ZERO: the cold start V = 0 without reading V (no per-step memset); as_given zeroes V each step
    zero_v = args.init == "as_given" or standin

    def zc(k, last):   # this step's results straight into host memory?
        return zero_copy and (not coll or k != last)

    def results_to_host(k, last):
        if zc(k, last):
            return   # stored into host memory by the solve kernel
        u0[:n].copy_(V[:, nx:nx + nu])
        if coll:   # N > 1 (or --rccl): one all_gather_into_tensor (RCCL over xGMI) to rank 0's device, then D2H there
            dist.all_gather_into_tensor(table, res, async_op=True).wait()   # stream-ordered on GPUs
        if rank == 0:
            host[k % 2].copy_(table, non_blocking=not standin)

    def launch(k, last):
        if zc(k, last):
            u0h, sth, ith = hviews[k % 2]
            solver.solve_batch(n, x0, up, tr, w, V, sth, ith, None, stream=sh, u0=u0h, u_lb=ulb, u_ub=uub)
        else:
            solver.solve_batch(n, x0, up, tr, w, V, st, it, None, stream=sh, u_lb=ulb, u_ub=uub)

    def block(k):   # instance block of timed step k; warm-up step j generates block K + j (never timed)
        return max(args.steps - 2 - k, 0)

    def solve(k, last, blk=None):
        if blk is not None:   # this step's instances, generated on the device inside the clock
            solver.synth(SEED, blk * Bt + first, n, x0, up, tr, stream=sh)
        if zero_v:
            V.zero_()   # cold start (reference first call: v_init = 0, ModelControl.cpp:29-50)
        launch(k, last)

    for k in range(args.warmup):   # the last warm-up step also initialises the RCCL gather (N > 1)
        solve(k, args.warmup - 1, args.steps + k)
        results_to_host(k, args.warmup - 1)
    sync = (lambda: torch.cuda.synchronize(dev)) if not standin else (lambda: None)
    sync()
    # The kernel's own duration (roofline): one pair of HIP events on the launch stream around the K back-to-back
    # launches of the timed region, / K.  No markers between launches: an event record between two launches adds a
    # queue gap of ~6-10 us per step, while back-to-back launches run with none (rocprofv3 kernel trace,
    # profiles/r03/gaps/), so the bracket / K is the average launch duration (with --init as_given it also holds the
    # per-step memset of V, a few microseconds).
    ev = ((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if not standin else None)
    if coll:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if ev:
        ev[0].record(stream)
    for k in range(args.steps):
        solve(k, args.steps - 1, block(k))
        if ev and k == args.steps - 1:
            ev[1].record(stream)   # after the last launch (N > 1: before its result gather)
        results_to_host(k, args.steps - 1)
    sync()
    if coll:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = ev[0].elapsed_time(ev[1]) / args.steps if ev else 0.0   # generation + solve, per step
    elapsed = mdist.max_over_ranks(elapsed, device=dev)
    # the same K solves again on the resident inputs of the last step (block 0), without the generation: the
    # solve-only rate beside the line's value, and the solve kernel's own mean duration for the roofline
    if coll:
        dist.barrier()
    sync()
    t1 = time.perf_counter()
    if ev:
        ev[0].record(stream)
    for k in range(args.steps):
        solve(k, args.steps - 1)
        if ev and k == args.steps - 1:
            ev[1].record(stream)
        results_to_host(k, args.steps - 1)
    sync()
    if coll:
        dist.barrier()
    elapsed_solve = mdist.max_over_ranks(time.perf_counter() - t1, device=dev)
    kern_ms = ev[0].elapsed_time(ev[1]) / args.steps if ev else 0.0

    def hbytes(k):
        return torch.from_numpy(np.frombuffer(hbuf[k % 2]._buf, dtype=np.uint8).copy())

    # zero-copy results check: None = unchecked (N > 1 needs two timed steps: the previous step's host buffer holds
    # the same instances as the gathered last step)
    zc_ok = None
    if zero_copy and not coll:   # the host buffer of the last step IS the result table; check it against V
        hb = hviews[(args.steps - 1) % 2]
        res.copy_(hbytes(args.steps - 1))
        host[(args.steps - 1) % 2].copy_(res.cpu())
        zc_ok = bool(np.array_equal(hb[0][:n * nu].reshape(n, nu), V[:, nx:nx + nu].cpu().numpy()))
    elif zero_copy and args.steps >= 2:   # N > 1: the previous step (same instances) stored into host memory
        zc_ok = bool(torch.equal(hbytes(args.steps - 2), res.cpu()))
    iters = it.cpu().numpy()[:n]
    # rank 0's host table of the last step against every rank's own results
    mine = res.cpu()
    ok = zc_ok is not False
    if rank == 0:
        last = host[(args.steps - 1) % 2]
        ok = bool(torch.equal(last[:nbytes], mine)) and ok
        conv = sum(int((last[r * nbytes + Bc * nu * 8:r * nbytes + Bc * nu * 8 + 4 * Bc].view(torch.int32)[:nrows[r]]
                        == 0).sum()) for r in range(world))
        tail = last
    else:
        conv = 0
        tail = None
    if coll:
        ok = bool(torch.equal(table[rank * nbytes:(rank + 1) * nbytes].cpu(), mine)) and ok
        ok = mdist.sum_over_ranks(int(not ok), device=dev if not standin else None) == 0
    total = Bt * args.steps
    value = total / elapsed
    out = {
        "metric": cfg["metric"],
        "value": value,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "value_solve_only": total / elapsed_solve,
        "ms_per_step_solve_only": elapsed_solve / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64" if not cfg["fp32"] else "f64 (fp32 Riccati factor)",
        "data": f"synthetic: counter-based splitmix64 {name} instances (SURVEY.md 8d), generated on device "
                f"from (seed, global instance index), so N = 1 and N > 1 solve identical instances",
        "config": {"workload": cfg["workload"] + (f"; control bounds |u| <= {args.u_bound} (projected SQP)"
                                                  if ulb is not None else "")
                   + (f"; state bounds |qdot| <= {args.x_bound} (interior point)"
                      if args.x_bound is not None and primary else ""),
                   "batch_per_gpu": n, "global_batch": Bt,
                   "horizon": N, "tol_grad": tol_grad, "tol_defect": tol_defect,
                   "kkt_solver": {0: "stand-in (test)", 1: "condensed (wave per instance)",
                                  2: "riccati (lane per instance)", 3: "riccati (16 lanes per instance)"}[ksolver],
                   "hessian": {1: "gauss-newton", 2: "exact (Lagrangian, IPOPT's default)"}[hess],
                   "init_states": {"zero": "reference cold start V = 0 (MMPC_INIT_ZERO: V not read)",
                                   "as_given": "reference cold start V = 0 (V zeroed every step)",
                                   "hold_x0": "x_1..x_N = x_0 (MMPC_INIT_HOLD_X0)"}[args.init],
                   "parallelism": (f"batch-shard x{world}; per-step results (u_0*, status, iters) stored by the "
                                   "solve kernel into each rank's pinned host memory (mmpc_host_alloc); the last "
                                   "step's table gathered to rank 0 by RCCL all_gather_into_tensor + D2H"
                                   if coll else "batch-shard x1; per-step results (u_0*, status, iters) stored "
                                                     "by the solve kernel into pinned host memory (mmpc_host_alloc)"),
                   "timed_region": ("per step: on-device generation of the step's instances (mmpc_synth_batch, "
                                    "the per-tick input packing) + cold-start solve + results (u_0*, status, iters) "
                                    "on the host"
                                    + ("; the last step's table of all ranks on rank 0's host" if coll else "")
                                    + "; value_solve_only: the same K solves on resident inputs")},
        "converged": conv,
        "gathered_results_match": ok,
        "zero_copy_results_checked": zc_ok is not None,
        "mean_sqp_iters": float(iters.mean()),
        "max_sqp_iters": int(iters.max()),
    }
    if name == "cfg3" and world > 1:
        out["config"]["workload"] = "cfg#4 (SURVEY.md 8d): " + cfg["workload"] + f", weak-scaled over {world} GPUs"
    if standin:
        out["standin"] = True
        if tail is not None:   # u_0*[:, 0] of every rank's slice of the gathered table
            out["standin_u0_first_col"] = [v for r in range(world)
                                           for v in tail[r * nbytes:r * nbytes + Bc * nu * 8].view(torch.float64)
                                           .view(Bc, nu)[:nrows[r], 0].tolist()]
    else:
        out["kernel_ms"] = kern_ms
        out["step_gpu_ms"] = step_ms   # generation + solve kernels of one step (HIP events)
        out["roofline"] = roofline(args, name, cfg, mmpc, solver, ksolver, N, nx, nu, n, iters, kern_ms, hess)
    if name == "cfg5" and world == 1 and not standin and not args.no_sweep:
        out["tolerance_sweep"] = cfg5_sweep(path, cfg, n, x0, up, tr, w, args.hessian)
    if (name == "cfg2" and primary and world == 1 and not standin and not args.no_sweep and args.u_bound is None
            and args.x_bound is None and args.tol is None and args.kkt == "auto" and args.hessian == "auto"):
        out["tolerance_sweep"] = cfg5_sweep(path, cfg, n, x0, up, tr, w, args.hessian, fp32=False)
    if (name == "cfg3" and world == 1 and not standin and not args.no_sweep and args.tol is None
            and (not primary or (args.u_bound is None and args.x_bound is None and args.kkt == "auto"
                                 and args.hessian == "auto"))):
        # the exo solve at the reference's IPOPT tolerance (ModelControl.cpp:54) beside the line's 1e-8 / 1e-10
        out["tolerance_sweep"] = cfg5_sweep(path, cfg, n, x0, up, tr, w, "auto", fp32=False)
        # and with IPOPT's exact Hessian (the line runs Gauss-Newton, the exo's AUTO choice): iteration histograms
        out["exact_hessian"] = hessian_compare(path, n, x0, up, tr, w, V, iters)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not standin and name != "cfg5":
        out["cpu_baseline"] = cpu_baseline(cfg, N, h, args.cpu_seconds, V.cpu().numpy(), iters, tol_grad,
                                           tol_defect, hess, None if ulb is None else args.u_bound,
                                           args.x_bound if primary else None, ksolver)
    if hbuf:
        for hb in hbuf:
            hb.close()
    if not standin:
        solver.close()
    return out


def cfg5_sweep(path, cfg, B, x0, up, tr, w, hessian, reps=5, fp32=True):
    """SURVEY.md 8d cfg#5: the fp32-factor solve over the outer tolerance {1e-5, 1e-6, 1e-8} (tol_grad = tol,
    tol_defect = tol / 100) -- % converged, mean / max SQP iterations, kernel ms (HIP events, median of `reps` after one untimed solve) and
    max_i ||V_i - V_i,fp64|| / ||V_i,fp64|| against the fp64-factor solve at the default tolerances.
    fp32=False (cfg#2, cfg#3): the same sweep of the fp64 solve -- what the kernel does at the reference's own
    IPOPT tolerance (tol = 1e-5, ModelControl.cpp:54) and at SURVEY.md A9's build criterion (1e-6 / 1e-8), beside
    the line's 1e-8 / 1e-10."""
    import torch
    import mmpc

    def run(tol, fp32):
        s = mmpc.Solver(path, tol_grad=tol, tol_defect=tol / 100, factor_fp32=int(fp32))
        s.reserve_workspace(B)
        V = torch.zeros((B, s.NV), dtype=torch.float64, device=x0.device)
        st = torch.zeros(B, dtype=torch.int32, device=x0.device)
        it = torch.zeros(B, dtype=torch.int32, device=x0.device)
        times = []
        for r in range(reps + 1):   # the first solve is an untimed warm-up of this tolerance's handle
            V.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.solve_batch(B, x0, up, tr, w, V, st, it, None)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times.append(e0.elapsed_time(e1))
        s.close()
        return V, st.cpu().numpy(), it.cpu().numpy(), float(np.median(times))

    Vref, st_ref, it_ref, t_ref = run(1e-8, False)
    nref = torch.linalg.vector_norm(Vref, dim=1)
    rows = []
    for tol in ((1e-5, 1e-6, 1e-8) if fp32 else (1e-5, 1e-6)):
        V, st, it, t = run(tol, fp32)
        rel = (torch.linalg.vector_norm(V - Vref, dim=1) / nref).max().item()
        rows.append({"factor": "fp32" if fp32 else "fp64", "tol_grad": tol, "tol_defect": tol / 100,
                     "converged_pct": float((st == 0).mean() * 100),
                     "mean_iters": float(it.mean()), "max_iters": int(it.max()), "kernel_ms": t,
                     "solves_per_s_kernel": B / (t * 1e-3), "max_rel_V_vs_fp64": rel})
    rows.append({"factor": "fp64", "tol_grad": 1e-8, "tol_defect": 1e-10, "converged_pct": float((st_ref == 0).mean() * 100),
                 "mean_iters": float(it_ref.mean()), "max_iters": int(it_ref.max()), "kernel_ms": t_ref,
                 "solves_per_s_kernel": B / (t_ref * 1e-3), "max_rel_V_vs_fp64": 0.0})
    return rows


def hessian_compare(path, B, x0, up, tr, w, V_gn, it_gn, reps=3):
    """The same batch with the exact Lagrangian Hessian (mmpc_opts.hessian = EXACT; IPOPT's default, nlp_hess_l at
    ModelGenerator.cpp:238) beside the line's Hessian: iteration histograms, kernel ms (HIP events, median of `reps`
    after one untimed solve) and the largest relative difference of the solutions (same KKT point)."""
    import torch
    import mmpc
    s = mmpc.Solver(path, hessian=mmpc.HESSIAN_EXACT, init_states=mmpc.INIT_ZERO)
    s.reserve_workspace(B)
    V = torch.zeros((B, s.NV), dtype=torch.float64, device=x0.device)
    st = torch.zeros(B, dtype=torch.int32, device=x0.device)
    it = torch.zeros(B, dtype=torch.int32, device=x0.device)
    times = []
    for r in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s.solve_batch(B, x0, up, tr, w, V, st, it, None)
        e1.record()
        torch.cuda.synchronize()
        if r:
            times.append(e0.elapsed_time(e1))
    ksolver = s.kkt_solver_for(B)
    s.close()
    hist = lambda a: {int(k): int(v) for k, v in zip(*np.unique(a, return_counts=True))}  # noqa: E731
    itn, stn = it.cpu().numpy(), st.cpu().numpy()
    scale = torch.clamp(V_gn.abs().amax(dim=1), min=1e-300)
    return {"hessian": "exact (Lagrangian, IPOPT's default)",
            "kkt_solver": {2: "riccati (lane per instance)", 3: "riccati (16 lanes per instance)"}.get(ksolver, ksolver),
            "converged": int((stn == 0).sum()), "mean_iters": float(itn.mean()), "max_iters": int(itn.max()),
            "iters_hist": hist(itn), "kernel_ms": float(np.median(times)),
            "line_hessian_iters_hist": hist(it_gn),
            "max_rel_V_vs_line": float(((V - V_gn).abs().amax(dim=1) / scale).max().item())}


def model_flops_per_iteration(mmpc, cfg, ksolver, N, hess):
    """Model-evaluation flops of one SQP iteration (full step accepted), reported beside the kernel's own KKT-algebra
    count as SURVEY.md 8(d) asks ("Dynamics/Jacobian evaluation flops ... reported separately"): per-evaluation costs
    from the compiled gfx950 code (mahi-mpc_amd/mmpc/model_flops.json, tools/model_flops.py; sin and cos one op each)
    x the evaluations per stage the kernel runs per iteration:
      16-lane kernel (sqp_group.h): the alpha = 1 trial with its Jacobian (phase A's data for the next iteration), and
        with the exact Hessian the stage Hessian W_k;
      lane kernel (sqp_lane.h): the Jacobian in the backward sweep; A dx + B du at (x_k, u_k) in the step sweep and
        A d at the full-step point (the next forward pass) -- directional derivatives for a model that has them (the
        exo: acc_jac_h + 2 jvp), Jacobians otherwise (3 acc_jac).
    The first iteration's initial evaluation and any alpha < 1 trial are not counted (a lower bound)."""
    try:
        tab = json.load(open(os.path.join(os.path.dirname(mmpc.__file__), "model_flops.json")))["models"]
    except (OSError, ValueError, KeyError):
        return None
    model = tab.get("ExoArm" if cfg["model"] == "exo_arm" else "TwoLinkArm")
    if model is None:
        return None
    if ksolver == 3:
        ev = {"acc_jac": 1, "hess": 1 if hess == mmpc.HESSIAN_EXACT else 0}
    elif ksolver == 2:
        ev = {"acc_jac_h": 1, "jvp": 2} if "jvp" in model else {"acc_jac": 3}
    else:
        return None
    ev = {k: v for k, v in ev.items() if v}
    if any(k not in model for k in ev):
        return None
    return {"total": N * sum(n * model[k]["flops"] for k, n in ev.items()), "evals_per_stage": ev}


def roofline(args, name, cfg, mmpc, solver, ksolver, N, nx, nu, B, iters, kern_ms, hess):
    """FP64-VALU roofline of the solve kernel (the only kernel of a step besides a memset and the result pack; a
    lane-kernel solve adds the 16-lane resume launch of its iteration tail, DESIGN.md 4b, inside the same bracket).

    achieved = the kernel's OWN algorithmic flop count (mmpc.*_flops_per_iteration: structure-exploiting, no
    flop on structural zeros, model evaluations excluded) x the SQP iterations its instances took / the mean
    kernel duration (HIP events on the launch stream).  peak = FP64 vector peak (no kernel issues MFMA: DESIGN.md
    "Why no MFMA"; cfg#5 prices its fp32 share at the fp64 peak, i.e. conservatively high).  The SURVEY.md 8(d)
    count (explicit condensing + dense Cholesky, 288 kflop/iter at cfg#2) is reported beside it as the
    algorithm-equivalent rate: it is NOT the work the kernel does."""
    riccati = ksolver in (2, 3)
    if riccati:
        fl = mmpc.riccati_flops_per_iteration(N, nx, nu, exact=hess == mmpc.HESSIAN_EXACT)
        model = "ExoArm" if cfg["model"] == "exo_arm" else "TwoLinkArm"
        if ksolver == 3:
            kname = f"sqp_group_kernel<{model}"
        else:
            kname = f"sqp_lane_kernel<{model}"
    else:
        fl = mmpc.flops_per_iteration(N)
        kname = f"sqp_wave_kernel<TwoLinkArm,{30 if 16 < N <= 30 else (16 if N <= 16 else 32)}>"
    sec = kern_ms * 1e-3
    own = float(iters.sum()) * fl["total"] / sec / 1e12
    survey = float(iters.sum()) * mmpc.survey_flops_per_iteration(N, nx, nu) / sec / 1e12
    traffic = None
    traffic_src, pmc = None, {}
    sha = lib_sha256(os.path.realpath(mmpc.LIB_PATH))
    pmc_status = "no PMC summary for this config/kernel"
    if os.path.exists(args.traffic_json):   # keyed "<config>:<kernel name prefix>", tied to a library build
        try:
            for key, tj in json.load(open(args.traffic_json)).items():
                if not (key.startswith(f"{name}:{kname}") and isinstance(tj, dict) and tj.get("batch") == B
                        and tj.get("horizon") == N):
                    continue
                if tj.get("lib_sha256") != sha:
                    pmc_status = f"PMC summary {tj.get('source')} measured another build ({tj.get('lib_sha256')})"
                    continue
                traffic, traffic_src, pmc = tj.get("hbm_bytes_per_launch"), tj.get("source"), tj
                pmc_status = "PMC of this exact library build (sha256 match)"
        except (OSError, ValueError):
            traffic = None
    alg_bytes = B * (8 * (nx + nu + N * nx + 2 * (nx * (N + 1) + nu * N)) + 12)   # SURVEY.md 8d, per launch
    mflops = model_flops_per_iteration(mmpc, cfg, ksolver, N, hess)
    # measured bandwidth side (VERDICT r5 ask 5): the PMC's HBM bytes of the solve kernel over that kernel's duration
    # in the same PMC session (its kernel-trace pass; the event bracket of a lane-kernel solve also holds the resume
    # launch, which the PMC entry does not count), as a fraction of the 8 TB/s HBM3E peak
    pmc_ms = pmc.get("kernel_ms_at_measurement") or kern_ms
    hbm_tbs = traffic / (pmc_ms * 1e-3) / 1e12 if traffic else None
    hbm_frac = hbm_tbs / HBM_PEAK_TBS if hbm_tbs else None
    fp64_frac = own / FP64_PEAK_TFLOPS
    bound = "hbm" if hbm_frac is not None and hbm_frac > fp64_frac else "fp64-valu"
    lane_tail = ksolver == 2 and not cfg.get("linear")   # tail_plan: the resume launch runs in the bracket
    return {"bound": bound, "achieved": own, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": fp64_frac, "traffic": traffic,
            "hbm_tbs_measured": hbm_tbs,
            "hbm_frac_measured": hbm_frac,
            "hbm_peak_tbs": HBM_PEAK_TBS,
            "bound_rule": ("the larger of frac (the kernel's own algorithmic FP64 flops / FP64 peak) and "
                           "hbm_frac_measured (PMC HBM bytes per launch / that launch's duration / HBM peak); "
                           "achieved / peak / frac stay the FP64 figures"),
            "traffic_source": traffic_src,
            "lib_sha256": sha,
            "pmc_status": pmc_status,
            "kernel": kname,
            "bracket": ("the lane kernel + the 16-lane resume launch of its iteration tail (DESIGN.md 4b): all of a "
                        "solve's iterations" if lane_tail else "the solve kernel"),
            "flops_per_iter_kernel_own_count": fl["total"],
            "flops_per_iter_survey_8d": mmpc.survey_flops_per_iteration(N, nx, nu),
            "survey_8d_equivalent_tflops": survey,
            "survey_8d_equivalent_frac": survey / FP64_PEAK_TFLOPS,
            "model_eval_flops_per_iter": mflops and mflops["total"],
            "model_evals_per_stage_iter": mflops and mflops["evals_per_stage"],
            "achieved_incl_model_evals": (float(iters.sum()) * (fl["total"] + mflops["total"]) / sec / 1e12
                                          if mflops else None),
            "frac_incl_model_evals": (float(iters.sum()) * (fl["total"] + mflops["total"]) / sec / 1e12
                                      / FP64_PEAK_TFLOPS if mflops else None),
            "algorithmic_hbm_bytes_per_launch": alg_bytes,
            "hbm_gbs_algorithmic": alg_bytes / sec / 1e9,
            "pmc_fp64_valu_flops_issued_per_launch": pmc.get("fp64_valu_flops_issued_per_launch"),
            "pmc_fp64_valu_frac_issued": (pmc["fp64_valu_flops_issued_per_launch"] / sec / 1e12 / FP64_PEAK_TFLOPS
                                          if pmc.get("fp64_valu_flops_issued_per_launch") else None),
            "pmc_mfma_counters": pmc.get("mfma_counters"),
            "pmc_lds_bank_conflict_cycles_per_launch": pmc.get("lds_bank_conflict_cycles"),
            "pmc_valu_active_frac": pmc.get("valu_active_frac"),
            "note": "frac = the kernel's own algorithmic flops / FP64 vector peak (no kernel issues MFMA: DESIGN.md "
                    "'Why no MFMA'); pmc_* = rocprofv3 counters (tools/pmc.sh) of the same kernel, shape and library "
                    "build (lib_sha256): issued FP64 VALU lane-flops incl. inactive-lane slots; *_incl_model_evals add "
                    "the model / Jacobian / Hessian evaluation flops (model_eval_flops_per_iter, SURVEY.md 8(d))"}


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args, argv))
    run_rank(args)


if __name__ == "__main__":
    main()
