#!/usr/bin/env python3
"""Benchmark of the MI355X batched NMPC solve path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 4096] [--horizon 30]

One "step" = one cold-started batched SQP solve of B independent cfg#2 instances (2-link arm,
nx=4, nu=2, N=30, h=2 ms, fp64), i.e. what the reference does per control tick in
ModelControl::calc_u (src/Mahi/Mpc/ModelControl.cpp:116-172) -- from V = 0 with x_0 pinned, the
reference's first-call state -- for B instances at once.  Inputs are generated on the device from
(seed, global instance index) before the timed region (weak scaling: every rank solves its own
B instances; results are independent of the GPU count).

Prints ONE JSON line on rank 0 (driver contract) with two extra objects:
  roofline      achieved algorithmic FP64 rate of the fused SQP kernel vs the MI355X FP64 peak,
                kernel time from HIP events on the launch stream;
  cpu_baseline  the oracle/ CPU restatement (same GN-SQP, fp64) on a bounded sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import json
import os
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
CONFIGS = {
    "cfg2": dict(model="two_link_arm", nx=4, nu=2, N=30, B=4096, weights=WEIGHTS, metric=METRIC,
                 workload="cfg#2: 2-link arm nx=4 nu=2, N=30, h=2 ms, cold-start GN-SQP to ||grad||<=1e-8, ||g||<=1e-10"),
    "cfg3": dict(model="exo_arm", nx=8, nu=4, N=50, B=65536, weights=WEIGHTS_EXO,
                 metric="MPC solves/sec (whole node), exo nx=8 N=50 batch (SURVEY.md 8d cfg#3/#4)",
                 workload="cfg#3: 4-DoF exo nx=8 nu=4 (build-defined parameters), N=50, h=2 ms, cold-start GN-SQP "
                          "(Riccati KKT) to ||grad||<=1e-8, ||g||<=1e-10"),
}
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector = FP64 matrix peak (AMD spec)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg2",
                    help="cfg2 = headline (BASELINE.json); cfg3 = exo workload of SURVEY.md 8d")
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU (cfg#2: 4096, cfg#3: 65536)")
    ap.add_argument("--kkt", choices=["auto", "condensed", "riccati", "group"], default="auto",
                    help="KKT solver (mmpc_opts.kkt_solver); auto = the library's choice")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip gathering the results to rank 0")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline wall time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--init", choices=["as_given", "hold_x0"], default="as_given",
                    help="mmpc_opts.init_states: the reference's cold start (V = 0) or x_1..x_N = x_0 (DESIGN 3d)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per launch per config (tools/pmc.sh + tools/pmc_summary.py)")
    return ap.parse_args()


def cpu_baseline(cfg, N, h, target_s):
    """Oracle (oracle/liboracle.so, the same GN-SQP in plain C + OpenMP) on a bounded sample."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as o
    model = o.EXO if cfg["model"] == "exo_arm" else o.TWO_LINK
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    w = np.array(cfg["weights"])
    n0 = 2 * threads
    x0, up, tr = o.synth(SEED, 0, n0, N, h, model=model)
    t = time.perf_counter()
    o.solve_batch(N, h, x0, up, tr, w, nthreads=threads, model=model)
    dt = time.perf_counter() - t
    n = int(max(n0, min(200000, n0 * target_s / max(dt, 1e-6))))
    x0, up, tr = o.synth(SEED, 0, n, N, h, model=model)
    t = time.perf_counter()
    r = o.solve_batch(N, h, x0, up, tr, w, nthreads=threads, model=model)
    dt = time.perf_counter() - t
    return dict(value=n / dt, unit="solves/s", cores=threads, kind="port",
                sample=f"first {n} {cfg['workload'].split(':')[0]} instances (seed {SEED}), cold start, {dt:.1f} s "
                       f"wall, {int((r['status'] == 0).sum())}/{n} converged, oracle dense condensed GN-SQP, "
                       f"{threads} OpenMP threads")


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import mmpc
    import mmpc.dist as mdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = CONFIGS[args.config]
    B = args.batch or cfg["B"]
    N = args.horizon or cfg["N"]
    nx, nu, h_us = cfg["nx"], cfg["nu"], 2000
    h = h_us * 1e-6

    tmpdir = tempfile.mkdtemp(prefix="mmpc_bench_")
    path = mmpc.write_model_json(os.path.join(tmpdir, f"{cfg['model']}.json"), cfg["model"], nx, nu, h_us, N,
                                 model=cfg["model"])
    ksolver = {"auto": 0, "condensed": 1, "riccati": 2, "group": 3}[args.kkt]
    solver = mmpc.Solver(path, device=local, kkt_solver=ksolver,
                         init_states=mmpc.INIT_HOLD_X0 if args.init == "hold_x0" else mmpc.INIT_AS_GIVEN)
    solver.reserve_workspace(B)
    ksolver = solver.kkt_solver_for(B)   # the AUTO choice, resolved by the library
    riccati = ksolver in (2, 3)
    NV = solver.NV
    f64 = dict(dtype=torch.float64, device=dev)
    x0 = torch.empty((B, nx), **f64)
    up = torch.empty((B, nu), **f64)
    tr = torch.empty((B, N, nx), **f64)
    w = torch.tensor(cfg["weights"], **f64)
    V = torch.zeros((B, NV), **f64)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    kkt = torch.empty(B, **f64)
    stream = torch.cuda.current_stream(dev)
    first, _ = mdist.shard(B, rank)
    solver.synth(SEED, first, B, x0, up, tr, stream=stream.cuda_stream)
    mdist.broadcast_shared(w)   # shared weights from rank 0 (identical here by construction)
    # N > 1: every step's per-instance results (u_0*, status, iterations) go to rank 0 -- one RCCL
    # all_gather_into_tensor over xGMI per step, issued async so it overlaps the next step's solve
    gather = mdist.ResultGather(B, nx, nu) if (world > 1 and not args.no_gather) else None

    def step():
        V.zero_()   # cold start (reference first call: v_init = 0, ModelControl.cpp:29-50)
        solver.solve_batch(B, x0, up, tr, w, V, st, it, kkt, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        V.zero_()
        ev[k][0].record(stream)
        solver.solve_batch(B, x0, up, tr, w, V, st, it, kkt, stream=stream.cuda_stream)
        ev[k][1].record(stream)
        if gather:
            gather.post(V, st, it)
    if gather:
        gather.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    elapsed = mdist.max_over_ranks(elapsed, device=dev)

    iters = it.cpu().numpy()
    status = st.cpu().numpy()
    if gather:   # rank 0 holds every instance's result of the last step
        last = gather.last()
        gathered_ok = bool(torch.equal(last[rank * B:(rank + 1) * B, :nu], V[:, nx:nx + nu]))
        conv = int((last[:, nu] == 0).sum().item())
        gathered_ok = bool(mdist.sum_over_ranks(int(not gathered_ok), device=dev) == 0)
    else:
        conv = int(mdist.sum_over_ranks(int((status == 0).sum()), device=dev))
    total = B * world * args.steps
    value = total / elapsed
    # algorithmic flops of one launch = per-iteration figure x the SQP iterations the launch's instances
    # actually took (unit of work = 1 solve = sum over its iterations), SURVEY.md 8(d)'s figure whichever KKT
    # solver ran -- except where that figure (which prices the condensed algorithm: 9.3 MFLOP/iter at cfg#3)
    # would put a Riccati kernel above the FP64 peak; there the kernel's own algorithmic count is used
    # (both are reported).
    survey_fl = float(iters.sum()) * mmpc.survey_flops_per_iteration(N, nx, nu)
    survey_tf = survey_fl / (kern_ms * 1e-3) / 1e12
    if riccati:
        fl = mmpc.riccati_flops_per_iteration(N, nx, nu)
        own_fl = float(iters.sum()) * fl["total"]
        achieved = survey_tf if survey_tf <= FP64_PEAK_TFLOPS else own_fl / (kern_ms * 1e-3) / 1e12
        kname = (f"sqp_{'group' if ksolver == 3 else 'lane'}_kernel<"
                 f"{'ExoArm' if cfg['model'] == 'exo_arm' else 'TwoLinkArm'}>")
    else:
        fl = mmpc.flops_per_iteration(N)
        own_fl = float(iters.sum()) * fl["total"]
        achieved = survey_fl / (kern_ms * 1e-3) / 1e12
        kname = f"sqp_wave_kernel<TwoLinkArm,{30 if 16 < N <= 30 else (16 if N <= 16 else 32)}>"
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json)).get(f"{args.config}:{kname}", {})
            if tj.get("batch") == B and tj.get("horizon") == N:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": cfg["metric"],
        "value": value,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic: counter-based splitmix64 {args.config} instances (SURVEY.md 8d), generated on device",
        "config": {"workload": cfg["workload"], "batch_per_gpu": B, "global_batch": B * world,
                   "horizon": N, "kkt_solver": {1: "condensed (wave per instance)", 2: "riccati (lane per instance)",
                                                3: "riccati (16 lanes per instance)"}[ksolver],
                   "init_states": "V as given (reference cold start V = 0)" if args.init == "as_given"
                   else "x_1..x_N = x_0 (MMPC_INIT_HOLD_X0)",
                   "parallelism": (f"batch-shard x{world}; per-step results (u_0*, status, iters) to rank 0 by "
                                   "RCCL all_gather_into_tensor, overlapped with the next solve"
                                   if gather else f"batch-shard x{world} (no collective on the solve path)")},
        "converged": conv,
        **({"gathered_results_match": gathered_ok} if gather else {}),
        "mean_sqp_iters": float(iters.mean()),
        "kernel_ms": kern_ms,
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "kernel": kname,
                     "flops_per_iter_survey_8d": mmpc.survey_flops_per_iteration(N, nx, nu),
                     "flops_per_iter_kernel_own_count": fl["total"],
                     "kernel_own_count_tflops": own_fl / (kern_ms * 1e-3) / 1e12,
                     "survey_8d_equivalent_tflops": survey_fl / (kern_ms * 1e-3) / 1e12},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, N, h, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
