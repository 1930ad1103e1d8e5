"""bench.py's multi-GPU launcher on CPU (gloo, stand-in solver): ``--gpus N`` without WORLD_SIZE starts N rank
processes, each solves its own shard of global instances [r B, (r+1) B), the per-step results reach rank 0's
host through one all_gather_into_tensor, and the JSON line reports the whole job (n_gpus = N,
global_batch = N B).  The stand-in solver is bench.py's plumbing double, not the solve path (no GPU here)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.slow
@pytest.mark.parametrize("gpus", [1, 2, 3])
def test_launcher_spawns_ranks(gpus):
    B = 8
    out = _run("--standin", "--gpus", str(gpus), "--batch", str(B), "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline")
    assert out["n_gpus"] == gpus
    assert out["config"]["global_batch"] == gpus * B and out["config"]["batch_per_gpu"] == B
    assert out["gathered_results_match"] is True
    assert out["converged"] == gpus * B
    assert out["steps"] == 3 and out["warmup"] == 1 and out["scaling"] == "weak"
    # rank r's rows are global instances r*B .. r*B+B-1 (u_0* := x0[:, 0] = global index in the stand-in)
    assert out["standin_u0_first_col"] == [float(i) for i in range(gpus * B)]
    assert out["value"] > 0 and out["ms_per_step"] > 0


def test_launcher_propagates_rank_failure():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--standin", "--gpus", "2",
                        "--config", "nope"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0


@pytest.mark.slow
@pytest.mark.parametrize("gpus", [2, 3])
def test_launcher_strong_scaling_ragged(gpus):
    """--strong: the global batch (here 10, ragged over 3 ranks) is split in contiguous shard_strong shards; the
    gathered table holds every global instance once, in order, and value counts the global batch per step."""
    out = _run("--standin", "--strong", "--gpus", str(gpus), "--batch", "10", "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline")
    assert out["scaling"] == "strong" and out["config"]["global_batch"] == 10
    assert out["gathered_results_match"] is True and out["converged"] == 10
    assert out["standin_u0_first_col"] == [float(i) for i in range(10)]


def test_model_eval_flops_table():
    """bench.py's roofline reports the model-evaluation flops beside the KKT algebra; the table
    comes from the compiled gfx950 code (tools/model_flops.py) and covers every evaluation the default lines use."""
    import bench
    import mmpc
    g = bench.model_flops_per_iteration(mmpc, bench.CONFIGS["cfg2"], 3, 30, mmpc.HESSIAN_EXACT)
    assert g["evals_per_stage"] == {"acc_jac": 1, "hess": 1} and 5_000 < g["total"] < 50_000
    gn = bench.model_flops_per_iteration(mmpc, bench.CONFIGS["cfg2"], 3, 30, mmpc.HESSIAN_GAUSS_NEWTON)
    assert gn["evals_per_stage"] == {"acc_jac": 1} and gn["total"] < g["total"]
    e = bench.model_flops_per_iteration(mmpc, bench.CONFIGS["cfg3"], 2, 50, mmpc.HESSIAN_GAUSS_NEWTON)
    f = bench.model_flops_per_iteration(mmpc, bench.CONFIGS["cfg5"], 2, 50, mmpc.HESSIAN_GAUSS_NEWTON)
    # the exo lane kernel: the backward sweep's h-scaled Jacobian and two directional derivatives (step sweep, next
    # forward pass at the full-step point), fp64 and fp32 factor alike
    assert e["evals_per_stage"] == {"acc_jac_h": 1, "jvp": 2} and f["evals_per_stage"] == e["evals_per_stage"]
    assert f["total"] == e["total"] > 50_000
    assert bench.model_flops_per_iteration(mmpc, bench.CONFIGS["cfg2"], 1, 30, mmpc.HESSIAN_GAUSS_NEWTON) is None


def test_forced_collectives_one_rank():
    """--rccl at N = 1: a one-rank process group (gloo in the stand-in, RCCL on a GPU) and the last step's table
    through all_gather_into_tensor, as the N > 1 path; the line names the process group."""
    out = _run("--standin", "--rccl", "--batch", "8", "--steps", "3", "--warmup", "1", "--no-cpu-baseline")
    assert out["n_gpus"] == 1 and out["gathered_results_match"] is True and out["converged"] == 8
    assert out["process_group"]["backend"] == "gloo" and out["process_group"]["world_size"] == 1
    assert out["standin_u0_first_col"] == [float(i) for i in range(8)]


def test_strong_rejects_batch_below_rank_count():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--standin", "--strong", "--gpus", "3",
                        "--batch", "2", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0
