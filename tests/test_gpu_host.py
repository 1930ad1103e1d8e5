"""GPU: the reference's closed-loop example driven through the drop-in C++ API (mahi-mpc_amd/host,
examples/model_control_example.cpp) against the same closed loop computed with the CPU oracle:
calc_u every 5th tick with warm start (ModelControl.cpp:159-163), control_at_time semantics
(ModelControl.cpp:192-197) and an explicit-Euler plant (model_control_example.cpp:81-86).
Tolerance: states/controls within 1e-7 relative over the run (the per-solve agreement is ~1e-12; the loop
only propagates it)."""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, WEIGHTS_CFG

pytestmark = pytest.mark.gpu
HOST = os.path.join(ROOT, "mahi-mpc_amd", "host")


def oracle_closed_loop(oracle, N, sim_s, linear, hessian=0):
    h, nx = 0.002, 4
    state, control = np.zeros(4), np.zeros(2)
    V = None
    rows = []
    t_us, cycle, res_t0 = 0, 0, None
    Vsol = None
    while t_us < int(round(sim_s * 1e6)) - 0:
        t = t_us * 1e-6
        tt, traj = t, []
        for i in range(N):
            row = []
            for j in range(nx):
                if j < nx // 2:
                    row.append((1.0 if j % 2 == 0 else -1.0) * math.sin(2 * math.pi * tt))
                else:
                    row.append((1.0 if (j - nx // 2) % 2 == 0 else -1.0) * 2 * math.pi * math.cos(2 * math.pi * tt))
            traj.append(row)
            tt += h
        if cycle % 5 == 0:
            r = oracle.solve_batch(N, h, state[None], control[None], np.array(traj)[None], np.array(WEIGHTS_CFG),
                                   V=V, is_linear=linear, hessian=hessian)
            V = r["V"]
            Vsol, res_t0, st, it = V[0], t_us, int(r["status"][0]), int(r["iters"][0])
        # control_at_time: last result with time < t, else the first (times in integer microseconds)
        times = [res_t0 + int(round(2000 * i)) for i in range(N)]
        i = 0
        while i < N and times[i] < t_us:
            i += 1
        k = 0 if i == 0 else i - 1
        control = Vsol[6 * k + 4:6 * k + 6].copy()
        rows.append([t, *state, *control, st, it])
        _, _, xd = oracle.two_link_jac(state, control)
        state = state + xd * h
        t_us += 2000
        cycle += 1
    return np.array(rows)


@pytest.mark.parametrize("linear", [False, True])
def test_closed_loop_example_matches_oracle(linear, oracle, model_json, mmpc_mod, tmp_path):
    subprocess.run(["make", "-s", "-C", HOST], check=True)
    N, sim_s = 20, 0.2
    args = [os.path.join(HOST, "bin", "model_control_example"), str(N), str(sim_s)] + (["l"] if linear else [])
    out = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rows = np.array([[float(v) for v in line.split(",")] for line in out.stdout.splitlines() if line and line[0].isdigit()])
    # the Hessian the example's one-instance solves resolve to (exact for the nonlinear 2-link arm)
    hess = mmpc_mod.Solver(model_json(N=N, is_linear=linear)).hessian_for(1)
    ref = oracle_closed_loop(oracle, N, sim_s, linear, hessian=hess - 1)
    assert rows.shape == ref.shape, (rows.shape, ref.shape)
    assert (rows[:, 7] == 0).all()                                  # every GPU solve converged
    np.testing.assert_allclose(rows[:, 1:7], ref[:, 1:7], rtol=1e-7, atol=1e-9)


def test_generated_linear_functions_casadi_abi(golden_kat, oracle, mmpc_mod, tmp_path):
    """<name>_get_A/_get_B/_get_x_dot_init of the generated <name>_linear_functions.so, called through the CasADi
    external C ABI (src/codegen_usage.cpp:73-181) with ctypes: CasADi column-major outputs equal to the device
    linearisation bit for bit, and to the sympy K2/K3 fixtures (2-link, 1e-11) / the oracle (exo, 1e-12)."""
    import ctypes as C
    mmpc_mod.lib()  # HIP runtime initialised as every caller in this process does it (torch first, mmpc.lib)
    subprocess.run(["make", "-s", "-C", HOST], check=True)
    out = subprocess.run([os.path.join(HOST, "bin", "host_selftest")], cwd=tmp_path, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731

    def call(lib, fn, x, u, nout):
        f = getattr(lib, fn)
        f.restype = C.c_int
        arg = (C.POINTER(C.c_double) * 2)(dp(x), dp(u))
        r = np.full(nout, np.nan)
        res = (C.POINTER(C.c_double) * 1)(dp(r))
        assert f(arg, res, None, None, 0) == 0
        return r

    rng = np.random.default_rng(3)
    for name, nx, nu in (("selftest_double_pendulum", 4, 2), ("selftest_exo", 8, 4)):
        lib = C.CDLL(str(tmp_path / f"{name}_linear_functions.so"))
        s = mmpc_mod.Solver(str(tmp_path / f"{name}.json"))
        if nx == 4:
            pts = [(np.array(p["x"], float), np.array(p["u"], float), np.array(p["A"]), np.array(p["B"]), 1e-11)
                   for p in golden_kat["K3"]["points"]]
        else:
            pts = []
            for _ in range(4):
                x, u = rng.uniform(-1, 1, nx), rng.uniform(-2, 2, nu)
                Ao, Bo, _ = oracle.exo_jac(x, u)
                pts.append((x, u, Ao, Bo, 1e-12))
        for x, u, Aref, Bref, tol in pts:
            A = call(lib, name + "_get_A", x, u, nx * nx).reshape(nx, nx).T   # column-major -> row-major
            Bm = call(lib, name + "_get_B", x, u, nx * nu).reshape(nu, nx).T
            xd = call(lib, name + "_get_x_dot_init", x, u, nx)
            Ad, Bd, xdd = s.linearize_host(x[None], u[None])
            np.testing.assert_array_equal(A, Ad[0])
            np.testing.assert_array_equal(Bm, Bd[0])
            np.testing.assert_array_equal(xd, xdd[0])
            np.testing.assert_allclose(A, Aref, rtol=tol, atol=tol * np.abs(Aref).max())
            np.testing.assert_allclose(Bm, Bref, rtol=tol, atol=tol * np.abs(Bref).max())


def test_calc_u_batch_enforces_control_limits(oracle, mmpc_mod, tmp_path):
    """ModelControl::calc_u_batch with update_control_limits (ModelControl.cpp:148-154,205-209): the batched
    solutions stay inside the control box and equal the oracle's bounded SQP with the Hessian the library resolves
    for that solve (same algorithm; 1e-10)."""
    subprocess.run(["make", "-s", "-C", HOST], check=True)
    N, B, lim = 30, 24, 2.0
    x0, up, tr = oracle.synth(20250213, 0, B, N, 0.002)
    stdin = "\n".join(" ".join(repr(float(v)) for v in np.concatenate([x0[b], up[b], tr[b].ravel()]))
                      for b in range(B))
    out = subprocess.run([os.path.join(HOST, "bin", "calc_u_batch_example"), str(N), str(lim)], cwd=tmp_path,
                         input=stdin, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rows = np.array([[float(v) for v in line.split()] for line in out.stdout.splitlines()
                     if line[:1].isdigit() or line[:1] == "-"])   # ModelGenerator prints progress lines first
    assert rows.shape == (B, 1 + 4 * (N + 1) + 2 * N)
    st, V = rows[:, 0].astype(int), rows[:, 1:]
    assert (st == 0).all(), st
    U = np.stack([V[:, 6 * k + 4:6 * k + 6] for k in range(N)], axis=1)
    assert (np.abs(U) <= lim).all()
    assert (np.abs(U) == lim).any()   # the limits bind for some of these instances
    s = mmpc_mod.Solver(str(tmp_path / "calc_u_batch_double_pendulum.json"))   # the JSON the example generated
    o = oracle.solve_batch(N, 0.002, x0, up, tr, np.array(WEIGHTS_CFG), u_lb=[-lim, -lim], u_ub=[lim, lim], solver=s)
    np.testing.assert_allclose(V, o["V"], rtol=0, atol=1e-10 * np.abs(o["V"]).max())


def test_threaded_loop_example(model_json, tmp_path):
    """ModelControl's worker thread (start_calc / set_state / control_at_time / stop_calc, ModelControl.cpp:75-114)
    in the reference's threaded example loop (thread_model_control_example.cpp:53-120, with Rm given): a 1 kHz
    plant thread publishes snapshots while the worker solves from the latest one on the GPU; every applied control
    is finite, the last solve converged, and the arm follows the 1 rad sinusoid (tracking error below its
    amplitude in the second half).  The TSan build of the same loop: tools/tsan_build.sh + tools/tsan_run.sh."""
    subprocess.run(["make", "-s", "-C", HOST], check=True)
    exe = os.path.join(HOST, "bin", "model_control_example")
    out = subprocess.run([exe, "20", "0.5", "n", "-", "thread"], cwd=tmp_path, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    line = [l for l in out.stdout.splitlines() if l.startswith("thread,")][-1].split(",")
    ticks, status, umax, err, finite = int(line[1]), int(line[2]), float(line[3]), float(line[4]), int(line[5])
    assert ticks >= 400 and finite == 1 and status == 0, line
    assert 0 < umax < 1e3 and err < 1.0, line
