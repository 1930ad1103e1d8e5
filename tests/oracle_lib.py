"""ctypes access to oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
always as the checker (never on the product path).  See oracle/mmpc_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

NX, NU = 4, 2                       # 2-link arm (model 0)
TWO_LINK, EXO, USER = 0, 1, 2
HESS_GAUSS_NEWTON, HESS_EXACT = 0, 1   # oracle_set_hessian (mmpc_opts.hessian after resolution)
KKT_DENSE, KKT_RICCATI = 0, 1          # oracle_set_kkt: explicit condensing + Cholesky, or the kernels' Riccati
DIMS = {TWO_LINK: (4, 2), EXO: (8, 4)}
USER_DIR = os.path.join(ORACLE_DIR, "_user")
_lib = None
_user = {}  # host-build path -> (CDLL, dims)

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_two_link_jac.argtypes = [_dp, _dp, _dp, _dp, _dp]
        L.oracle_two_link_xdot.argtypes = [_dp, _dp, _dp]
        L.oracle_f_lin.argtypes = [C.c_int, C.c_int, C.c_double, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp]
        L.oracle_nlp_eval.argtypes = [C.c_int, C.c_int, C.c_double, _dp, _dp, _dp, _dp, _dp, _dp]
        L.oracle_reduced_gradient.argtypes = [C.c_int, C.c_int, C.c_double, _dp, _dp, _dp, _dp, _dp, _dp]
        L.oracle_solve_batch.argtypes = [
            C.c_int, C.c_int, C.c_int, C.c_double, C.c_int64, _dp, _dp, _dp, _dp, C.c_int64,
            C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.c_double, _dp, _ip, _ip, _dp, _dp, C.c_int,
        ]
        L.oracle_solve_batch.restype = C.c_int
        L.oracle_solve_batch_xb.argtypes = [
            C.c_int, C.c_int, C.c_int, C.c_double, C.c_int64, _dp, _dp, _dp, _dp, C.c_int64,
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.c_double, _dp, _ip, _ip, _dp,
            _dp, C.c_int,
        ]
        L.oracle_solve_batch_xb.restype = C.c_int
        L.oracle_synth_two_link.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int, C.c_double, _dp, _dp, _dp]
        L.oracle_synth_exo.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int, C.c_double, _dp, _dp, _dp]
        L.oracle_exo_jac.argtypes = [_dp, _dp, _dp, _dp, _dp]
        L.oracle_exo_mass.argtypes = [_dp, _dp]
        L.oracle_exo_hess.argtypes = [_dp, _dp, _dp, _dp]
        L.oracle_two_link_hess.argtypes = [_dp, _dp, _dp, _dp]
        L.oracle_set_hessian.argtypes = [C.c_int]
        L.oracle_set_kkt.argtypes = [C.c_int]
        L.oracle_set_bound_release.argtypes = [C.c_int]
        L.oracle_nlp_hess.argtypes = [C.c_int, C.c_int, C.c_double, _dp, _dp, _dp, _dp, C.c_double, C.c_void_p, _dp]
        L.oracle_nlp_hess.restype = C.c_int
        L.oracle_exact_fallbacks.argtypes = [C.c_int]
        L.oracle_exact_fallbacks.restype = C.c_longlong
        L.oracle_set_ip_rule.argtypes = [C.c_int]
        _lib = L
    return _lib


class UserModelHost:
    """Host build of an SX-generated device model (oracle/_user/<name>_host.so, from <name>_model.h)."""

    def __init__(self, name):
        path = os.path.join(USER_DIR, f"{name}_host.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} (run make -C mahi-mpc_amd/host user && make -C oracle user)")
        L = C.CDLL(path)
        dims = (C.c_int * 3)()
        L.user_model_dims(C.byref(dims, 0), C.byref(dims, 4), C.byref(dims, 8))
        self.nx, self.nu, self.nq = dims[0], dims[1], dims[2]
        self.na = self.nx - self.nq
        for f, n in (("user_model_eval", 3), ("user_model_eval_acc_jac", 6), ("user_model_jac", 5),
                     ("user_model_hess", 4)):
            getattr(L, f).restype = None
            getattr(L, f).argtypes = [C.c_void_p] * n
        self.L, self.name = L, name

    def eval(self, x, u):
        xd = np.zeros(self.nx)
        self.L.user_model_eval(c64(x).ctypes.data, c64(u).ctypes.data, xd.ctypes.data)
        return xd

    def jac(self, x, u):
        A = np.zeros(self.nx * self.nx); B = np.zeros(self.nx * self.nu); xd = np.zeros(self.nx)
        x, u = c64(x), c64(u)
        self.L.user_model_jac(x.ctypes.data, u.ctypes.data, A.ctypes.data, B.ctypes.data, xd.ctypes.data)
        return A.reshape(self.nx, self.nx), B.reshape(self.nx, self.nu), xd

    def hess(self, x, u, lam):
        """sum_r lam[r] d^2 f_r / d(x,u)^2 ((nx+nu)^2), lam over all nx rows"""
        K = self.nx + self.nu
        W = np.zeros(K * K)
        self.L.user_model_hess(c64(x).ctypes.data, c64(u).ctypes.data, c64(lam).ctypes.data, W.ctypes.data)
        return W.reshape(K, K)

    def acc_jac(self, x, u):
        na, nq, nu = self.na, self.nq, self.nu
        acc = np.zeros(na); Fq = np.zeros(max(1, na * nq)); Fqd = np.zeros(na * na); Fu = np.zeros(na * nu)
        x, u = c64(x), c64(u)
        self.L.user_model_eval_acc_jac(x.ctypes.data, u.ctypes.data, acc.ctypes.data, Fq.ctypes.data,
                                       Fqd.ctypes.data, Fu.ctypes.data)
        return acc, Fq[:na * nq].reshape(na, nq), Fqd.reshape(na, na), Fu.reshape(na, nu)


def use_user_model(name) -> int:
    """Register the host build of generated model `name` as the oracle's USER model; returns USER."""
    m = UserModelHost(name)
    fn = C.cast(m.L.user_model_jac, C.c_void_p).value
    lib().oracle_set_user_model.argtypes = [C.c_int, C.c_int, C.c_void_p]
    assert lib().oracle_set_user_model(m.nx, m.nu, fn) == 0
    lib().oracle_set_user_model_hess.argtypes = [C.c_void_p]
    assert lib().oracle_set_user_model_hess(C.cast(m.L.user_model_hess, C.c_void_p).value) == 0
    _user["active"] = m  # keep the library loaded
    DIMS[USER] = (m.nx, m.nu)
    return USER


def c64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def two_link_hess(x, u, lam):
    """sum_r lam_r d^2 f_r / d(x,u)^2 of the 2-link arm (6x6)"""
    W = np.zeros(36)
    lib().oracle_two_link_hess(c64(x), c64(u), c64(lam), W)
    return W.reshape(6, 6)


def two_link_jac(x, u):
    A = np.zeros(16); B = np.zeros(8); xd = np.zeros(4)
    lib().oracle_two_link_jac(c64(x), c64(u), A, B, xd)
    return A.reshape(4, 4), B.reshape(4, 2), xd


def exo_jac(x, u):
    A = np.zeros(64); B = np.zeros(32); xd = np.zeros(8)
    lib().oracle_exo_jac(c64(x), c64(u), A, B, xd)
    return A.reshape(8, 8), B.reshape(8, 4), xd


def exo_mass(q):
    M = np.zeros(16)
    lib().oracle_exo_mass(c64(q), M)
    return M.reshape(4, 4)


def f_lin(h, A, B, x, u, xdot_init, x_init, u_init):
    out = np.zeros(4)
    lib().oracle_f_lin(4, 2, h, c64(A).ravel(), c64(B).ravel(), c64(x), c64(u), c64(xdot_init),
                       c64(x_init), c64(u_init), out)
    return out


def nlp_eval(N, h, V, u_prev, traj, weights, model=TWO_LINK):
    nx, _ = DIMS[model]
    J = np.zeros(1); g = np.zeros(N * nx)
    lib().oracle_nlp_eval(model, N, h, c64(V), c64(u_prev), c64(traj).ravel(), c64(weights), J, g)
    return float(J[0]), g


def nlp_hess(N, h, V, u_prev, traj, weights, lam_f=1.0, lam_g=None, model=TWO_LINK):
    """nlp_hess_l stage blocks [N][K][K] of lam_f J + lam_g^T g at V"""
    nx, nu = DIMS[model]
    K = nx + nu
    out = np.zeros(N * K * K)
    lg = None if lam_g is None else c64(lam_g).reshape(-1)
    rc = lib().oracle_nlp_hess(model, N, h, c64(V).reshape(-1), c64(u_prev), c64(traj).reshape(-1), c64(weights),
                               float(lam_f), None if lg is None else lg.ctypes.data, out)
    if rc != 0:
        raise ValueError("model has no second derivatives")
    return out.reshape(N, K, K)


def reduced_gradient(N, h, x0, U, u_prev, traj, weights, model=TWO_LINK):
    _, nu = DIMS[model]
    g = np.zeros(N * nu)
    lib().oracle_reduced_gradient(model, N, h, c64(x0), c64(U).ravel(), c64(u_prev), c64(traj).ravel(),
                                  c64(weights), g)
    return g


def synth(seed, first, B, N, h, model=TWO_LINK):
    nx, nu = DIMS[model]
    x0 = np.zeros((B, nx)); up = np.zeros((B, nu)); tr = np.zeros((B, N, nx))
    fn = lib().oracle_synth_exo if model == EXO else lib().oracle_synth_two_link
    fn(seed, first, B, N, h, x0.reshape(-1), up.reshape(-1), tr.reshape(-1))
    return x0, up, tr


def solve_batch(N, h, x0, u_prev, traj, weights, V=None, u_lb=None, u_ub=None, max_iter=200,
                tol_grad=1e-8, tol_defect=1e-10, nthreads=0, is_linear=False, model=TWO_LINK, x_lb=None, x_ub=None,
                init_states=0, hessian=HESS_GAUSS_NEWTON, solver=None, kkt=KKT_DENSE, bound_release=False):
    """solver: the GPU mmpc.Solver being checked -- the oracle then runs the Hessian that solver resolves for this
    batch (mmpc_resolve_hessian: exact for unbounded 2-link / generated-model solves on the group kernel) and, with
    control bounds, that kernel's active-set rule (the 16-lane Riccati kernel also releases holds whose QP multiplier
    points into the box: bound_release).
    kkt: KKT_DENSE (default; explicit condensing) or KKT_RICCATI (the kernels' recursion; unbounded solves)."""
    if solver is not None:
        fin = lambda b: b is not None and bool((np.abs(np.asarray(b, dtype=np.float64)) < 1e19).any())  # noqa: E731
        B = int(np.asarray(x0).reshape(-1, DIMS[model][0]).shape[0])
        hessian = {1: HESS_GAUSS_NEWTON, 2: HESS_EXACT}[solver.hessian_for(B, fin(u_lb) or fin(u_ub))]
        bound_release = solver.kkt_solver_for(B) == 3
    lib().oracle_set_init_states(int(init_states))
    lib().oracle_set_hessian(int(hessian))
    lib().oracle_set_kkt(int(kkt))
    lib().oracle_set_bound_release(int(bool(bound_release)))
    try:
        return _solve_batch(N, h, x0, u_prev, traj, weights, V, u_lb, u_ub, max_iter, tol_grad, tol_defect, nthreads,
                            is_linear, model, x_lb, x_ub)
    finally:
        lib().oracle_set_init_states(0)
        lib().oracle_set_hessian(HESS_GAUSS_NEWTON)
        lib().oracle_set_kkt(KKT_DENSE)
        lib().oracle_set_bound_release(0)


def _solve_batch(N, h, x0, u_prev, traj, weights, V, u_lb, u_ub, max_iter, tol_grad, tol_defect, nthreads,
                 is_linear, model, x_lb, x_ub):
    NX, NU = DIMS[model]
    x0 = c64(x0).reshape(-1, NX)
    B = x0.shape[0]
    NV = NX * (N + 1) + NU * N
    weights = c64(weights)
    w_stride = 0 if weights.ndim == 1 else weights.shape[1]
    V = np.zeros((B, NV)) if V is None else c64(V).reshape(B, NV).copy()
    st = np.zeros(B, np.int32); it = np.zeros(B, np.int32); kkt = np.zeros(B); J = np.zeros(B)
    lb = None if u_lb is None else c64(u_lb)
    ub = None if u_ub is None else c64(u_ub)
    xl = None if x_lb is None else c64(x_lb)
    xu = None if x_ub is None else c64(x_ub)
    ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    rc = lib().oracle_solve_batch_xb(
        model, int(is_linear), N, h, B, x0.reshape(-1), c64(u_prev).reshape(-1), c64(traj).reshape(-1), weights.reshape(-1),
        w_stride, ptr(lb), ptr(ub), ptr(xl), ptr(xu), max_iter, tol_grad, tol_defect, V.reshape(-1), st, it, kkt, J,
        nthreads)
    assert rc == 0
    return dict(V=V, status=st, iters=it, kkt=kkt, J=J)


def exact_fallbacks(reset=True) -> int:
    """exact-Hessian iterations of the oracle whose QP was not positive definite and took the Gauss-Newton step, since
    the last reset (instrumentation for the tests that exercise that path)"""
    return int(lib().oracle_exact_fallbacks(1 if reset else 0))


def set_ip_rule(rule: int) -> None:
    """barrier rule of the oracle's interior-point solve: 0 = IPOPT's monotone rule (the kernels'), 1 = Mehrotra
    predictor-corrector, 2 = Mehrotra's probing without the corrector term (round-5 experiment)"""
    lib().oracle_set_ip_rule(int(rule))
