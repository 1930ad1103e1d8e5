"""Python binding of the mmpc C-ABI (include/mmpc.h) -- MI355X batched nonlinear MPC.

This is a thin ctypes layer over ``lib/libmmpc.so``; every compute call runs the HIP
kernels on the GPU.  There is no CPU fallback: if the library or a GPU is missing the
calls raise ``MmpcError``.

Reference mapping (mahi-mpc):
  Solver(...)            ~ ModelControl::load_model      (src/Mahi/Mpc/ModelControl.cpp:21-73)
  Solver.solve_batch*    ~ m_solver(m_solver_args)       (src/Mahi/Mpc/ModelControl.cpp:159), batched
  Solver.linearize*      ~ <name>_get_A/_get_B/_get_x_dot_init externals (ModelGenerator.cpp:51-53)
  write_model_json       ~ ModelGenerator::save_param_file (ModelGenerator.cpp:261-270)
"""
from __future__ import annotations

import ctypes as C
import json
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                      # mahi-mpc_amd/
REPO = os.path.dirname(ROOT)
LIB_PATH = os.environ.get("MMPC_LIB_PATH") or os.path.join(ROOT, "lib", "libmmpc.so")
HEADER_PATH = os.path.join(REPO, "include", "mmpc.h")

OK = 0
STATUS = {0: "converged", 1: "max_iter", 2: "linesearch_failed", 3: "nonfinite",
          4: "factorization_failed", 5: "bounds_violated"}
STATUS_CONVERGED, STATUS_MAX_ITER, STATUS_LINESEARCH_FAILED = 0, 1, 2
STATUS_NONFINITE, STATUS_FACTORIZATION_FAILED, STATUS_BOUNDS_VIOLATED = 3, 4, 5
ERR = {-1: "invalid_arg", -2: "io", -3: "parse", -4: "unsupported", -5: "hip", -6: "no_device"}


class MmpcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"mmpc error {code} ({ERR.get(code, '?')}): {msg}")
        self.code = code


KKT_AUTO, KKT_CONDENSED, KKT_RICCATI, KKT_RICCATI_GROUP = 0, 1, 2, 3
INIT_AS_GIVEN, INIT_HOLD_X0, INIT_ZERO = 0, 1, 2
HESSIAN_AUTO, HESSIAN_GAUSS_NEWTON, HESSIAN_EXACT = 0, 1, 2
MODEL_TWO_LINK_ARM, MODEL_EXO_ARM, MODEL_USER = 0, 1, 2
USER_LIB_DIR = os.path.join(ROOT, "lib", "user")
BUILTIN_MODELS = ("two_link_arm", "double_pendulum", "exo_arm", "exo")  # "mmpc_model" names libmmpc.so serves   # models generated from SX by ModelGenerator (make -C host user)


class Opts(C.Structure):
    _fields_ = [("max_iter", C.c_int32), ("device", C.c_int32), ("tol_grad", C.c_double),
                ("tol_defect", C.c_double), ("kkt_solver", C.c_int32), ("factor_fp32", C.c_int32),
                ("init_states", C.c_int32), ("hessian", C.c_int32), ("tail_cap", C.c_int32),
                ("tail_wave_max", C.c_int32), ("tail_rounds", C.c_int32)]


class ModelInfo(C.Structure):
    _fields_ = [("name", C.c_char * 128), ("model_id", C.c_int32), ("num_x", C.c_int32), ("num_u", C.c_int32),
                ("num_shooting_nodes", C.c_int32), ("num_v", C.c_int32), ("num_g", C.c_int32),
                ("is_linear", C.c_int32), ("step_size", C.c_double), ("timespan_us", C.c_int64),
                ("step_size_us", C.c_int64), ("u_min", C.c_double * 16), ("u_max", C.c_double * 16),
                ("x_min", C.c_double * 16), ("x_max", C.c_double * 16)]


_libs = {}
_vp = C.c_void_p


def build(force: bool = False) -> str:
    """Compile lib/libmmpc.so for gfx950 with hipcc (make -C mahi-mpc_amd)."""
    import subprocess
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", ROOT], check=True)
    return LIB_PATH


def header_functions(path: str = HEADER_PATH):
    """Names of every function declared in include/mmpc.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mmpc_\w+)\s*\(", text)))


def lib(path: str | None = None):
    """The C-ABI library: libmmpc.so (built-in models) or a model's generated <name>.so (same ABI)."""
    path = os.path.abspath(path or LIB_PATH)
    if path not in _libs:
        if not os.path.exists(path):
            raise MmpcError(-2, f"{path} not built (run make -C mahi-mpc_amd)")
        # PyTorch-ROCm ships its own HIP runtime: if libmmpc's initialises first, torch later sees no GPU
        # (observed on the MI355X box), so torch -- when present -- initialises before the library is loaded
        try:
            import torch
            torch.cuda.is_available()
        except ImportError:
            pass
        L = C.CDLL(path)  # RTLD_LOCAL: each model library keeps its own kernels (linked with -Bsymbolic)
        L.mmpc_abi_version.restype = C.c_int
        L.mmpc_default_opts.argtypes = [C.POINTER(Opts)]
        L.mmpc_create.argtypes = [C.c_char_p, C.POINTER(Opts), C.POINTER(_vp)]
        L.mmpc_create_from_json.argtypes = [C.c_char_p, C.POINTER(Opts), C.POINTER(_vp)]
        L.mmpc_destroy.argtypes = [_vp]
        L.mmpc_get_model_info.argtypes = [_vp, C.POINTER(ModelInfo)]
        L.mmpc_set_opts.argtypes = [_vp, C.POINTER(Opts)]
        L.mmpc_reserve_workspace.argtypes = [_vp, C.c_int64, C.POINTER(C.c_uint64)]
        L.mmpc_solve_batch.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64] + [_vp] * 7
        L.mmpc_solve_batch_host.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64] + [_vp] * 6
        L.mmpc_solve_batch_u0.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64] + [_vp] * 8
        L.mmpc_host_alloc.argtypes = [C.c_uint64, C.POINTER(_vp)]
        L.mmpc_host_free.argtypes = [_vp]
        L.mmpc_linearize_batch.argtypes = [_vp, C.c_int64] + [_vp] * 6
        L.mmpc_linearize_batch_host.argtypes = [_vp, C.c_int64] + [_vp] * 5
        L.mmpc_nlp_eval_batch.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64] + [_vp] * 3
        L.mmpc_synth_batch.argtypes = [_vp, C.c_uint64, C.c_int64, C.c_int64] + [_vp] * 4
        L.mmpc_nlp_derivs_batch.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64] + [_vp] * 4
        L.mmpc_nlp_hess_batch.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64, C.c_double, _vp, _vp, _vp]
        L.mmpc_shard.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.mmpc_multi_create.argtypes = [C.c_char_p, C.POINTER(Opts), C.POINTER(C.c_int32), C.c_int32, C.POINTER(_vp)]
        L.mmpc_multi_destroy.argtypes = [_vp]
        L.mmpc_multi_num_devices.argtypes = [_vp, C.POINTER(C.c_int32)]
        L.mmpc_multi_handle.argtypes = [_vp, C.c_int32, C.POINTER(_vp)]
        L.mmpc_multi_solve_batch_host.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64] + [_vp] * 6
        L.mmpc_multi_solve_batch_rccl.argtypes = [_vp, C.c_int64] + [_vp] * 4 + [C.c_int64] + [_vp] * 7
        L.mmpc_rccl_version.argtypes = [C.POINTER(C.c_int32)]
        L.mmpc_resolve_kkt_solver.argtypes = [_vp, C.c_int64, C.POINTER(C.c_int32)]
        L.mmpc_resolve_hessian.argtypes = [_vp, C.c_int64, C.c_int32, C.POINTER(C.c_int32)]
        L.mmpc_set_state_bounds.argtypes = [_vp, _vp, _vp]
        L.mmpc_get_state_bounds.argtypes = [_vp, _vp, _vp]
        L.mmpc_status_string.argtypes = [C.c_int32]
        L.mmpc_status_string.restype = C.c_char_p
        L.mmpc_last_error.restype = C.c_char_p
        _libs[path] = L
    return _libs[path]


def model_library(model_json: str) -> str:
    """Library serving the model of <name>.json: for a model generated from SX expressions ("mmpc_model" naming
    no built-in model) its dll_filepath, resolved against the JSON's directory as ModelControl does; else
    libmmpc.so (built-in models, and reference-written JSONs whose dll_filepath is a CasADi NLP library)."""
    try:
        with open(model_json) as fh:
            m = json.load(fh)
    except (OSError, ValueError):
        return LIB_PATH  # mmpc_create reports the I/O or parse error
    m = m.get("model", m) if isinstance(m, dict) else {}
    dll = m.get("dll_filepath") or ""
    if m.get("mmpc_model") in (None, *BUILTIN_MODELS) or not dll or os.path.basename(dll) == "libmmpc.so":
        return LIB_PATH
    cands = [dll] if os.path.isabs(dll) else [os.path.join(os.path.dirname(os.path.abspath(model_json)), dll), dll]
    for c in cands:
        if os.path.exists(c):
            return os.path.abspath(c)
    raise MmpcError(-2, f"model library {dll} of {model_json} not found")


def _check(rc, L=None):
    if rc != OK:
        raise MmpcError(rc, (L or lib()).mmpc_last_error().decode())


def default_opts() -> Opts:
    o = Opts()
    lib().mmpc_default_opts(C.byref(o))
    return o


def write_model_json(path, name, num_x, num_u, step_size_us, num_shooting_nodes, is_linear=False,
                     u_min=None, u_max=None, x_min=None, x_max=None, dll_filepath="", extra=None, model=None):
    """Write <name>.json exactly as ModelGenerator::save_param_file does (ModelParameters.cpp:37-50),
    including the +-10e30 defaults of the ModelParameters constructor (ModelParameters.cpp:14-24).
    ``model`` ("two_link_arm" / "exo_arm") adds the "mmpc_model" key naming the built-in dynamics."""
    def dflt(v, n, s):
        return list(v) if v is not None else [s * 10e30] * n
    m = {"name": name, "timespan": int(step_size_us) * int(num_shooting_nodes), "step_size": int(step_size_us),
         "num_x": num_x, "num_u": num_u, "num_shooting_nodes": num_shooting_nodes,
         "x_min": dflt(x_min, num_x, -1), "u_min": dflt(u_min, num_u, -1),
         "x_max": dflt(x_max, num_x, 1), "u_max": dflt(u_max, num_u, 1),
         "dll_filepath": dll_filepath, "is_linear": bool(is_linear)}
    if model:
        m["mmpc_model"] = model
    if extra:
        m.update(extra)
    with open(path, "w") as fh:
        json.dump({"model": m}, fh)
    return path


def _ptr(a):
    """device/host pointer of a torch tensor, numpy array, int address or None."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    if isinstance(a, np.ndarray):
        assert a.flags.c_contiguous
        return a.ctypes.data
    raise TypeError(type(a))


class HostBuffer:
    """Pinned host memory mapped into the devices' address space (mmpc_host_alloc): a solve kernel stores its
    per-tick results (u_0*, status, iters) straight into it -- on the host once the stream has completed.
    ``view(offset, dtype, count)`` gives numpy views; pass them (or their addresses) as solve outputs."""

    def __init__(self, nbytes: int, path: str | None = None):
        self._L = lib(path)
        p = _vp()
        rc = self._L.mmpc_host_alloc(int(nbytes), C.byref(p))
        if rc != 0:
            raise MmpcError(rc, self._L.mmpc_last_error().decode())
        self.ptr = p.value or 0
        self.nbytes = int(nbytes)
        self._buf = (C.c_char * self.nbytes).from_address(self.ptr) if self.nbytes else None
        if self.nbytes:   # hipHostMalloc does not zero: rows a ragged shard never writes must compare equal
            C.memset(self.ptr, 0, self.nbytes)

    def view(self, offset: int, dtype, count: int) -> np.ndarray:
        dt = np.dtype(dtype)
        assert offset % dt.itemsize == 0 and offset + count * dt.itemsize <= self.nbytes
        return np.frombuffer(self._buf, dtype=dt, count=count, offset=offset)

    def close(self):
        if self.ptr:
            self._buf = None
            self._L.mmpc_host_free(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


class Solver:
    """One loaded model (the reference's ModelControl without the thread/bookkeeping)."""

    def __init__(self, model_json=None, json_text=None, max_iter=None, tol_grad=None, tol_defect=None,
                 device=None, kkt_solver=None, factor_fp32=None, library=None, init_states=None, hessian=None,
                 tail_cap=None, tail_wave_max=None, tail_rounds=None):
        self._L = L = lib(library or (model_library(model_json) if model_json is not None else None))
        o = Opts()
        L.mmpc_default_opts(C.byref(o))
        if kkt_solver is not None:
            o.kkt_solver = kkt_solver
        if factor_fp32 is not None:
            o.factor_fp32 = int(factor_fp32)
        if init_states is not None:
            o.init_states = int(init_states)
        if hessian is not None:
            o.hessian = int(hessian)
        if tail_cap is not None:      # the lane solver's iteration-tail hand-over (ABI 6; -1 = default, 0 = off)
            o.tail_cap = int(tail_cap)
        if tail_wave_max is not None:
            o.tail_wave_max = int(tail_wave_max)
        if tail_rounds is not None:
            o.tail_rounds = int(tail_rounds)
        if max_iter is not None:
            o.max_iter = max_iter
        if tol_grad is not None:
            o.tol_grad = tol_grad
        if tol_defect is not None:
            o.tol_defect = tol_defect
        if device is not None:
            o.device = device
        h = _vp()
        if json_text is not None:
            self._check(L.mmpc_create_from_json(json_text.encode(), C.byref(o), C.byref(h)))
        else:
            self._check(L.mmpc_create(os.fsencode(model_json), C.byref(o), C.byref(h)))
        self._h = h
        info = ModelInfo()
        self._check(L.mmpc_get_model_info(h, C.byref(info)))
        self.info = info
        self.nx, self.nu, self.N = info.num_x, info.num_u, info.num_shooting_nodes
        self.NV = info.num_v
        self.h = info.step_size

    def _check(self, rc):
        _check(rc, self._L)

    def reserve_workspace(self, B) -> int:
        """Pre-allocate the Riccati solver workspace for up to B instances; returns its size in bytes."""
        n = C.c_uint64(0)
        self._check(self._L.mmpc_reserve_workspace(self._h, B, C.byref(n)))
        return int(n.value)

    def close(self):
        if getattr(self, "_h", None):
            self._L.mmpc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- device-pointer API (torch tensors on the GPU or raw addresses) ----
    def solve_batch(self, B, x0, u_prev, traj, weights, V, status=None, iters=None, kkt=None,
                    weights_stride=0, u_lb=None, u_ub=None, stream=None, u0=None):
        """Device-pointer solve (stream-ordered).  u0: optional [B][nu] output of u_0* (mmpc_solve_batch_u0);
        u0 / status / iters may be HostBuffer views (results stored by the kernel straight into host memory)."""
        if u0 is None:
            self._check(self._L.mmpc_solve_batch(self._h, B, _ptr(x0), _ptr(u_prev), _ptr(traj), _ptr(weights),
                                                 weights_stride, _ptr(u_lb), _ptr(u_ub), _ptr(V), _ptr(status),
                                                 _ptr(iters), _ptr(kkt), stream))
        else:
            self._check(self._L.mmpc_solve_batch_u0(self._h, B, _ptr(x0), _ptr(u_prev), _ptr(traj), _ptr(weights),
                                                    weights_stride, _ptr(u_lb), _ptr(u_ub), _ptr(V), _ptr(status),
                                                    _ptr(iters), _ptr(kkt), _ptr(u0), stream))

    def synth(self, seed, first_index, B, x0, u_prev, traj, stream=None):
        self._check(self._L.mmpc_synth_batch(self._h, seed, first_index, B, _ptr(x0), _ptr(u_prev), _ptr(traj), stream))

    def nlp_eval(self, B, V, u_prev, traj, weights, J, defect_inf, weights_stride=0, stream=None):
        self._check(self._L.mmpc_nlp_eval_batch(self._h, B, _ptr(V), _ptr(u_prev), _ptr(traj), _ptr(weights),
                                         weights_stride, _ptr(J), _ptr(defect_inf), stream))

    def nlp_derivs(self, B, V, u_prev, traj, weights, J=None, grad=None, jac_blocks=None, weights_stride=0,
                   stream=None):
        """J, dJ/dV and the defect-Jacobian stage blocks at V (device pointers; nlp_grad_f / nlp_jac_g)."""
        self._check(self._L.mmpc_nlp_derivs_batch(self._h, B, _ptr(V), _ptr(u_prev), _ptr(traj), _ptr(weights),
                                                  weights_stride, _ptr(J), _ptr(grad), _ptr(jac_blocks), stream))

    def nlp_hess(self, B, V, u_prev, traj, weights, lam_f, lam_g, blocks, weights_stride=0, stream=None):
        """nlp_hess_l stage blocks [B][N][K][K] of lam_f J + lam_g^T g at V (device pointers)."""
        self._check(self._L.mmpc_nlp_hess_batch(self._h, B, _ptr(V), _ptr(u_prev), _ptr(traj), _ptr(weights),
                                                weights_stride, float(lam_f), _ptr(lam_g), _ptr(blocks), stream))

    def linearize(self, B, x, u, A, Bm, xdot, stream=None):
        self._check(self._L.mmpc_linearize_batch(self._h, B, _ptr(x), _ptr(u), _ptr(A), _ptr(Bm), _ptr(xdot), stream))

    # ---- host (numpy) API, synchronous ----
    def solve_batch_host(self, x0, u_prev, traj, weights, V=None, u_lb=None, u_ub=None):
        nx, nu, N, NV = self.nx, self.nu, self.N, self.NV
        x0 = _f64(x0, (-1, nx))
        B = x0.shape[0]
        u_prev = _f64(u_prev, (B, nu))
        traj = _f64(traj, (B, N, nx))
        weights = _f64(weights)
        ws = 0 if weights.ndim == 1 else weights.shape[-1]
        V = np.zeros((B, NV)) if V is None else _f64(V, (B, NV)).copy()
        st = np.zeros(B, np.int32)
        it = np.zeros(B, np.int32)
        kkt = np.zeros(B)
        lb = None if u_lb is None else _f64(u_lb)
        ub = None if u_ub is None else _f64(u_ub)
        self._check(self._L.mmpc_solve_batch_host(self._h, B, _ptr(x0), _ptr(u_prev), _ptr(traj), _ptr(weights), ws,
                                           _ptr(lb), _ptr(ub), _ptr(V), _ptr(st), _ptr(it), _ptr(kkt)))
        return dict(V=V, status=st, iters=it, kkt=kkt)

    def set_state_bounds(self, x_lb=None, x_ub=None):
        """x_lb <= x_k <= x_ub for k = 1..N (None = unbounded); finite bounds select the interior-point variant."""
        lb = None if x_lb is None else _f64(x_lb, (self.nx,))
        ub = None if x_ub is None else _f64(x_ub, (self.nx,))
        self._check(self._L.mmpc_set_state_bounds(self._h, _ptr(lb), _ptr(ub)))

    def state_bounds(self):
        lb, ub = np.zeros(self.nx), np.zeros(self.nx)
        self._check(self._L.mmpc_get_state_bounds(self._h, _ptr(lb), _ptr(ub)))
        return lb, ub

    def kkt_solver_for(self, B: int) -> int:
        """KKT_* solver a solve of B instances runs (the AUTO choice resolved)."""
        v = C.c_int32()
        self._check(self._L.mmpc_resolve_kkt_solver(self._h, B, C.byref(v)))
        return v.value

    def hessian_for(self, B: int, u_bounded: bool = False) -> int:
        """HESSIAN_GAUSS_NEWTON or HESSIAN_EXACT: what a solve of B instances runs (the AUTO choice resolved)."""
        v = C.c_int32()
        self._check(self._L.mmpc_resolve_hessian(self._h, B, int(bool(u_bounded)), C.byref(v)))
        return v.value

    def linearize_host(self, x, u):
        nx, nu = self.nx, self.nu
        x = _f64(x, (-1, nx))
        B = x.shape[0]
        u = _f64(u, (B, nu))
        A = np.zeros((B, nx * nx)); Bm = np.zeros((B, nx * nu)); xd = np.zeros((B, nx))
        self._check(self._L.mmpc_linearize_batch_host(self._h, B, _ptr(x), _ptr(u), _ptr(A), _ptr(Bm), _ptr(xd)))
        # column-major per instance (CasADi DM order) -> (B, nx, nx) row-major views
        return (A.reshape(B, nx, nx).transpose(0, 2, 1), Bm.reshape(B, nu, nx).transpose(0, 2, 1), xd)


def shard(B: int, n: int, i: int) -> tuple:
    """(first, count) of shard i of B instances over n shards (mmpc_shard; the C-ABI's partition)."""
    f, c = C.c_int64(), C.c_int64()
    _check(lib().mmpc_shard(B, n, i, C.byref(f), C.byref(c)))
    return f.value, c.value


class MultiSolver:
    """One process over several devices (mmpc_multi_*): contiguous shards, one handle and stream per device."""

    def __init__(self, model_json, devices, **opts):
        self._L = L = lib(model_library(model_json))
        o = Opts()
        L.mmpc_default_opts(C.byref(o))
        for k, v in opts.items():
            setattr(o, k, v)
        devs = (C.c_int32 * len(devices))(*devices)
        m = _vp()
        _check(L.mmpc_multi_create(os.fsencode(model_json), C.byref(o), devs, len(devices), C.byref(m)), L)
        self._m = m
        info = ModelInfo()
        h = _vp()
        _check(L.mmpc_multi_handle(m, 0, C.byref(h)), L)
        _check(L.mmpc_get_model_info(h, C.byref(info)), L)
        self.nx, self.nu, self.N, self.NV = info.num_x, info.num_u, info.num_shooting_nodes, info.num_v

    def num_devices(self) -> int:
        n = C.c_int32()
        _check(self._L.mmpc_multi_num_devices(self._m, C.byref(n)), self._L)
        return n.value

    def solve_batch_host(self, x0, u_prev, traj, weights, V=None, u_lb=None, u_ub=None):
        nx, nu, N, NV = self.nx, self.nu, self.N, self.NV
        x0 = _f64(x0, (-1, nx))
        B = x0.shape[0]
        u_prev, traj, weights = _f64(u_prev, (B, nu)), _f64(traj, (B, N, nx)), _f64(weights)
        ws = 0 if weights.ndim == 1 else weights.shape[-1]
        V = np.zeros((B, NV)) if V is None else _f64(V, (B, NV)).copy()
        st, it, kkt = np.zeros(B, np.int32), np.zeros(B, np.int32), np.zeros(B)
        lb = None if u_lb is None else _f64(u_lb)
        ub = None if u_ub is None else _f64(u_ub)
        _check(self._L.mmpc_multi_solve_batch_host(self._m, B, _ptr(x0), _ptr(u_prev), _ptr(traj), _ptr(weights), ws,
                                                   _ptr(lb), _ptr(ub), _ptr(V), _ptr(st), _ptr(it), _ptr(kkt)), self._L)
        return dict(V=V, status=st, iters=it, kkt=kkt)

    def solve_batch_rccl(self, x0, u_prev, traj, weights, V, status=None, iters=None, kkt=None, u_lb=None,
                         u_ub=None, weights_stride=None, stream=None):
        """mmpc_multi_solve_batch_rccl: torch tensors on the FIRST device of the handle (fp64, contiguous; weights
        [nx+2nu] shared or [B][nx+2nu], or a flat buffer with an explicit weights_stride); V is updated in place,
        status / iters (int32) / kkt filled if given.  stream: the hipStream_t (int) the inputs were produced on --
        default torch's current stream of x0's device."""
        B = x0.shape[0]
        ws = (0 if weights.dim() == 1 else weights.shape[-1]) if weights_stride is None else int(weights_stride)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(x0.device).cuda_stream
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        _check(self._L.mmpc_multi_solve_batch_rccl(self._m, B, p(x0), p(u_prev), p(traj), p(weights), ws, p(u_lb),
                                                   p(u_ub), p(V), p(status), p(iters), p(kkt),
                                                   C.c_void_p(stream) if stream else None), self._L)

    def close(self):
        if getattr(self, "_m", None):
            self._L.mmpc_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rccl_version() -> int:
    """ncclGetVersion of the RCCL the multi-device RCCL path loads (mmpc_rccl_version), e.g. 22606; 0 if none"""
    v = C.c_int32()
    return v.value if lib().mmpc_rccl_version(C.byref(v)) == OK else 0


def flops_per_iteration(N: int, nx: int = 4, nu: int = 2) -> dict:
    """Algorithmic flop count of ONE SQP iteration of the HIP kernel (mul+add = 2), counted from
    sqp_wave.h phase by phase (structure-exploiting: no flop on structural zeros).  See DESIGN.md."""
    M = N * nu
    f = {}
    f["defect_recursion"] = N * (2 * nx * nx + 2 * nx)          # d_{k+1} = A d + c ; e
    f["adjoint"] = (N - 1) * (2 * nx * nx + 2 * nx)             # lam recursion
    f["gradient"] = M * (2 * nx + 8)
    f["lyapunov"] = N * (4 * nx ** 3 + 2 * nu * nx * nx)        # P A, A^T (PA), Z = B^T P
    # H rows: lower part sum over rows of (i+1) steps, upper part (N-1-i) steps; each step = vector x A
    # (2 nx^2) plus nu outputs (2 nx each)
    steps = sum((i + 1) + (N - 1 - i) for i in range(N)) * nu
    f["hessian"] = steps * (2 * nx * nx + 2 * nu * nx)
    f["gauss_jordan"] = sum(2 * (M - 1) * (M - k) for k in range(M)) + M  # rows x remaining cols, + rhs
    f["dx_recursion"] = N * (2 * nx * nx + 2 * nu * nx + nx)
    f["merit"] = N * (2 * nx * (nx + nu) + 12)
    f["total"] = sum(f.values())
    return f


def riccati_flops_per_iteration(N: int, nx: int = 8, nu: int = 4, exact: bool = False) -> dict:
    """Algorithmic flop count (mul+add = 2) of ONE SQP iteration of the lane-per-instance Riccati kernel
    (sqp_lane.h), structure-exploiting for second-order models (A = [[I, hI],[hFq, I+hFqd]],
    B = [[0],[hFu]], nq = nx/2).  Model evaluations are excluded (SURVEY.md 8d counts them separately)."""
    nq, ns = nx // 2, nx + nu
    at_mul = 2 * nq * nx + 2 * nx            # A^T v or A v with the block structure
    f = {}
    f["defect_recursion"] = N * (at_mul + nx)
    f["adjoint_gradient"] = N * (at_mul + 2 * nq * nu + 6 * nu)
    st = 0
    st += nx * nu * 2 * nq                    # G = P_xx B + P_xu
    st += 2 * nx * nx                         # mv = P_xx c + p_x
    st += nu * (nu + 1) // 2 * 4 * nq         # H_ww
    st += nu * (2 * nq + 2 * nx + 4)          # h_w
    st += nu * at_mul                         # H_wx = (A^T G)^T
    st += nx * (nx * (2 * nq + 2) + at_mul)   # A^T P_xx A by columns
    st += at_mul + 2 * nx                     # p_x
    st += nu ** 3 // 3 + nu * nu * (ns + 1)   # Cholesky + forward solve
    st += nu * nu * (ns + 1)                  # back solve (K)
    st += ns * (ns + 1) // 2 * 2 * nu + ns * 2 * nu  # P~ = ... - Y^T Y, p~
    f["riccati"] = N * st
    if exact:   # the stage Hessian W_k enters P~_xx, H_ww and H_wx (its evaluation is a model evaluation: excluded)
        f["riccati"] += N * (nx * nx + nu * nu + nx * nu)
    f["step_recursion"] = N * (2 * nu * ns + at_mul + 2 * nq * nu + nx)
    f["merit"] = N * (4 * nx + 8 * nu)
    f["total"] = sum(f.values())
    return f


def survey_flops_per_iteration(N: int, nx: int = 4, nu: int = 2) -> int:
    """SURVEY.md 8(d) reference count (explicit Gamma + block-triangular G^T Q G + Cholesky)."""
    M, S = N * nu, N * nx
    return int(N * (N - 1) / 2 * 2 * nx * nx * nu + N * (N + 1) * (N + 2) / 6 * 2 * nu * nu * nx
               + M ** 3 / 3 + 4 * M * M + 2 * S * M + N * (nx * nx + nx * nu))
