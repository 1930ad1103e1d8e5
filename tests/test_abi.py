"""CPU: the C-ABI library loads, exports every function include/mmpc.h declares, and its host-only
logic (model-file loading per ModelParameters.cpp:52-72, option validation, error reporting) works
without a GPU.  No compute entry point is called here."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest


def test_library_exports_every_header_symbol(mmpc_mod):
    L = mmpc_mod.lib()
    names = mmpc_mod.header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), f"libmmpc.so does not export {n}"
    # and the exported dynamic symbol table says the same (no C++ mangling on the ABI)
    out = subprocess.run(["nm", "-D", "--defined-only", mmpc_mod.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert set(names) <= exported


def test_library_is_gfx950_code_object(mmpc_mod):
    """the fat binary carries a gfx950 (MI355X) code object and nothing else"""
    data = open(mmpc_mod.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_abi_version_and_defaults(mmpc_mod):
    assert mmpc_mod.lib().mmpc_abi_version() == 6
    o = mmpc_mod.default_opts()
    assert o.max_iter == 200 and o.device == -1   # ipopt.max_iter, ModelControl.cpp:55
    assert o.tol_grad == 1e-8 and o.tol_defect == 1e-10
    assert o.kkt_solver == mmpc_mod.KKT_AUTO
    assert o.hessian == mmpc_mod.HESSIAN_AUTO
    assert (o.tail_cap, o.tail_wave_max, o.tail_rounds) == (-1, -1, -1)   # the hand-over's default policy (ABI 6)


@pytest.mark.parametrize("field,bad", [("tail_cap", -2), ("tail_cap", 1000), ("tail_wave_max", 65),
                                       ("tail_wave_max", -2), ("tail_rounds", 0), ("tail_rounds", -3)])
def test_tail_opts_validated(field, bad, model_json, mmpc_mod):
    o = mmpc_mod.default_opts()
    setattr(o, field, bad)
    h = C.c_void_p()
    L = mmpc_mod.lib()
    assert L.mmpc_create(model_json(N=30).encode(), C.byref(o), C.byref(h)) == -1   # MMPC_ERR_INVALID_ARG
    assert field in L.mmpc_last_error().decode()


def test_load_model_json_like_reference(model_json, mmpc_mod):
    s = mmpc_mod.Solver(model_json(N=30, h_us=2000))
    i = s.info
    assert i.name == b"nonlinear_double_pendulum"
    assert (i.num_x, i.num_u, i.num_shooting_nodes) == (4, 2, 30)
    assert i.num_v == 4 * 31 + 2 * 30 == 184 and i.num_g == 120
    assert i.step_size == pytest.approx(0.002) and i.step_size_us == 2000 and i.timespan_us == 60000
    assert i.is_linear == 0 and i.model_id == 0
    # ModelParameters.cpp:66-69: x bounds of exactly +-10e30 become +-inf; u bounds stay +-10e30
    assert all(i.x_min[k] == float("-inf") and i.x_max[k] == float("inf") for k in range(4))
    assert all(i.u_min[k] == -10e30 and i.u_max[k] == 10e30 for k in range(2))
    s.close()


def test_load_model_null_bounds_and_linear(tmp_path, mmpc_mod):
    # nlohmann writes +-inf as null; ex_model_generate.cpp:48-53 style bounds
    m = {"model": {"name": "linear_double_pendulum", "timespan": 50000, "step_size": 2000, "num_x": 4,
                   "num_u": 2, "num_shooting_nodes": 25, "x_min": [None] * 4, "u_min": [None] * 2,
                   "x_max": [None] * 4, "u_max": [None] * 2, "dll_filepath": "x.so", "is_linear": True}}
    p = tmp_path / "lin.json"
    p.write_text(json.dumps(m))
    s = mmpc_mod.Solver(str(p))
    assert s.info.is_linear == 1 and s.N == 25
    assert s.info.x_min[0] == float("-inf") and s.info.u_max[1] == 10e30


@pytest.mark.parametrize("text,code", [
    ("{", -3),
    ('{"model": {"name": "x"}}', -3),
    ('{"model": {"name": "x", "num_x": 6, "num_u": 3, "num_shooting_nodes": 50, "step_size": 2000}}', -4),
    ('{"model": {"name": "x", "num_x": 4, "num_u": 2, "num_shooting_nodes": 10, "step_size": 2000,'
     ' "mmpc_model": "exo_arm"}}', -3),
    ('{"model": {"name": "x", "num_x": 4, "num_u": 2, "num_shooting_nodes": 10, "step_size": 2000,'
     ' "mmpc_model": "nope"}}', -4),
    ('{"model": {"name": "x", "num_x": 4, "num_u": 2, "num_shooting_nodes": 10, "step_size": 2000,'
     ' "u_min": [1, 2, 3]}}', -3),
])
def test_bad_model_files_are_api_errors(text, code, mmpc_mod):
    with pytest.raises(mmpc_mod.MmpcError) as ei:
        mmpc_mod.Solver(json_text=text)
    assert ei.value.code == code
    assert mmpc_mod.lib().mmpc_last_error().decode() != ""


def test_missing_file_is_io_error(mmpc_mod, tmp_path):
    with pytest.raises(mmpc_mod.MmpcError) as ei:
        mmpc_mod.Solver(str(tmp_path / "nope.json"))
    assert ei.value.code == -2


def test_load_exo_model(tmp_path, mmpc_mod):
    # SURVEY.md 8a A3b / 8d cfg#3: nx=8 nu=4 N=50 resolves to the built-in exo by its dimensions
    p = mmpc_mod.write_model_json(str(tmp_path / "exo.json"), "exo", 8, 4, 2000, 50)
    s = mmpc_mod.Solver(p)
    assert s.info.model_id == mmpc_mod.MODEL_EXO_ARM and s.NV == 8 * 51 + 4 * 50 == 608
    s.close()
    p = mmpc_mod.write_model_json(str(tmp_path / "exo2.json"), "exo2", 8, 4, 2000, 50, model="exo_arm")
    assert mmpc_mod.Solver(p).info.model_id == mmpc_mod.MODEL_EXO_ARM


def test_workspace_size_and_solver_choice(tmp_path, model_json, mmpc_mod):
    # B = 0: size query only (no device needed); an unknown kkt_solver is rejected at creation
    p = mmpc_mod.write_model_json(str(tmp_path / "exo.json"), "exo", 8, 4, 2000, 50)
    s = mmpc_mod.Solver(p)
    assert s.reserve_workspace(0) == 0
    with pytest.raises(mmpc_mod.MmpcError):
        s.reserve_workspace(-1)
    with pytest.raises(mmpc_mod.MmpcError):
        mmpc_mod.Solver(p, kkt_solver=7)


def test_auto_solver_policy(tmp_path, model_json, mmpc_mod):
    """MMPC_KKT_AUTO (include/mmpc.h), resolved without a GPU"""
    m = mmpc_mod
    s = m.Solver(model_json(N=30))                              # cfg#2 shape (exact Hessian: the group kernel)
    assert s.kkt_solver_for(4096) == m.KKT_RICCATI_GROUP and s.kkt_solver_for(2560) == m.KKT_RICCATI_GROUP
    assert s.kkt_solver_for(1) == m.KKT_RICCATI_GROUP and s.kkt_solver_for(65536) == m.KKT_RICCATI
    s = m.Solver(model_json(N=30, name="gn"), hessian=m.HESSIAN_GAUSS_NEWTON)   # Gauss-Newton: condensed small B
    assert s.kkt_solver_for(2560) == m.KKT_CONDENSED and s.kkt_solver_for(1) == m.KKT_CONDENSED
    assert s.kkt_solver_for(4096) == m.KKT_RICCATI_GROUP
    s = m.Solver(model_json(N=60))                              # N*nu > 64
    assert s.kkt_solver_for(64) == m.KKT_RICCATI_GROUP and s.kkt_solver_for(16384) == m.KKT_RICCATI_GROUP
    assert s.kkt_solver_for(16667) == m.KKT_RICCATI
    assert m.Solver(model_json(N=30), factor_fp32=1).kkt_solver_for(4096) == m.KKT_RICCATI
    p = m.write_model_json(str(tmp_path / "exo.json"), "exo", 8, 4, 2000, 50, model="exo_arm")
    assert m.Solver(p).kkt_solver_for(65536) == m.KKT_RICCATI and m.Solver(p).kkt_solver_for(64) == m.KKT_RICCATI
    p = m.write_model_json(str(tmp_path / "exo20.json"), "exo20", 8, 4, 2000, 20, model="exo_arm")
    assert m.Solver(p).kkt_solver_for(4096) == m.KKT_RICCATI_GROUP and m.Solver(p).kkt_solver_for(8192) == m.KKT_RICCATI
    for k in (m.KKT_CONDENSED, m.KKT_RICCATI, m.KKT_RICCATI_GROUP):
        assert m.Solver(model_json(N=30), kkt_solver=k).kkt_solver_for(4096) == k


def test_hessian_policy(tmp_path, model_json, mmpc_mod):
    """mmpc_opts.hessian (include/mmpc.h) resolved without a GPU: AUTO = exact for unbounded nonlinear 2-link solves
    on the group kernel, Gauss-Newton for control-bounded (faster there) / state-bounded / linear /
    exo / lane-kernel solves; EXACT with control bounds is supported on the group kernel (the held controls fixed in
    the exact QP); EXACT on the lane kernel (round 4; with control bounds since round 5; the exo too); EXACT where
    unsupported (state bounds, the fp32 factor, linear mode) is an API error."""
    m = mmpc_mod
    s = m.Solver(model_json(N=30))
    assert s.hessian_for(4096) == m.HESSIAN_EXACT and s.hessian_for(64) == m.HESSIAN_EXACT
    assert s.hessian_for(4096, u_bounded=True) == m.HESSIAN_GAUSS_NEWTON
    assert s.hessian_for(65536) == m.HESSIAN_GAUSS_NEWTON                 # lane kernel
    s.set_state_bounds([-np.inf, -np.inf, -1.5, -1.5], [np.inf, np.inf, 1.5, 1.5])
    assert s.hessian_for(4096) == m.HESSIAN_GAUSS_NEWTON                  # state bounds: interior point, GN
    s.set_state_bounds(None, None)
    assert m.Solver(model_json(N=30, name="lin", is_linear=True)).hessian_for(64) == m.HESSIAN_GAUSS_NEWTON
    assert m.Solver(model_json(N=30, name="gn"), hessian=m.HESSIAN_GAUSS_NEWTON).hessian_for(4096) == 1
    p = m.write_model_json(str(tmp_path / "exo20.json"), "exo20", 8, 4, 2000, 20, model="exo_arm")
    assert m.Solver(p).hessian_for(4096) == m.HESSIAN_GAUSS_NEWTON     # exo AUTO: Gauss-Newton
    assert m.Solver(p, hessian=m.HESSIAN_EXACT).hessian_for(4096) == m.HESSIAN_EXACT
    p50 = m.write_model_json(str(tmp_path / "exo50.json"), "exo50", 8, 4, 2000, 50, model="exo_arm")
    assert m.Solver(p50, hessian=m.HESSIAN_EXACT).hessian_for(65536) == m.HESSIAN_EXACT    # lane kernel
    # lane kernel with control bounds: honoured since round 5 (held controls fixed in the exact stage QPs)
    assert m.Solver(p50, hessian=m.HESSIAN_EXACT).hessian_for(65536, u_bounded=True) == m.HESSIAN_EXACT
    with pytest.raises(m.MmpcError) as ei:                                # lane kernel, fp32 factor
        m.Solver(p50, hessian=m.HESSIAN_EXACT, factor_fp32=1).hessian_for(65536)
    assert ei.value.code == -4
    with pytest.raises(m.MmpcError):                                      # linear mode
        m.Solver(model_json(N=30, name="lin2", is_linear=True), hessian=m.HESSIAN_EXACT).hessian_for(64)
    with pytest.raises(m.MmpcError):
        m.Solver(model_json(N=30, name="bad"), hessian=7)
    s = m.Solver(model_json(N=30, name="ex"), hessian=m.HESSIAN_EXACT)
    assert s.hessian_for(4096) == m.HESSIAN_EXACT and s.hessian_for(4096, u_bounded=True) == m.HESSIAN_EXACT
    s.set_state_bounds([-1.0] * 4, [1.0] * 4)   # round 6: EXACT honoured under state bounds (interior point)
    assert s.hessian_for(4096) == m.HESSIAN_EXACT


def test_invalid_opts_rejected(model_json, mmpc_mod):
    with pytest.raises(mmpc_mod.MmpcError):
        mmpc_mod.Solver(model_json(), tol_grad=0.0)
    with pytest.raises(mmpc_mod.MmpcError):
        mmpc_mod.Solver(model_json(), max_iter=-1)


def test_null_and_negative_args(model_json, mmpc_mod):
    L = mmpc_mod.lib()
    s = mmpc_mod.Solver(model_json())
    # B < 0 and null pointers are rejected before any device work
    assert L.mmpc_solve_batch(s._h, -1, None, None, None, None, 0, None, None, None, None, None, None, None) == -1
    assert L.mmpc_solve_batch(s._h, 4, None, None, None, None, 0, None, None, None, None, None, None, None) == -1
    # B == 0 is a no-op success (empty batch)
    assert L.mmpc_solve_batch(s._h, 0, None, None, None, None, 0, None, None, None, None, None, None, None) == 0
    assert L.mmpc_destroy(None) == 0


def test_status_strings(mmpc_mod):
    L = mmpc_mod.lib()
    for k, v in mmpc_mod.STATUS.items():
        assert L.mmpc_status_string(k).decode() == v
    assert L.mmpc_status_string(99).decode() == "unknown"


def test_flop_model(mmpc_mod):
    # SURVEY.md 8(d) quotes 288,080 flop/iter for cfg#2 and 96,053 for cfg#1
    assert abs(mmpc_mod.survey_flops_per_iteration(30) - 288080) <= 1
    f = mmpc_mod.flops_per_iteration(30)
    assert f["total"] > 0 and f["gauss_jordan"] > f["hessian"] / 4
    # cfg#3: 9,276,266 flop/iter condensed vs the Riccati recursion of the exo path
    assert abs(mmpc_mod.survey_flops_per_iteration(50, 8, 4) - 9276266) <= 1
    r = mmpc_mod.riccati_flops_per_iteration(50, 8, 4)
    assert 0 < r["total"] < 9276266 / 30


def test_shard_partition_matches_multiprocess_split(mmpc_mod):
    """mmpc_shard (the multi-device C-ABI's partition) = mmpc/dist.py shard_strong for every (B, n, i), covers
    [0, B) exactly once in order, ragged B included; invalid arguments are API errors (no device needed)."""
    import mmpc.dist as mdist
    for B in (0, 1, 5, 37, 4096, 65537):
        for n in (1, 2, 3, 7, 8):
            nxt = 0
            for i in range(n):
                f, c = mmpc_mod.shard(B, n, i)
                assert (f, c) == mdist.shard_strong(B, i, n)
                assert f == nxt and c >= 0
                nxt = f + c
            assert nxt == B
    for bad in ((-1, 2, 0), (10, 0, 0), (10, 2, 2), (10, 2, -1)):
        with pytest.raises(mmpc_mod.MmpcError):
            mmpc_mod.shard(*bad)


def test_rccl_is_loadable_for_the_multi_device_path(mmpc_mod):
    """mmpc_multi_solve_batch_rccl loads librccl with dlopen (no link-time dependency): the version it would use"""
    v = mmpc_mod.rccl_version()
    if not os.path.exists("/opt/rocm/lib/librccl.so.1"):
        pytest.skip("no librccl in this image")
    assert v >= 21000, v


def test_reserve_workspace_bytes_include_the_tail_hand_over(tmp_path, mmpc_mod):
    """mmpc_reserve_workspace reports its size before touching a device: the solver workspace, the iteration-tail
    hand-over list and a state-bounded solve's resume workspace (sized for 256 CUs until a device was
    queried) -- the latter whether or not the handle has state bounds yet, so that setting them after the reservation
    never grows the workspace inside a solve (a hipFree under a captured graph)"""
    p = mmpc_mod.write_model_json(str(tmp_path / "exo.json"), "exo", 8, 4, 2000, 50, model="exo_arm")
    s = mmpc_mod.Solver(p)
    b = C.c_uint64(0)
    s._L.mmpc_reserve_workspace(s._h, 65536, C.byref(b))   # no GPU here: an error code, the size set before it
    plain = b.value
    lane_ws = 65536 * 8 * (51 + 1) * (5 * 8 + 2 * 4 + 4 * 13 + 5 * 12)   # lane_ws_doubles(8, 4, 4, 50, xb) x B x 8 B
    assert plain > lane_ws + 256 + 65536 * 24
    s.set_state_bounds([-np.inf] * 4 + [-1.5] * 4, [np.inf] * 4 + [1.5] * 4)
    s._L.mmpc_reserve_workspace(s._h, 65536, C.byref(b))
    assert b.value == plain
    s.set_state_bounds(None, None)
    s._L.mmpc_reserve_workspace(s._h, 65536, C.byref(b))
    assert b.value == plain
